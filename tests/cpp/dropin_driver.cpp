// Drives the C++ drop-in (slam_ros_amd/host/robot_ekf.hpp) the way slam_ros/main.cpp:135-174
// drives Robot: localize(lines, NULL, encoderPose), read xPos/yPos/thetaPos, getEllipse,
// publish and clear lineIntervals. The `line` / message types here are test doubles with the
// fields the drop-in reads (simplifyPath.h:62-79, std_msgs::Float32MultiArray::data).
//
// Built two ways: with the test doubles below against robot_ekf.hpp, or (-DUSE_ROBOT_H) against
// the catkin drop-in header slam_ros_amd/host/Robot.h itself, with stub std_msgs / lineFitting.h
// / simplifyPath.h / gsl_matrix.h headers (tests/cpp/stubs) standing in for ROS and GSL.
//
// usage: dropin_driver <scenario.txt> <out_P.bin>
//   scenario: nscans, then per scan "ex ey eth L" and L rows
//   "alfa r R00 R01 R10 R11 a0 r0 a1 r1" (lineInterval endpoints, robot frame).
// stdout: per scan "scan k x y theta matches nint ellipse_ok ax0 ax1 angle" + "match ..." +
//   "ints ..." (the lineIntervals floats published that cycle); exit 3 if the GPU path fails.
#include <cstdio>
#include <stdexcept>
#include <vector>

#ifdef USE_ROBOT_H
#include "Robot.h"

struct Mat2 {
    double data[4] = {0, 0, 0, 0};
    gsl_matrix m{2, 2, 2, nullptr, nullptr, 0};
};
typedef Robot Rover;
static gsl_matrix* as_cov(Mat2& c)
{
    c.m.data = c.data;
    return &c.m;
}
#else
#include "robot_ekf.hpp"

struct Mat2 {
    size_t size1 = 2, size2 = 2, tda = 2;
    double data[4] = {0, 0, 0, 0};
};
struct polar_point {
    polar_point(double a = 0, double rr = 0) : alfa(a), r(rr) {}
    double alfa, r;
};
struct line {
    double alfa = 0, r = 0;
    Mat2* C_AR = nullptr;
    std::vector<polar_point> lineInterval;
};
struct Float32MultiArray {
    std::vector<float> data;
};
typedef slam_ekf::BasicRobot<line, Float32MultiArray, 100> Rover;
static Mat2* as_cov(Mat2& c) { return &c; }
#endif

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    FILE* f = std::fopen(argv[1], "r");
    if (!f) return 2;
    int nscans = 0;
    if (std::fscanf(f, "%d", &nscans) != 1) return 2;
    try {
        // main.cpp:98 allocates the robot on the heap (P_t0 is a 330 KB member)
        Rover* rp = new Rover(0, 0, 0);
        Rover& rover = *rp;
        for (int k = 0; k < nscans; k++) {
            double enc[3];
            int L = 0;
            if (std::fscanf(f, "%lf %lf %lf %d", &enc[0], &enc[1], &enc[2], &L) != 4) return 2;
            std::vector<Mat2> covs((size_t)L > 0 ? (size_t)L : 1);
            std::vector<line> lines((size_t)L);
            for (int i = 0; i < L; i++) {
                line& l = lines[i];
                double a0, r0, a1, r1;
                if (std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf %lf", &l.alfa, &l.r,
                                &covs[i].data[0], &covs[i].data[1], &covs[i].data[2], &covs[i].data[3],
                                &a0, &r0, &a1, &r1) != 10)
                    return 2;
                l.C_AR = as_cov(covs[i]);
                l.lineInterval = {polar_point(a0, r0), polar_point(a1, r1)};
            }
            rover.localize(lines, nullptr, enc);
            float axii[2] = {0, 0}, angle = 0;
            const bool ok = rover.getEllipse(axii, angle);
            std::printf("scan %d %.17g %.17g %.17g %d %zu %d %.9g %.9g %.9g\n", k, rover.xPos,
                        rover.yPos, rover.thetaPos, rover.matchesNum(),
                        rover.lineIntervals.data.size(), ok ? 1 : 0, axii[0], axii[1], angle);
            std::printf("match");
            for (int i = 0; i < L; i++) std::printf(" %d", rover.lastResult().match[i]);
            std::printf("\nints");
            for (float v : rover.lineIntervals.data) std::printf(" %.9g", v);
            std::printf("\n");
            rover.lineIntervals.data.clear();
        }
        // the mirror (default policy kFull) already holds the full P after the last localize
        FILE* o = std::fopen(argv[2], "wb");
        if (!o) return 2;
        std::fwrite(rover.P_t0, sizeof(double), sizeof(rover.P_t0) / sizeof(double), o);
        std::fclose(o);
        delete rp;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    }
    return 0;
}
