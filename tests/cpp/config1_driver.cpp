// Config 1 end to end on the host side of the path: a 360-beam scan of a room is
// ray-cast from the true pose, lines are extracted (slam_ros_amd/host/line_extraction.hpp, the
// restatement of lineFitting.cpp / simplifyPath.cpp / main.cpp:37-61) and, in `slam` mode, fed to
// the drop-in Robot (robot_ekf.hpp over libslam_ekf.so) the way main.cpp:135-152 does.
//
// usage: config1_driver extract|slam <scenario.txt>
//   scenario: "xmin ymin xmax ymax npillars" + npillars × "cx cy", then "nposes" + nposes × "x y θ"
//   (true poses; the encoder reports them, as realRoboPose does in simulation, main.cpp:84-89)
// stdout per pose: "pose k L" then L × "line alfa r C00 C01 C10 C11 a0 r0 a1 r1" (robot frame,
//   interval end points as SetEndPoints leaves them); slam mode adds
//   "est k x y theta matches", "match j0 j1 …" and the cycle's published messages (ros_output.hpp):
//   "pub ok tx ty tz rx ry rz rw nfloats floats…". Exit 3 if the GPU path fails.
#include <cstdio>
#include <cstring>
#include <stdexcept>
#include <vector>

#include "line_extraction.hpp"
#include "robot_ekf.hpp"
#include "ros_output.hpp"

namespace lx = slam_ekf::lx;

struct Mat2 {
    size_t size1 = 2, size2 = 2, tda = 2;
    double data[4] = {0, 0, 0, 0};
};
struct line {
    double alfa = 0, r = 0;
    Mat2* C_AR = nullptr;
    std::vector<lx::PolarPoint> lineInterval;
};
struct Float32MultiArray {
    std::vector<float> data;
};

int main(int argc, char** argv)
{
    if (argc < 3) return 2;
    const bool slam = std::strcmp(argv[1], "slam") == 0;
    FILE* f = std::fopen(argv[2], "r");
    if (!f) return 2;
    double xmin, ymin, xmax, ymax;
    int np = 0;
    if (std::fscanf(f, "%lf %lf %lf %lf %d", &xmin, &ymin, &xmax, &ymax, &np) != 5) return 2;
    std::vector<lx::XY> pillars((size_t)np);
    for (int k = 0; k < np; k++)
        if (std::fscanf(f, "%lf %lf", &pillars[k].x, &pillars[k].y) != 2) return 2;
    int nposes = 0;
    if (std::fscanf(f, "%d", &nposes) != 1) return 2;
    std::vector<double> poses(3 * (size_t)nposes);
    for (int k = 0; k < nposes; k++)
        if (std::fscanf(f, "%lf %lf %lf", &poses[3 * k], &poses[3 * k + 1], &poses[3 * k + 2]) != 3) return 2;
    std::fclose(f);
    const lx::Room room = lx::make_room(xmin, ymin, xmax, ymax, pillars);
    try {
        slam_ekf::BasicRobot<line, Float32MultiArray, 64>* rover = nullptr;
        if (slam) rover = new slam_ekf::BasicRobot<line, Float32MultiArray, 64>(0, 0, 0);   // main.cpp:98
        for (int k = 0; k < nposes; k++) {
            const double* pose = &poses[3 * k];
            const std::vector<float> msg = lx::raycast_room(room, pose);
            const std::vector<lx::Line> ext = lx::lines_from_scan(msg);
            std::printf("pose %d %zu\n", k, ext.size());
            std::vector<Mat2> covs(ext.size());
            std::vector<line> lines(ext.size());
            for (size_t i = 0; i < ext.size(); i++) {
                const lx::Line& l = ext[i];
                std::printf("line %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g %.17g\n", l.alfa, l.r,
                            l.C[0], l.C[1], l.C[2], l.C[3], l.interval[0].alfa, l.interval[0].r,
                            l.interval[1].alfa, l.interval[1].r);
                for (int c = 0; c < 4; c++) covs[i].data[c] = l.C[c];
                lines[i].alfa = l.alfa;
                lines[i].r = l.r;
                lines[i].C_AR = &covs[i];
                lines[i].lineInterval = l.interval;
            }
            if (rover) {
                rover->localize(lines, nullptr, pose);   // main.cpp:144
                std::printf("est %d %.17g %.17g %.17g %d\nmatch", k, rover->xPos, rover->yPos, rover->thetaPos,
                            rover->matchesNum());
                for (size_t i = 0; i < lines.size(); i++) std::printf(" %d", rover->lastResult().match[i]);
                std::printf("\n");
                slam_ekf::TransformMsg msg;                 // main.cpp:150-174
                std::vector<float> pub_lines;
                const bool ok = slam_ekf::publish_cycle(*rover, msg, pub_lines);
                std::printf("pub %d %.17g %.17g %.17g %.9g %.9g %.9g %.9g %zu", ok ? 1 : 0, msg.translation.x,
                            msg.translation.y, msg.translation.z, msg.rotation.x, msg.rotation.y, msg.rotation.z,
                            msg.rotation.w, pub_lines.size());
                for (float v : pub_lines) std::printf(" %.9g", v);
                std::printf("\n");
            }
        }
        delete rover;
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    }
    return 0;
}
