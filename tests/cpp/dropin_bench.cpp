// Per-call cost of the C++ drop-in (slam_ros_amd/host/robot_ekf.hpp) on the path slam_ros/main.cpp
// actually calls (main.cpp:139-174): one Robot at the reference's capacity (LINESIZE 100,
// Robot.h:13-14), fp64, synchronous Robot::localize per scan, with the P_t0 mirror refreshed
// after every call (kFull, the default: the reference's member always holds the full P) or only
// its pose block (kPoseBlock). Timing harness, not a test: DESIGN §5 / profiles/r06_dropin.
//
// usage: dropin_bench <scenario.txt> <state.bin> <warmup> <timed>
//   scenario.txt: the dropin_driver format (nscans, then per scan "ex ey eth L" and L rows
//   "alfa r R00 R01 R10 R11 a0 r0 a1 r1"); state.bin: n*n P, n y, then saved and the pose
//   (doubles) of the map the scans observe, uploaded after the constructor.
// stdout: one JSON object: µs per call (median, mean, p90) for each mirror policy, and the
//   parts — ekf_localize alone, ekf_get_pose_cov, ekf_download_state of the full P.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <stdexcept>
#include <vector>

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

struct Scan {
    double enc[3];
    std::vector<Mat2> covs;
    std::vector<line> lines;
};

static double now_us()
{
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static void stats(const char* name, std::vector<double> v, bool last)
{
    std::sort(v.begin(), v.end());
    double sum = 0;
    for (double x : v) sum += x;
    std::printf("  \"%s\": {\"median_us\": %.3f, \"mean_us\": %.3f, \"p90_us\": %.3f, \"min_us\": %.3f, \"calls\": %zu}%s\n",
                name, v[v.size() / 2], sum / v.size(), v[(v.size() * 9) / 10], v[0], v.size(), last ? "" : ",");
}

int main(int argc, char** argv)
{
    if (argc < 5) return 2;
    const int warm = std::atoi(argv[3]), timed = std::atoi(argv[4]);
    FILE* f = std::fopen(argv[1], "r");
    if (!f) return 2;
    int nscans = 0;
    if (std::fscanf(f, "%d", &nscans) != 1) return 2;
    std::vector<Scan> scans((size_t)nscans);
    for (auto& sc : scans) {
        int L = 0;
        if (std::fscanf(f, "%lf %lf %lf %d", &sc.enc[0], &sc.enc[1], &sc.enc[2], &L) != 4) return 2;
        sc.covs.resize((size_t)std::max(L, 1));
        sc.lines.resize((size_t)L);
        for (int i = 0; i < L; i++) {
            line& l = sc.lines[i];
            double a0, r0, a1, r1;
            Mat2& c = sc.covs[i];
            if (std::fscanf(f, "%lf %lf %lf %lf %lf %lf %lf %lf %lf %lf", &l.alfa, &l.r, &c.data[0], &c.data[1],
                            &c.data[2], &c.data[3], &a0, &r0, &a1, &r1) != 10)
                return 2;
            l.lineInterval = {polar_point(a0, r0), polar_point(a1, r1)};
        }
        for (int i = 0; i < L; i++) sc.lines[i].C_AR = &sc.covs[i];
    }
    std::fclose(f);
    const int n = Rover::kState;
    std::vector<double> P((size_t)n * n), y((size_t)n), tail(4);
    FILE* b = std::fopen(argv[2], "rb");
    if (!b || std::fread(P.data(), sizeof(double), P.size(), b) != P.size() ||
        std::fread(y.data(), sizeof(double), y.size(), b) != y.size() || std::fread(tail.data(), sizeof(double), 4, b) != 4)
        return 2;
    std::fclose(b);
    if (warm + timed > nscans) return 2;
    try {
        std::printf("{\n");
        for (int pass = 0; pass < 2; pass++) {
            const bool full = pass == 0;
            Rover* rp = new Rover(0, 0, 0);   // main.cpp:98 (P_t0 is a 330 KB member: heap)
            Rover& rover = *rp;
            rover.setMirror(full ? Rover::kFull : Rover::kPoseBlock);
            if (ekf_upload_state(rover.context(), 0, P.data(), y.data(), (int)tail[0], &tail[1]) != EKF_OK) return 3;
            std::vector<double> t;
            int matches = 0;
            for (int k = 0; k < warm + timed; k++) {
                const double t0 = now_us();
                rover.localize(scans[k].lines, nullptr, scans[k].enc);
                const double t1 = now_us();
                if (k >= warm) {
                    t.push_back(t1 - t0);
                    matches += rover.matchesNum();
                }
                rover.lineIntervals.data.clear();   // main.cpp:174
            }
            stats(full ? "localize_mirror_full" : "localize_mirror_pose_block", t, false);
            std::printf("  \"%s_matches_per_call\": %.3f,\n", full ? "full" : "pose_block", (double)matches / timed);
            if (!full) {
                // the parts, on the same context and scans (the state keeps evolving: the same workload)
                std::vector<double> tl, tp, td;
                ekf_ctx* c = rover.context();
                std::vector<ekf_line> buf((size_t)EKF_MAX_LINES);
                std::vector<double> Pd((size_t)n * n);
                for (int k = 0; k < timed; k++) {
                    const Scan& sc = scans[warm + k];
                    std::fill(buf.begin(), buf.end(), ekf_line{});
                    for (size_t i = 0; i < sc.lines.size(); i++) {
                        buf[i].alpha = sc.lines[i].alfa;
                        buf[i].r = sc.lines[i].r;
                        for (int q = 0; q < 4; q++) buf[i].R[q] = sc.covs[i].data[q];
                    }
                    const int32_t nl = (int32_t)sc.lines.size();
                    ekf_result res{};
                    const double t0 = now_us();
                    ekf_localize(c, sc.enc, buf.data(), &nl, &res);
                    const double t1 = now_us();
                    double P33[9];
                    ekf_get_pose_cov(c, 0, P33);
                    const double t2 = now_us();
                    int s = 0;
                    double pose[3];
                    ekf_download_state(c, 0, Pd.data(), nullptr, &s, pose);
                    const double t3 = now_us();
                    tl.push_back(t1 - t0);
                    tp.push_back(t2 - t1);
                    td.push_back(t3 - t2);
                }
                stats("part_ekf_localize", tl, false);
                stats("part_ekf_get_pose_cov", tp, false);
                stats("part_ekf_download_state_full_P", td, true);
            }
            delete rp;
        }
        std::printf("}\n");
    } catch (const std::exception& e) {
        std::fprintf(stderr, "%s\n", e.what());
        return 3;
    }
    return 0;
}
