// robot_ekf.hpp — C++ host side of the drop-in for HuaiLeiTang/slam_ros `class Robot`
// (slam_ros/Robot.h:21-77), layered over the C-ABI of libslam_ekf.so (include/slam_ekf.h).
//
// BasicRobot<Line, IntervalMsg, N> keeps the reference's public surface — the constructor
// Robot(x, y, theta) (Robot.cpp:20-35), localize(lines, rot, encoder) (Robot.h:74,
// Robot.cpp:126-904), getEllipse(axii, angle) (Robot.h:73, Robot.cpp:73-124), the public
// xPos / yPos / thetaPos (Robot.h:54-56), lineIntervals (Robot.h:59) and P_t0 (Robot.h:62) —
// and adds the two halves predict(encoder) / update(lines). The EKF state lives
// on the GPU; P_t0 keeps the reference's type (double[SLAMSIZE*SLAMSIZE], Robot.h:62) as a host
// mirror. Mirror policy (setMirror): kFull (default) refreshes all of P_t0 after every call, as
// the reference's member always holds the full P; kPoseBlock refreshes only [0:3, 0:3] (what
// getEllipse reads, Robot.cpp:75-77) and leaves the rest as of the last downloadP() — for large
// capacities, where the full download costs O(n²) per scan. The per-call cost of kFull: a drain
// of the deferred flush (so the flush interval has no effect), an unpack into the context's
// persistent n × n device scratch and an n² × 8-byte device-to-host copy.
//
// The types are template parameters so that the core compiles without ROS or GSL:
//   Line         needs .alfa, .r, .C_AR (pointer to a 2x2 matrix with .data and .tda, the
//                fields of gsl_matrix; simplifyPath.h:62-79) and .lineInterval (a sequence
//                of points with .alfa and .r);
//   IntervalMsg  needs .data, a std::vector<float> (std_msgs::Float32MultiArray).
// slam_ros_amd/host/Robot.h instantiates it with the reference's `line` and
// std_msgs::Float32MultiArray for the catkin package.
//
// Errors follow the reference (Robot.cpp:128, 909-917): localize never throws and always leaves
// a committed state; numeric conditions are printed. A missing GPU / library is not a numeric
// condition: the constructor throws (no CPU fallback exists).
#pragma once

#include <cmath>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

#include "slam_ekf.h"

namespace slam_ekf {

// Robot::normalizeRadian (Robot.cpp:62-71), including its non-standard fold for |rad| >= 2π
inline void normalize_radian(double& rad)
{
    if (rad > M_PI)
        rad -= 2 * M_PI + std::floor(rad / (2 * M_PI)) * 2 * M_PI;
    else if (rad < -M_PI)
        rad += 2 * M_PI + std::floor(std::fabs(rad) / (2 * M_PI)) * 2 * M_PI;
}

template <class Line, class IntervalMsg, int N = 100>
class BasicRobot {
public:
    static constexpr int kLines = N;            // LINESIZE (Robot.h:13)
    static constexpr int kState = 2 * N + 3;    // SLAMSIZE (Robot.h:14)

    enum Mirror { kPoseBlock = 0, kFull = 1 };

    double xPos = 0, yPos = 0, thetaPos = 0;    // Robot.h:54-56
    IntervalMsg lineIntervals;                  // Robot.h:59
    double P_t0[kState * kState] = {};          // Robot.h:62 (host mirror, row-major; see Mirror)

    // Robot::Robot(x, y, theta), Robot.cpp:20-35
    BasicRobot(double x, double y, double theta, int precision = EKF_PREC_F64, int device = -1)
    {
        ekf_config cfg;
        ekf_config_init(&cfg);
        cfg.capacity = N;
        cfg.instances = 1;
        cfg.precision = precision;
        precision_ = precision;
        cfg.device = device;
        cfg.max_lines = EKF_MAX_LINES;
        int rc = ekf_create(&cfg, &ctx_);
        if (rc != EKF_OK) throw std::runtime_error(std::string("slam_ekf: ekf_create: ") + ekf_strerror(rc));
        rc = ekf_reset_instance(ctx_, 0, x, y, theta);
        if (rc != EKF_OK) {
            ekf_destroy(ctx_);
            throw std::runtime_error(std::string("slam_ekf: reset: ") + ekf_strerror(rc));
        }
        xPos = x;
        yPos = y;
        thetaPos = theta;
        refresh_mirror();
    }
    ~BasicRobot()
    {
        if (ctx_) ekf_destroy(ctx_);
    }
    BasicRobot(const BasicRobot&) = delete;
    BasicRobot& operator=(const BasicRobot&) = delete;

    // Robot::localize (Robot.h:74). SIMULATIONOFF (Robot.h:18) is true in the reference: the
    // motion input is the absolute encoder pose and `rot` is never used (Robot.cpp:130-148).
    void localize(const std::vector<Line>& lines, float* rot = nullptr, const double* encoder = nullptr)
    {
        (void)rot;
        if (!encoder) {
            std::fprintf(stderr, "Robot::localize: encoder pose required (SIMULATIONOFF)\n");
            return;
        }
        std::vector<ekf_line> buf;
        if (!pack(lines, buf)) return;
        const int32_t nl = (int32_t)lines.size();
        ekf_result res{};
        if (report(ekf_localize(ctx_, encoder, buf.data(), &nl, &res), "ekf_localize")) finish(lines, res);
    }

    // predict half: motion model and P_pre (Robot.cpp:130-286)
    void predict(const double* encoder, const float* rot = nullptr)
    {
        (void)rot;
        if (!encoder) return;
        report(ekf_predict(ctx_, encoder), "ekf_predict");
    }

    // update half: association, Kalman updates, augmentation, reset (Robot.cpp:288-904)
    void update(const std::vector<Line>& lines)
    {
        std::vector<ekf_line> buf;
        if (!pack(lines, buf)) return;
        const int32_t nl = (int32_t)lines.size();
        ekf_result res{};
        if (report(ekf_update(ctx_, buf.data(), &nl, &res), "ekf_update")) finish(lines, res);
    }

    // Robot::getEllipse (Robot.h:73, Robot.cpp:73-124)
    bool getEllipse(float axii[2], float& angle)
    {
        return ekf_get_ellipse(ctx_, 0, axii, &angle) == 1;
    }

    void normalizeRadian(double& rad) { normalize_radian(rad); }

    void setMirror(Mirror m)
    {
        mirror_ = m;
        refresh_mirror();
    }
    Mirror mirror() const { return mirror_; }

    // full covariance into P_t0 (and optionally the state vector)
    bool downloadP(std::vector<double>* y = nullptr, int* saved = nullptr)
    {
        std::vector<double> yy((size_t)kState);
        int s = 0;
        double pose[3];
        const int rc = ekf_download_state(ctx_, 0, P_t0, yy.data(), &s, pose);
        if (rc != EKF_OK) return false;
        if (y) *y = yy;
        if (saved) *saved = s;
        return true;
    }

    int matchesNum() const { return last_.matches; }
    const ekf_result& lastResult() const { return last_; }
    ekf_ctx* context() { return ctx_; }

private:
    ekf_ctx* ctx_ = nullptr;
    int precision_ = EKF_PREC_F64;
    ekf_result last_{};
    Mirror mirror_ = kFull;

    static bool report(int rc, const char* what)
    {
        if (rc != EKF_OK) std::fprintf(stderr, "slam_ekf: %s: %s\n", what, ekf_strerror(rc));
        return rc == EKF_OK;
    }

    // the context reads max_lines (= EKF_MAX_LINES) entries per instance: the buffer always
    // holds that many, zero past the scan's lines
    static bool pack(const std::vector<Line>& lines, std::vector<ekf_line>& out)
    {
        if ((int)lines.size() > EKF_MAX_LINES) {
            std::fprintf(stderr, "slam_ekf: %zu lines exceed EKF_MAX_LINES\n", lines.size());
            return false;
        }
        out.assign((size_t)EKF_MAX_LINES, ekf_line{});
        for (size_t i = 0; i < lines.size(); i++) {
            ekf_line& o = out[i];
            o.alpha = lines[i].alfa;
            o.r = lines[i].r;
            const auto* C = lines[i].C_AR;   // 2x2 gsl_matrix (lineFitting.cpp:379-450)
            for (int a = 0; a < 2; a++)
                for (int b = 0; b < 2; b++) o.R[a * 2 + b] = C ? C->data[a * C->tda + b] : 0.0;
        }
        return true;
    }

    void finish(const std::vector<Line>& lines, const ekf_result& res)
    {
        last_ = res;
        if (res.status & EKF_ST_SINGULAR_S)
            std::fprintf(stderr, "slam_ekf: singular innovation covariance (GSL_EDOM)\n");
        if (res.status & EKF_ST_CAPACITY)
            std::fprintf(stderr, "slam_ekf: landmark capacity exceeded\n");
        if (res.status & EKF_ST_SYNC_TIMEOUT)
            std::fprintf(stderr, "slam_ekf: association exchange timed out\n");
        if ((res.status & EKF_ST_RANGE) && precision_ == EKF_PREC_F16)   // near fp16's range: re-choose the exponent
            report(ekf_rescale(ctx_, 0, EKF_EXP_AUTO), "ekf_rescale");
        else if (res.status & EKF_ST_RANGE)
            std::fprintf(stderr, "slam_ekf: landmark variance near the storage range (diverged filter)\n");
        // (EKF_ST_PRECISION is informational: the update still committed)
        xPos = res.pose[0];
        yPos = res.pose[1];
        thetaPos = res.pose[2];
        // STORING LINE INTERVALS (Robot.cpp:869-879): world-frame endpoints of every line added
        // as a landmark, in extraLines order, with the pose after the update; the reference
        // narrows the endpoint angle to float before use
        for (int i = 0; i < res.nlines && i < (int)lines.size(); i++) {
            if (res.match[i] >= 0) continue;
            const auto& iv = lines[i].lineInterval;
            if (iv.size() != 2) continue;
            push_endpoint(iv.front().alfa, iv.front().r);
            push_endpoint(iv.back().alfa, iv.back().r);
        }
        refresh_mirror();
    }

    void push_endpoint(double alfa, double r)
    {
        const float alpha = (float)alfa;
        const double a = alpha + thetaPos;
        const double rr = r + xPos * std::cos(alpha) + yPos * std::sin(alpha);
        lineIntervals.data.push_back((float)(std::cos(a) * rr));   // polar2descart, lineFitting.cpp:170-176
        lineIntervals.data.push_back((float)(std::sin(a) * rr));
    }

    void refresh_mirror()
    {
        if (mirror_ == kFull) {
            int s = 0;
            double pose[3];
            if (ekf_download_state(ctx_, 0, P_t0, nullptr, &s, pose) == EKF_OK) return;
        }
        double P33[9];
        if (ekf_get_pose_cov(ctx_, 0, P33) != EKF_OK) return;
        for (int a = 0; a < 3; a++)
            for (int b = 0; b < 3; b++) P_t0[(size_t)a * kState + b] = P33[a * 3 + b];
    }
};

}  // namespace slam_ekf
