// line_extraction.hpp — the caller side of the EKF update: laser scan →
// observed lines {alpha, r, C_AR}, as slam_ros/main.cpp:37-61 and lineFitting.cpp /
// simplifyPath.cpp / vec2.cpp produce them, without GSL or ROS. Host code, C++11, header-only.
//
//   scan_to_points  main.cpp:37-56       ranges > 0.05, alfa = θ − π, variance 0.01 (no noise:
//                                        SIMULATIONOFF, Robot.h:18)
//   extract_lines   lineFitting.cpp:650-702 (LineExtraction): sort by angle, split where
//                   consecutive points are > 0.5 apart (:548-589), rotate so that the last split
//                   starts the sequence, split again, then per segment the recursive
//                   split-and-fit (simplifyPath.cpp:108-177), then LineConversion (:608-649)
//   to_robot_frame  main.cpp:57-61       alfa += π, folded into (−π, π]
//   raycast_room    config 1 input: a 360-beam scan of a rectangular room with
//                   square pillars, message layout [r0, θ0, r1, θ1, …] (main.cpp:41-56)
//
// The reference's constants and quirks are kept where they change numbers: π is 3.14159265 in
// the line code (lineFitting.h:8) and M_PI in main.cpp; a fitted line passes through degrees and
// back (lineFitting.cpp:17-23, :280); the angle part of the line covariance is 1/12·1.5 == 0
// (integer division, :419) and the off-diagonals are forced to 0 (:446-448); the residual sum
// starts at 0 (its accumulator is uninitialised in the reference, :108). The pairwise sums of
// the fit keep the reference's O(n²) order of summation.
#pragma once

#include <algorithm>
#include <cmath>
#include <cstddef>
#include <utility>
#include <vector>

#include "slam_ekf.h"

namespace slam_ekf {
namespace lx {

constexpr double kPi = 3.14159265;   // lineFitting.h:8

struct PolarPoint {                  // simplifyPath.h:49-60 (polar_point)
    double alfa = 0.0, r = 0.0;
    double weight = 1.0, variance = 1.0;
};

struct XY {                          // simplifyPath.h:27-46 (Point) and vec2.h (Vec2)
    double x, y;
};

struct Line {                        // simplifyPath.h:62-79 (line)
    double alfa = 0.0, r = 0.0;      // normal angle (rad) and distance
    double b = 0.0, m = 0.0;         // y = b + m·x, set by the constructor
    double C[4] = {0.0, 0.0, 0.0, 0.0};   // C_AR, row-major 2×2
    std::vector<PolarPoint> interval;     // end points (lineInterval)
};

inline XY to_xy(const PolarPoint& p) { return XY{std::cos(p.alfa) * p.r, std::sin(p.alfa) * p.r}; }

inline PolarPoint to_polar(const XY& v)
{
    PolarPoint p;
    p.r = std::sqrt(v.x * v.x + v.y * v.y);
    p.alfa = std::atan2(v.y, v.x);
    return p;
}

// line(alfa_deg, r) (lineFitting.cpp:17-23)
inline Line make_line_deg(double alfa_deg, double r)
{
    Line l;
    l.alfa = alfa_deg * (kPi / 180);
    l.r = r;
    l.b = l.r / std::sin(l.alfa);
    l.m = -1 / std::tan(l.alfa);
    return l;
}

// Weighted total-least-squares line in polar form (lineFitting.cpp:240-282)
inline Line fit_line(const std::vector<PolarPoint>& P)
{
    const size_t n = P.size();
    double wi = 0.0;
    for (size_t i = 0; i < n; i++) wi = wi + P[i].weight;
    double s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0, sr = 0.0;
    for (size_t i = 0; i < n; i++)
        for (size_t j = i + 1; j < n; j++)
            s1 = s1 + P[i].weight * P[j].weight * P[i].r * P[j].r * std::sin(P[i].alfa + P[j].alfa);
    for (size_t i = 0; i < n; i++)
        s2 = s2 + (P[i].weight - wi) * P[i].weight * P[i].r * P[i].r * std::sin(2 * P[i].alfa);
    for (size_t i = 0; i < n; i++)
        for (size_t j = i + 1; j < n; j++)
            s3 = s3 + P[i].weight * P[j].weight * P[i].r * P[j].r * std::cos(P[i].alfa + P[j].alfa);
    for (size_t i = 0; i < n; i++)
        s4 = s4 + (P[i].weight - wi) * P[i].weight * P[i].r * P[i].r * std::cos(2 * P[i].alfa);
    const double alfa = 0.5 * std::atan2((2 / wi) * s1 + (1 / wi) * s2, (2 / wi) * s3 + (1 / wi) * s4);
    for (size_t i = 0; i < n; i++) sr = sr + P[i].weight * P[i].r * std::cos(P[i].alfa - alfa);
    return make_line_deg(alfa * 180 / kPi, sr / wi);
}

// Sum of the points' distances to the chord of the fitted line over the points' x range
// (lineFitting.cpp:96-127)
inline double residual_error(const std::vector<PolarPoint>& P, const Line& l)
{
    if (P.size() < 2) return 0.0;
    std::vector<XY> v(P.size());
    for (size_t i = 0; i < P.size(); i++) v[i] = to_xy(P[i]);
    const XY f{v[0].x, l.b + v[0].x * l.m};
    const XY e{v.back().x, l.b + v.back().x * l.m};
    const XY p{e.x - f.x, e.y - f.y};
    const double pn = std::sqrt(p.x * p.x + p.y * p.y);
    double sum = 0.0;
    for (size_t i = 1; i < v.size(); i++) {
        const XY pp{v[i].x - f.x, v[i].y - f.y};
        sum = sum + std::fabs(pp.x * p.y - p.x * pp.y) / pn;
    }
    return sum;
}

// Index of the point farthest from the chord first–last (simplifyPath.cpp:37-57)
inline size_t farthest_from_chord(const std::vector<XY>& v)
{
    const XY f = v[0], e = v.back();
    const XY p{e.x - f.x, e.y - f.y};
    const double pn = std::sqrt(p.x * p.x + p.y * p.y);
    size_t index = 0;
    double best = -1;
    for (size_t i = 1; i < v.size(); i++) {
        const XY pp{v[i].x - f.x, v[i].y - f.y};
        const double d = std::fabs(pp.x * p.y - p.x * pp.y) / pn;
        if (d > best) {
            best = d;
            index = i;
        }
    }
    return index;
}

// LineAlap / alfanorm (lineFitting.cpp:357-378)
inline void flip_negative(Line& l)
{
    if (l.r < 0) {
        l.r = std::fabs(l.r);
        l.alfa = l.alfa < 0 ? kPi + l.alfa : -kPi + l.alfa;
    }
}

inline double fold_once(double a)
{
    if (a > kPi) return a - 2 * kPi;
    if (a < -kPi) return a + 2 * kPi;
    return a;
}

// C_AR of a fitted line: forward differences (step 1e-6) of (alfa, r) with respect to every
// point's r and alfa, propagated through diag(1.5·variance², 1/12·1.5 == 0); off-diagonals
// zeroed (lineFitting.cpp:379-450). The product keeps GSL dgemm's order over k.
inline void line_covariance(std::vector<PolarPoint> P, double C[4])
{
    const size_t n = P.size();
    Line base = fit_line(P);
    flip_negative(base);
    if (base.alfa < 0) base.alfa = base.alfa + 2 * kPi;
    const double eps = 0.000001;
    std::vector<double> F0(2 * n), F1(2 * n), Cx(2 * n);
    for (int pass = 0; pass < 2; pass++)
        for (size_t i = 0; i < n; i++) {
            double& x = pass == 0 ? P[i].r : P[i].alfa;
            const double keep = x;
            x = x + eps;
            Line l = fit_line(P);
            flip_negative(l);
            const double a = l.alfa < 0 ? l.alfa + 2 * kPi : l.alfa;
            F0[pass * n + i] = fold_once(a - base.alfa) / eps;
            F1[pass * n + i] = (l.r - base.r) / eps;
            x = keep;
        }
    for (size_t i = 0; i < n; i++) {
        Cx[i] = P[i].variance * P[i].variance * 1.5;
        Cx[n + i] = 1 / 12 * 1.5;   // integer division, as written (lineFitting.cpp:419)
    }
    double c00 = 0.0, c11 = 0.0;
    for (size_t k = 0; k < 2 * n; k++) {
        c00 += (F0[k] * Cx[k]) * F0[k];
        c11 += (F1[k] * Cx[k]) * F1[k];
    }
    C[0] = c00;
    C[1] = 0.0;
    C[2] = 0.0;
    C[3] = c11;
}

// The end points of a segment: the first / last point projected on the line through the fitted
// line's points at the middle and at that end (simplifyPath.cpp:59-105)
inline PolarPoint end_on_line(const std::vector<PolarPoint>& P, const Line& l, bool last)
{
    const PolarPoint& at = last ? P.back() : P.front();
    if (P.size() < 4) return at;
    PolarPoint mid, end;
    mid.alfa = P[P.size() / 2].alfa;
    mid.r = l.r / std::cos(mid.alfa - l.alfa);
    end.alfa = at.alfa;
    end.r = l.r / std::cos(at.alfa - l.alfa);
    const XY p = to_xy(at), vm = to_xy(mid), ve = to_xy(end);
    const XY fe{ve.x - vm.x, ve.y - vm.y}, fp{p.x - vm.x, p.y - vm.y};
    auto length = [](const XY& a) {
        const double t = std::pow(a.x, 2) + std::pow(a.y, 2);
        return t > 0 ? std::sqrt(std::pow(a.x, 2) + std::pow(a.y, 2)) : 0.0;
    };
    const double lfe = length(fe), lfp = length(fp);
    const double cosang = (fe.x * fp.x + fe.y * fp.y) / (lfe * lfp);
    const double s = cosang * lfp;
    const XY q{vm.x + (fe.x / lfe) * s, vm.y + (fe.y / lfe) * s};
    return to_polar(q);
}

// line::SetEndPoints (lineFitting.cpp:44-51)
inline void set_end_points(Line& l)
{
    for (int k = 0; k < 2; k++) {
        l.interval[k].r = l.r / std::cos(l.interval[k].alfa - l.alfa);
        l.interval[k].alfa = l.interval[k].alfa + kPi;
        l.interval[k].alfa = l.interval[k].alfa > kPi ? l.interval[k].alfa - 2.0 * kPi : l.interval[k].alfa;
    }
}

// Recursive split-and-fit (simplifyPath.cpp:108-177): fit a line to the points; if the points'
// residual exceeds the expected one by three deviations, split at the point farthest from the
// chord and recurse, else keep the line with its covariance and end points.
inline void split_and_fit(const std::vector<PolarPoint>& P, std::vector<Line>& out)
{
    if (P.size() < 2) return;
    Line l = fit_line(P);
    double sum_di = 0.0, sum_var = 0.0;
    for (size_t i = 0; i < P.size(); i++)
        sum_di = sum_di + std::fabs(std::cos(P[i].alfa - l.alfa)) * 2 * (P[i].variance) / (std::sqrt(2 * kPi));
    for (size_t i = 0; i < P.size(); i++)
        sum_var = sum_var + std::cos(P[i].alfa - l.alfa) * std::cos(P[i].alfa - l.alfa) * P[i].variance *
                                P[i].variance * ((kPi - 2) / kPi);
    sum_var = std::sqrt(sum_var);
    const double t = residual_error(P, l);
    if (t > sum_di + sum_var * 3) {
        std::vector<XY> v(P.size());
        for (size_t i = 0; i < P.size(); i++) v[i] = to_xy(P[i]);
        const size_t index = farthest_from_chord(v);
        split_and_fit(std::vector<PolarPoint>(P.begin(), P.begin() + index), out);
        split_and_fit(std::vector<PolarPoint>(P.begin() + index, P.end()), out);
        return;
    }
    line_covariance(P, l.C);
    const Line at = l;
    l.interval.push_back(end_on_line(P, at, false));
    l.interval.push_back(end_on_line(P, at, true));
    set_end_points(l);
    out.push_back(l);
}

// LineConversion (lineFitting.cpp:608-649): drop lines with a negative, NaN or large (> 0.01)
// angle variance or an all-zero (alfa, r); then flip negative r
inline void drop_and_orient(std::vector<Line>& lines)
{
    std::vector<Line> kept;
    for (size_t i = 0; i < lines.size(); i++) {
        const Line& l = lines[i];
        if (l.C[0] < 0 || l.C[3] < 0) continue;
        if (std::isnan(l.C[0]) || std::isnan(l.C[1]) || std::isnan(l.C[2]) || std::isnan(l.C[3])) continue;
        if (l.alfa == 0 && l.r == 0) continue;
        if (l.C[0] > 0.01) continue;
        kept.push_back(l);
    }
    for (size_t i = 0; i < kept.size(); i++) flip_negative(kept[i]);
    lines.swap(kept);
}

// Split positions where consecutive points are more than 0.5 apart (lineFitting.cpp:561-607)
inline std::vector<size_t> gaps(const std::vector<PolarPoint>& P)
{
    std::vector<size_t> split;
    for (size_t i = 0; i + 1 < P.size(); i++) {
        const double d = std::sqrt(std::pow(P[i].r, 2) + std::pow(P[i + 1].r, 2) -
                                   2 * P[i].r * P[i + 1].r * std::cos(P[i + 1].alfa - P[i].alfa));
        if (d > 0.5) split.push_back(i + 1);
    }
    return split;
}

// LineExtraction (lineFitting.cpp:650-702)
inline std::vector<Line> extract_lines(std::vector<PolarPoint> P)
{
    std::vector<Line> lines;
    if (P.empty()) return lines;
    std::stable_sort(P.begin(), P.end(),
                     [](const PolarPoint& a, const PolarPoint& b) { return (a.alfa + kPi) < (b.alfa + kPi); });
    std::vector<size_t> split = gaps(P);
    if (!split.empty()) {
        std::rotate(P.begin(), P.begin() + split.back(), P.end());
        split = gaps(P);
    }
    if (split.empty()) {
        split_and_fit(P, lines);
    } else {
        std::vector<size_t> cut;
        cut.push_back(0);
        cut.insert(cut.end(), split.begin(), split.end());
        cut.push_back(P.size());
        for (size_t s = 0; s + 1 < cut.size(); s++)
            split_and_fit(std::vector<PolarPoint>(P.begin() + cut[s], P.begin() + cut[s + 1]), lines);
    }
    drop_and_orient(lines);
    return lines;
}

// main.cpp:37-56: message [r0, θ0, r1, θ1, …] → points (ranges > 0.05)
inline std::vector<PolarPoint> scan_to_points(const float* data, size_t count)
{
    std::vector<PolarPoint> pts;
    for (size_t i = 0; i + 1 < count; i += 2) {
        if (data[i] > 0.05) {
            PolarPoint p;
            p.alfa = data[i + 1] - M_PI;
            p.r = data[i];
            p.variance = 0.01;
            pts.push_back(p);
        }
    }
    return pts;
}

// main.cpp:57-61
inline void to_robot_frame(std::vector<Line>& lines)
{
    for (size_t i = 0; i < lines.size(); i++) {
        lines[i].alfa += M_PI;
        lines[i].alfa = lines[i].alfa > M_PI ? lines[i].alfa - 2.0 * M_PI : lines[i].alfa;
    }
}

// The EKF input (include/slam_ekf.h ekf_line), as Robot::localize reads a line
inline std::vector<ekf_line> to_ekf_lines(const std::vector<Line>& lines)
{
    std::vector<ekf_line> out(lines.size());
    for (size_t i = 0; i < lines.size(); i++) {
        out[i].alpha = lines[i].alfa;
        out[i].r = lines[i].r;
        for (int k = 0; k < 4; k++) out[i].R[k] = lines[i].C[k];
    }
    return out;
}

// ---- config 1 input: a 360-beam scan of a rectangular room with square pillars ----
struct Segment {
    double x0, y0, x1, y1;
};

struct Room {
    std::vector<Segment> walls;
};

inline Room make_room(double xmin, double ymin, double xmax, double ymax,
                      const std::vector<XY>& pillars = std::vector<XY>(), double half = 0.25)
{
    Room room;
    room.walls.push_back({xmin, ymin, xmax, ymin});
    room.walls.push_back({xmax, ymin, xmax, ymax});
    room.walls.push_back({xmax, ymax, xmin, ymax});
    room.walls.push_back({xmin, ymax, xmin, ymin});
    for (size_t k = 0; k < pillars.size(); k++) {
        const double cx = pillars[k].x, cy = pillars[k].y;
        room.walls.push_back({cx - half, cy - half, cx + half, cy - half});
        room.walls.push_back({cx + half, cy - half, cx + half, cy + half});
        room.walls.push_back({cx + half, cy + half, cx - half, cy + half});
        room.walls.push_back({cx - half, cy + half, cx - half, cy - half});
    }
    return room;
}

// Beam k at robot-frame angle θ_k = k·2π/beams from pose (x, y, θ): the range to the nearest
// wall (0 if none within max_range). Message layout [r0, θ0, r1, θ1, …], θ ∈ [0, 2π).
inline std::vector<float> raycast_room(const Room& room, const double pose[3], int beams = 360,
                                       double max_range = 30.0)
{
    std::vector<float> msg(2 * (size_t)beams);
    for (int k = 0; k < beams; k++) {
        const double th = 2.0 * M_PI * k / beams;
        const double phi = pose[2] + th;
        const double dx = std::cos(phi), dy = std::sin(phi);
        double best = max_range;
        for (size_t w = 0; w < room.walls.size(); w++) {
            const Segment& s = room.walls[w];
            const double ex = s.x1 - s.x0, ey = s.y1 - s.y0;
            const double den = dx * ey - dy * ex;
            if (std::fabs(den) < 1e-12) continue;
            const double qx = s.x0 - pose[0], qy = s.y0 - pose[1];
            const double t = (qx * ey - qy * ex) / den;      // along the beam
            const double u = (qx * dy - qy * dx) / den;      // along the wall
            if (t > 1e-9 && u >= 0.0 && u <= 1.0 && t < best) best = t;
        }
        msg[2 * k] = best < max_range ? (float)best : 0.0f;
        msg[2 * k + 1] = (float)th;
    }
    return msg;
}

// The whole caller side for one scan: message → robot-frame lines with C_AR
inline std::vector<Line> lines_from_scan(const std::vector<float>& msg)
{
    std::vector<Line> lines = extract_lines(scan_to_points(msg.data(), msg.size()));
    to_robot_frame(lines);
    return lines;
}

}  // namespace lx
}  // namespace slam_ekf
