// ekf_layout.h — HBM layout of the EKF state (host + device).
//
// The reference keeps P_t0 as a dense row-major n×n double array (Robot.h:62). Here P is split:
//   * robot strip  Rs[3][n]  (fp64): rows 0..2 of P (P_rr and the robot–landmark block). It is
//     the only part the motion model touches (Fx = I outside rows 0..2, Robot.cpp:153-167) and
//     the part every association step reads;
//   * landmark block P_ll = P[3:, 3:] (M = 2N square, symmetric), stored packed: only the
//     upper-triangular 32×32 tiles (bi <= bj), each tile a contiguous 32×32 block laid out in
//     the MFMA accumulator order of the storage precision, so the covariance downdate loads and
//     stores a tile as whole 16-byte-per-lane vectors straight into/out of the accumulators.
//     Diagonal tiles hold both triangles.
//
// f32 tile (v_mfma_f32_32x32x2_f32 C/D map: col = lane&31, row = (reg&3) + 8*(reg>>2) +
//   4*(lane>>5)): element (r, c) lives at lane = c + 32*((r>>2)&1), reg = (r&3) + 4*(r>>3);
//   stored at ((reg>>2)*64 + lane)*4 + (reg&3)   → one dwordx4 per lane per register quad.
// f64 tile (four 16×16 v_mfma_f64_16x16x4_f64 blocks; C/D map col = lane&15,
//   row = (lane>>4) + 4*reg): block (r>>4, c>>4), lane = (c&15) + 16*(r&3), reg = (r&15)>>2;
//   stored at ((blk*2 + (reg>>1))*64 + lane)*2 + (reg&1) → per block two dwordx4 per lane, each
//   instruction's 64 lanes one contiguous 1 KB (registers 0-1 of every lane, then 2-3).
#pragma once

#include <stddef.h>
#include <stdint.h>

#if defined(__HIPCC__)
#define EKF_HD __host__ __device__ __forceinline__
#else
#define EKF_HD inline
#endif

namespace ekf {

constexpr int TILE = 32;            // tile edge (both precisions)
constexpr int TILE_ELEMS = TILE * TILE;
#ifndef EKF_SCAN_THREADS
#define EKF_SCAN_THREADS 192
#endif
constexpr int SCAN_THREADS = EKF_SCAN_THREADS;   // association kernel: threads (= owned landmarks) per workgroup
constexpr int SCAN_BLOCK = SCAN_THREADS + 64;   // + one wave that replays the guessed winners' chain
constexpr int MAX_CAPACITY = 32768;             // landmarks per instance
constexpr int DD_THREADS = 256;     // downdate kernel: 4 waves, one tile per wave

struct Dims {
    int N;        // landmark capacity
    int n;        // 3 + 2N
    int M;        // 2N
    int nb;       // tile rows = ceil(M / 32)
    int64_t ntiles;   // nb(nb+1)/2
    int max_lines;
    int kmax;     // operand k columns: 2*max_lines rounded up to a multiple of 16
};

EKF_HD Dims make_dims(int N, int max_lines)
{
    Dims d;
    d.N = N;
    d.n = 3 + 2 * N;
    d.M = 2 * N;
    d.nb = (d.M + TILE - 1) / TILE;
    d.ntiles = (int64_t)d.nb * (d.nb + 1) / 2;
    d.max_lines = max_lines;
    d.kmax = ((2 * max_lines + 15) / 16) * 16;   // 8 f32 / 4 f64 k-steps per operand chunk
    return d;
}

// linear index of upper tile (bi <= bj), row-major over the upper triangle
EKF_HD int64_t tile_index(int bi, int bj, int nb)
{
    return (int64_t)bi * nb - (int64_t)bi * (bi - 1) / 2 + (bj - bi);
}

// offset of element (r, c) (0..31) inside one tile
EKF_HD int tile_off_f32(int r, int c)
{
    const int lane = c + 32 * ((r >> 2) & 1);
    const int g = r >> 3;
    return (g * 64 + lane) * 4 + (r & 3);
}

EKF_HD int tile_off_f64(int r, int c)
{
    const int blk = (r >> 4) * 2 + (c >> 4);
    const int rr = r & 15, cc = c & 15;
    const int lane = cc + 16 * (rr & 3);
    const int reg = rr >> 2;
    return ((blk * 2 + (reg >> 1)) * 64 + lane) * 2 + (reg & 1);
}

// element offset of P_ll(i, j) (0 <= i, j < M) in the packed tile array; symmetric lookup
template <typename T>
EKF_HD int64_t ll_offset(int i, int j, int nb);

template <>
EKF_HD int64_t ll_offset<float>(int i, int j, int nb)
{
    int bi = i >> 5, bj = j >> 5;
    int r = i & 31, c = j & 31;
    if (bi > bj) {
        int t = bi; bi = bj; bj = t;
        t = r; r = c; c = t;
    }
    return tile_index(bi, bj, nb) * TILE_ELEMS + tile_off_f32(r, c);
}

template <>
EKF_HD int64_t ll_offset<double>(int i, int j, int nb)
{
    int bi = i >> 5, bj = j >> 5;
    int r = i & 31, c = j & 31;
    if (bi > bj) {
        int t = bi; bi = bj; bj = t;
        t = r; r = c; c = t;
    }
    return tile_index(bi, bj, nb) * TILE_ELEMS + tile_off_f64(r, c);
}

// Downdate operands, per 32-row block rb, in MFMA operand order (see ekf_kernels.hip):
//   f32: op[rb][lane][s]        = X[rb*32 + (lane&31)][2s + (lane>>5)]          s < kmax/2
//   f64: op[rb][lane][h*ks + s] = X[rb*32 + 16h + (lane&15)][4s + (lane>>4)]    s < kmax/4
EKF_HD int64_t op_index_f32(int row, int k, int kmax)
{
    const int rb = row >> 5;
    const int lane = (row & 31) + 32 * (k & 1);
    const int s = k >> 1;
    return ((int64_t)rb * 64 + lane) * (kmax / 2) + s;
}

// bf16 operand planes (EKF_ARITH_BF16X6, kmax = 16): element (row, k) of plane pl (0 hi, 1 mid,
// 2 lo) in bf16 units; lane and slot as op_index_f32, so a lane's 8 values of one plane are one
// 16-byte v_mfma_f32_32x32x16_bf16 operand (its k-slot 8h + s carries k = 2s + h: the same
// permutation on both operands leaves every dot product's terms unchanged)
EKF_HD int64_t op_index_bf(int row, int k, int pl)
{
    const int rb = row >> 5;
    const int lane = (row & 31) + 32 * (k & 1);
    const int s = k >> 1;
    return (((int64_t)rb * 3 + pl) * 64 + lane) * 8 + s;
}

// The same operand order for npl planes per 32-row block: 3 (EKF_ARITH_BF16X6: hi, mid, lo bf16)
// or 2 (EKF_ARITH_F16X3: hi, lo fp16 of the row-scaled value)
EKF_HD int64_t op_index_pl(int row, int k, int pl, int npl)
{
    const int rb = row >> 5;
    const int lane = (row & 31) + 32 * (k & 1);
    const int s = k >> 1;
    return (((int64_t)rb * npl + pl) * 64 + lane) * 8 + s;
}

// EKF_ARITH_F16X3 plane exponent σ of an instance whose largest landmark variance is vmax: the
// planes hold fp16 parts of 2^σ·V, and every operand value of a plain step obeys |V_ik| ≤
// sqrt(P_ii) (V·Vᵀ is the step's downdate, P − V·Vᵀ ⪰ 0, and variances only shrink between
// augmentations), so |2^σ·V| ≤ 2^12: two binades below fp16's largest finite value, and values
// down to 2^-17 of the largest keep their full 22-bit hi + lo split. An empty map (vmax = 0) keeps
// PLANE_SIGMA_EMPTY until its first landmark.
constexpr int PLANE_SIGMA_EMPTY = 0;
// RES_PSIG of a step whose planes do not carry the instance's dynamic range (EKF_ARITH_F16X3: some
// active landmark's variance below 2^-4·4^-σ, where the fp16 lo part loses bits relative to that
// landmark's own scale): the flush runs the instance's group in the exact form (an exponent no
// plane uses, so it also differs from every other step's)
constexpr int PLANE_SIGMA_EXACT = -100000;
// the smallest 4^σ·variance whose rows keep the 22-bit split relative to their own scale: a row
// value x = 2^σ·V with |x| ~ sqrt(4^σ·var) keeps its lo part normal (|lo| ≈ 2^-11·|x| >= 2^-14)
// while 4^σ·var >= 2^-4 ... 2^-6; below it the split's error is no longer 2^-22 of the row's scale
constexpr double PLANE_VAR_MIN = 0.0625;   // 2^-4
EKF_HD int plane_sigma(double vmax)
{
    if (!(vmax > 0.0) || vmax > 1e300) return PLANE_SIGMA_EMPTY;
    // the largest s with vmax·4^s <= 2^24, i.e. sqrt(vmax)·2^s <= 2^12 (exact power-of-four steps)
    int s = 12;
    const double lim = 16777216.0;   // 2^24
    double x = vmax * 16777216.0;    // vmax·4^12
    while (x > lim && s > -60) { x *= 0.25; s--; }
    while (x * 4.0 <= lim && s < 60) { x *= 4.0; s++; }
    return s;
}

EKF_HD int64_t op_index_f64(int row, int k, int kmax)
{
    const int rb = row >> 5;
    const int h = (row >> 4) & 1;
    const int ks = kmax / 4;
    const int lane = (row & 15) + 16 * (k & 3);
    const int s = k >> 2;
    return ((int64_t)rb * 64 + lane) * (2 * ks) + h * ks + s;
}

}  // namespace ekf
