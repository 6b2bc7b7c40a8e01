// ekf_kernels.hip — gfx950 kernels of the EKF-SLAM update (slam_ros Robot::localize).
//
// Per scan (one "step"), all E ensemble instances at once:
//   1. scan_kernel (⌈N/256⌉ cooperating 256-thread workgroups per instance, stream S)
//        predict of the robot strip (Robot.cpp:130-286: Fx = I outside rows 0..2), then for
//        every observed line in order: Mahalanobis gating of all unmatched saved landmarks in
//        parallel + min-index reduction (== the reference's first passing candidate,
//        Robot.cpp:313-504); for a match the gain chain in deferred low-rank form
//        (Robot.cpp:515-602): W_t = P_{t-1}·H_tᵀ, K_t = W_t·S_t⁻¹, U_t = K_t·S_t, y += K_t·v_t.
//        Landmark augmentation (Robot.cpp:776-866) and the capacity reset decision
//        (Robot.cpp:893-904) run at the end of the same kernel; the new landmarks' rows of the
//        landmark block go to the step's slot (patch buffers), the rank-2m operands U/V to the
//        slot's MFMA-ordered operand buffers.
//   2. flush (stream S; D when pipelined): one pass over the packed landmark block applying a
//        group of T steps in order — per step X ← X − U_t·V_tᵀ (rank 2m on MFMA, the reference's
//        m dense n×n passes of Robot.cpp:560-572 fused), then that step's augmented rows, or the
//        reset. Each stored tile is read and written once per group. fp32/fp16 storage:
//        flush_f32_wave_kernel (groups of 6-8 steps: barrier-free waves, one wave-tile of
//        prefetch), flush_f32_persist2_kernel (≤ 4 steps, LDS-staged super-tiles),
//        flush_f32_sb_kernel (otherwise); fp64: downdate_f64_kernel (one tile per wave).
//
// Deferred reads: between flushes the association kernels read the landmark block with the
// pending steps applied on read (pll_block): per element, the same k-ordered fp32/fp64 FMA chain
// the MFMA executes, then the patch rounded to storage, so every read sees bit-for-bit the value
// the flush will store (tests/test_gpu_parity.py::test_deferred_flush_equals_drained).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <type_traits>

#include "ekf_kernels.h"

namespace ekf {

#define EKF_PI 3.14159265358979323846


// Storage type T of the landmark block → compute type C (MFMA / FMA chain) and tile layout L.
// fp16 storage computes in fp32 on the f32 layout and rounds to fp16 after every step, in the
// flush and in the on-read replay alike, so the stored value never depends on when it is flushed.
// It holds 2^x·P with a per-instance exponent x (ScanParams/DowndateParams::pexp, default 10:
// |P| < 64 representable, normal down to 6e-8; chosen at upload from the largest landmark
// variance, ekf_api.hip choose_exponent). The fp16 path computes in that scaled domain
// throughout: the scan writes the U operand scaled by 2^x (exact), so flush and on-read replay
// both run acc = 2^x·X − (2^x·U)·Vᵀ, bit-for-bit 2^x × the unscaled chain, and round with two
// conversions per element; values leave the scaled domain only where they are read as P.
template <typename T> struct Stor {
    using C = T;
    using L = T;
    static constexpr bool half = false;
};
template <> struct Stor<_Float16> {
    using C = float;
    using L = float;
    static constexpr bool half = true;
};

template <typename T>
__device__ __forceinline__ T to_store(typename Stor<T>::C x)
{
    return (T)x;
}

template <typename T>
__device__ __forceinline__ typename Stor<T>::C from_store(T h)
{
    return (typename Stor<T>::C)h;
}

template <typename T>
__device__ __forceinline__ typename Stor<T>::C round_step(typename Stor<T>::C x)
{
    if constexpr (Stor<T>::half) {
        // the same instruction on every path: the compiler may otherwise pair two roundings into
        // v_cvt_pk_f16_f32 at some call sites, which does not round fp16 subnormals like
        // v_cvt_f16_f32 (the flush and the on-read replay must round bit-identically)
        float r;
        asm("v_cvt_f16_f32 %0, %1\n\tv_cvt_f32_f16 %0, %0" : "=v"(r) : "v"(x));
        return r;
    } else {
        return (typename Stor<T>::C)(T)x;
    }
}

// P value (fp64) → scaled compute domain (exponent ex, fp16 storage only), and back: power-of-two
// scalings, exact in fp32 / fp64
template <typename T>
__device__ __forceinline__ typename Stor<T>::C to_domain(double v, int ex)
{
    using C = typename Stor<T>::C;
    if constexpr (Stor<T>::half) return ldexpf((C)v, ex);
    else return (C)v;
}

template <typename T>
__device__ __forceinline__ double from_domain(typename Stor<T>::C x, int ex)
{
    if constexpr (Stor<T>::half) return ldexp((double)x, -ex);
    else return (double)x;
}

// the storage exponent of instance e (0 unless fp16)
template <typename T>
__device__ __forceinline__ int storage_exp(const int* pexp, int e);

// A flush's U operand rows of instance e: as stored, or (DowndateParams::usym: symmetric operands,
// U = −2^x·V exactly) the V rows times us_of(). Either way the same fp32 values reach the MFMAs.
template <typename TS>
__device__ __forceinline__ float us_of(const DowndateParams& p, int e)
{
    return p.usym ? -ldexpf(1.0f, storage_exp<TS>(p.pexp, e)) : 1.0f;
}
__device__ __forceinline__ const float* u_rows_flush(const DowndateParams& p, const Slot& sq, int e, size_t opstride)
{
    return reinterpret_cast<const float*>(p.usym ? sq.Vop : sq.Uop) + e * opstride;
}

template <typename T>
__device__ __forceinline__ int storage_exp(const int* pexp, int e)
{
    if constexpr (Stor<T>::half) return pexp[e];
    else return 0;
}

__device__ __forceinline__ double normalize_radian(double rad)
{
    // Robot.cpp:62-71
    if (fabs(rad) <= EKF_PI) return rad;   // (the common case, one test)
    if (rad > EKF_PI) {
        rad = rad - (2.0 * EKF_PI + floor(rad / (2.0 * EKF_PI)) * 2.0 * EKF_PI);
    } else if (rad < -EKF_PI) {
        rad = rad + (2.0 * EKF_PI + floor(fabs(rad) / (2.0 * EKF_PI)) * 2.0 * EKF_PI);
    }
    return rad;
}

// 1/a for a finite nonzero a of moderate exponent: v_rcp_f64 and two Newton steps (within an ulp;
// the association chain's divisions, which sit on its critical path, take this instead of the
// correctly rounded division)
__device__ __forceinline__ double rcp_nr(double a)
{
    double r = __builtin_amdgcn_rcp(a);
    double e = fma(-a, r, 1.0);
    r = fma(r, e, r);
    e = fma(-a, r, 1.0);
    return fma(r, e, r);
}

// gsl_linalg_LU_decomp + LU_invert on 2x2 (Robot.cpp:449-457): partial pivoting, the elimination
// and the two back substitutions of GSL, with the pivots' reciprocals (rcp_nr) in place of the
// divisions (agrees with GSL within an ulp or two per entry); false when U is singular (GSL_EDOM),
// leaving Si untouched.
__device__ __forceinline__ bool lu_invert2(const double S[4], double Si[4])
{
    // the row swap by selects and the elimination unconditionally (a zero pivot makes r0 infinite,
    // and the function then returns before using anything derived from it): the same values as
    // the branching form, without exec-mask branches on the association's serial chain
    const bool sw = fabs(S[2]) > fabs(S[0]);
    double a0 = sw ? S[2] : S[0], a1 = sw ? S[3] : S[1], a2 = sw ? S[0] : S[2], a3 = sw ? S[1] : S[3];
    const int p0 = sw ? 1 : 0, p1 = sw ? 0 : 1;
    const double r0 = rcp_nr(a0);
    const double l = a2 * r0;
    a2 = l;
    a3 -= l * a1;
    if (a0 == 0.0 || a3 == 0.0) return false;
    const double r3 = rcp_nr(a3);
#pragma unroll
    for (int c = 0; c < 2; c++) {
        double b0 = (p0 == c) ? 1.0 : 0.0;
        double b1 = (p1 == c) ? 1.0 : 0.0;
        b1 = b1 - a2 * b0;
        const double x1 = b1 * r3;
        const double x0 = (b0 - a1 * x1) * r0;
        Si[c] = x0;
        Si[2 + c] = x1;
    }
    return true;
}

// ---------------------------------------------------------------------------------------
// Landmark block as seen by a step: X plus the pending (not yet flushed) steps, in order.
// ---------------------------------------------------------------------------------------
template <typename T>
struct PllView {
    const T* X;
    int nb, kmax, M, max_lines;
    int e;            // instance
    int ex;           // storage exponent of instance e (fp16)
    size_t opstride;  // operand elements per instance
    int npend;        // pending steps (oldest first)
    const Slot* pend;
    const int4* ctl;  // per pending step {reset, ks, nadd, s0} of instance e (LDS copy)
    int rnd;          // fp16: round after every pending step, as the exact flush does (0 under
                      // the split-bf16 flush, which rounds once per group)
    int usym;         // symmetric operands: U = us·V, the U rows not stored (ScanParams::usym)
    float us;         // −2^ex if usym, else 1 (U rows read as stored)
};

// Step q's U rows as stored, or its V rows (scaled by v.us on use) for symmetric operands
template <typename T>
__device__ __forceinline__ const float* u_rows_f32(const PllView<T>& v, const Slot& sq)
{
    return reinterpret_cast<const float*>(v.usym ? sq.Vop : sq.Uop) + v.e * v.opstride;
}

// fp16 rounding of a replayed element (identity for fp32 / fp64 storage)
template <typename T>
__device__ __forceinline__ typename Stor<T>::C vround(const PllView<T>& v, typename Stor<T>::C x)
{
    return v.rnd ? round_step<T>(x) : x;
}

typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef float f32x2v __attribute__((ext_vector_type(2)));

// Staged rows of a guessed column (LDS, per column and pending step: [U | V][row half][8]):
// the U side as in the operand layout, row half rh = (k parity) · 2 + (row of the pair), 8 k each;
// the V side interleaved by row pair, (rh, k) at (rh >> 1) · 16 + 2k + (rh & 1), so that one
// float2 holds both rows of a k (a packed-FMA operand).
__device__ __forceinline__ int stage_v_index(int rh, int k) { return (rh >> 1) * 16 + 2 * k + (rh & 1); }

// EKF_ARITH_BF16X6: v = hi + mid + lo, each a bf16 (the upper half of an fp32): truncation leaves
// an exact fp32 remainder of at most 16, then 8 significant bits, so the three parts are exact.
// Packs (a, b) into one dword per part, a in the low half (operand element order)
__device__ __forceinline__ void split_pack(float a, float b, unsigned (&o)[3])
{
#pragma unroll
    for (int pl = 0; pl < 3; pl++) {
        const unsigned ua = __builtin_bit_cast(unsigned, a) & 0xffff0000u;
        const unsigned ub = __builtin_bit_cast(unsigned, b) & 0xffff0000u;
        o[pl] = (ua >> 16) | ub;
        a -= __builtin_bit_cast(float, ua);
        b -= __builtin_bit_cast(float, ub);
    }
}

// Stored 2×2 block at rows a0, a0+1 and columns b0, b0+1 (a0, b0 even, a0's tile <= b0's):
// acc = {(a0,b0), (a0,b0+1), (a0+1,b0), (a0+1,b0+1)}. In the f32 tile layout the two rows of a
// column are adjacent and the two columns are 4 elements apart: two paired loads.
template <typename T>
__device__ __forceinline__ void load_block(const PllView<T>& v, int a0, int b0, typename Stor<T>::C (&acc)[4])
{
    using L = typename Stor<T>::L;
    if constexpr (sizeof(L) == 4) {
        const T* x = v.X + ll_offset<L>(a0, b0, v.nb);
        if constexpr (sizeof(T) == 4) {
            const float2 c0 = *reinterpret_cast<const float2*>(x);
            const float2 c1 = *reinterpret_cast<const float2*>(x + 4);
            acc[0] = from_store<T>(c0.x); acc[2] = from_store<T>(c0.y);
            acc[1] = from_store<T>(c1.x); acc[3] = from_store<T>(c1.y);
        } else {
            typedef T t2 __attribute__((ext_vector_type(2)));
            const t2 c0 = *reinterpret_cast<const t2*>(x);
            const t2 c1 = *reinterpret_cast<const t2*>(x + 4);
            acc[0] = from_store<T>(c0.x); acc[2] = from_store<T>(c0.y);
            acc[1] = from_store<T>(c1.x); acc[3] = from_store<T>(c1.y);
        }
    } else {
#pragma unroll
        for (int p = 0; p < 2; p++)
#pragma unroll
            for (int c = 0; c < 2; c++) acc[p * 2 + c] = from_store<T>(v.X[ll_offset<L>(a0 + p, b0 + c, v.nb)]);
    }
}

// The rows a step appended (Robot.cpp:845-862) replace block (i0, j0) if it lies in them:
// requested orientation, rounded as they are stored.
template <typename T>
__device__ __forceinline__ void patch_block(const PllView<T>& v, const Slot& sq, int4 cw, int i0, int j0,
                                            bool swap, typename Stor<T>::C (&acc)[4])
{
    const int nadd = cw.z, s0 = cw.w;
    const int li = i0 >> 1, lj = j0 >> 1;
    const int hi = li > lj ? li : lj;
    if (hi >= s0 && hi < s0 + nadd) {
        const int qa = hi - s0;
        const double* pdg = sq.patch_diag + (size_t)v.e * v.max_lines * 4;
        const double* prw = sq.patch + ((size_t)v.e * v.max_lines + qa) * 2 * v.M;
        double raw[4];
        if (li == lj) {
            raw[0] = pdg[qa * 4 + 0]; raw[1] = pdg[qa * 4 + 1];
            raw[2] = pdg[qa * 4 + 2]; raw[3] = pdg[qa * 4 + 3];
        } else if (li > lj) {
            raw[0] = prw[j0]; raw[1] = prw[j0 + 1];
            raw[2] = prw[v.M + j0]; raw[3] = prw[v.M + j0 + 1];
        } else {
            raw[0] = prw[i0]; raw[1] = prw[v.M + i0];
            raw[2] = prw[i0 + 1]; raw[3] = prw[v.M + i0 + 1];
        }
        if (swap) {
            acc[0] = vround<T>(v, to_domain<T>(raw[0], v.ex)); acc[1] = vround<T>(v, to_domain<T>(raw[2], v.ex));
            acc[2] = vround<T>(v, to_domain<T>(raw[1], v.ex)); acc[3] = vround<T>(v, to_domain<T>(raw[3], v.ex));
        } else {
            acc[0] = vround<T>(v, to_domain<T>(raw[0], v.ex)); acc[1] = vround<T>(v, to_domain<T>(raw[1], v.ex));
            acc[2] = vround<T>(v, to_domain<T>(raw[2], v.ex)); acc[3] = vround<T>(v, to_domain<T>(raw[3], v.ex));
        }
    }
}

// One pending step's downdate on B blocks (i0, j0[b]) in their stored orientations (pll_blocks):
// the owned rows i0, i0+1 of U and V are loaded once per k-chunk (their lanes' addresses are
// spread over many cache lines) and each column landmark's rows once (U_col for a transposed
// block, V_col otherwise; the guessed columns are the same for the whole wave). Per element the
// FMA chain of pll_blocks' per-block form, operand for operand.
template <typename T, int B>
__device__ __forceinline__ void pll_shared_step(const PllView<T>& v, const Slot& sq, int ks, int i0,
                                                const int (&j0)[B], const bool (&swap)[B],
                                                typename Stor<T>::C (&acc)[B][4])
{
    using C = typename Stor<T>::C;
    if constexpr (sizeof(C) == 4) {
        const int kh = v.kmax / 2;
        const float* U = u_rows_f32(v, sq);
        const float* V = reinterpret_cast<const float*>(sq.Vop) + v.e * v.opstride;
        const float us = v.us;
        auto row = [&](int r) { return ((size_t)(r >> 5) * 64 + (r & 31)) * kh; };
        const float* uo = U + row(i0);
        const float* vo = V + row(i0);
        const float* xc[B];
#pragma unroll
        for (int b = 0; b < B; b++) xc[b] = (swap[b] ? U : V) + row(j0[b]);
        for (int s0 = 0; s0 < ks; s0 += 4) {
            // [row, row + 1] × [k half 0, k half 1] of the owned U and V rows
            const f32x4v ue0 = *reinterpret_cast<const f32x4v*>(uo + s0) * us;
            const f32x4v ue1 = *reinterpret_cast<const f32x4v*>(uo + kh + s0) * us;
            const f32x4v uo0 = *reinterpret_cast<const f32x4v*>(uo + 32 * kh + s0) * us;
            const f32x4v uo1 = *reinterpret_cast<const f32x4v*>(uo + 33 * kh + s0) * us;
            const f32x4v ve0 = *reinterpret_cast<const f32x4v*>(vo + s0);
            const f32x4v ve1 = *reinterpret_cast<const f32x4v*>(vo + kh + s0);
            const f32x4v vo0 = *reinterpret_cast<const f32x4v*>(vo + 32 * kh + s0);
            const f32x4v vo1 = *reinterpret_cast<const f32x4v*>(vo + 33 * kh + s0);
#pragma unroll
            for (int b = 0; b < B; b++) {
                const f32x4v ce0 = *reinterpret_cast<const f32x4v*>(xc[b] + s0);
                const f32x4v ce1 = *reinterpret_cast<const f32x4v*>(xc[b] + kh + s0);
                const f32x4v co0 = *reinterpret_cast<const f32x4v*>(xc[b] + 32 * kh + s0);
                const f32x4v co1 = *reinterpret_cast<const f32x4v*>(xc[b] + 33 * kh + s0);
                const bool sw = swap[b];
                const f32x4v ae0 = sw ? ce0 * us : ue0, ae1 = sw ? ce1 * us : ue1, ao0 = sw ? co0 * us : uo0,
                             ao1 = sw ? co1 * us : uo1;
                const f32x4v be0 = sw ? ve0 : ce0, be1 = sw ? ve1 : ce1, bo0 = sw ? vo0 : co0, bo1 = sw ? vo1 : co1;
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    if (s0 + s >= ks) break;
                    acc[b][0] = fmaf(ao0[s], bo0[s], fmaf(ae0[s], be0[s], acc[b][0]));
                    acc[b][1] = fmaf(ao0[s], bo1[s], fmaf(ae0[s], be1[s], acc[b][1]));
                    acc[b][2] = fmaf(ao1[s], bo0[s], fmaf(ae1[s], be0[s], acc[b][2]));
                    acc[b][3] = fmaf(ao1[s], bo1[s], fmaf(ae1[s], be1[s], acc[b][3]));
                }
            }
        }
    } else {
        const int kq = v.kmax / 4;
        const double* U = reinterpret_cast<const double*>(sq.Uop) + v.e * v.opstride;
        const double* V = reinterpret_cast<const double*>(sq.Vop) + v.e * v.opstride;
        auto row = [&](int r) { return ((size_t)(r >> 5) * 64 + (r & 15)) * (2 * kq) + ((r >> 4) & 1) * kq; };
        const double* uo = U + row(i0);
        const double* vo = V + row(i0);
        const double* xc[B];
#pragma unroll
        for (int b = 0; b < B; b++) xc[b] = (swap[b] ? U : V) + row(j0[b]);
        for (int s = 0; s < ks; s++)
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const size_t o = (size_t)16 * kk * 2 * kq + s;
                const double u0 = uo[o], u1 = uo[o + 2 * kq];
                const double w0 = vo[o], w1 = vo[o + 2 * kq];
#pragma unroll
                for (int b = 0; b < B; b++) {
                    const double c0 = xc[b][o], c1 = xc[b][o + 2 * kq];
                    const bool sw = swap[b];
                    const double x0 = sw ? c0 : u0, x1 = sw ? c1 : u1;
                    const double y0 = sw ? w0 : c0, y1 = sw ? w1 : c1;
                    acc[b][0] = fma(x0, y0, (double)acc[b][0]);
                    acc[b][1] = fma(x0, y1, (double)acc[b][1]);
                    acc[b][2] = fma(x1, y0, (double)acc[b][2]);
                    acc[b][3] = fma(x1, y1, (double)acc[b][3]);
                }
            }
    }
#pragma unroll
    for (int b = 0; b < B; b++)
#pragma unroll
        for (int k = 0; k < 4; k++) acc[b][k] = vround<T>(v, acc[b][k]);
}

// 2x2 blocks (i0, i0+1) × (j0[b], j0[b]+1), b < B, of the landmark block (i0, j0[b] even) as
// they will be once the pending steps are flushed: per step (in order) a reset, or the rank-2m
// downdate as the k-ordered FMA chain the MFMA executes, then the step's augmented rows rounded
// to storage. The B blocks share one pass over the pending steps so that their loads overlap.
template <typename T, int B>
__device__ __forceinline__ void pll_blocks(const PllView<T>& v, int i0, const int (&j0)[B], double (&out)[B][4])
{
    using C = typename Stor<T>::C;
    bool swap[B];
    int a0[B], b0[B];
    C acc[B][4];
#pragma unroll
    for (int b = 0; b < B; b++) {
        swap[b] = (i0 >> 5) > (j0[b] >> 5);
        a0[b] = swap[b] ? j0[b] : i0;   // stored orientation
        b0[b] = swap[b] ? i0 : j0[b];
        load_block<T>(v, a0[b], b0[b], acc[b]);
    }
    for (int q = 0; q < v.npend; q++) {
        const Slot& sq = v.pend[q];
        const int4 cw = v.ctl[q];
        if (cw.x) {
#pragma unroll
            for (int b = 0; b < B; b++) acc[b][0] = acc[b][1] = acc[b][2] = acc[b][3] = (C)0;
            continue;
        }
        const int ks = cw.y;
        if (ks > 0 && B > 1) {
            // several blocks: the owned rows' U and V loaded once per k-chunk, each column's
            // one operand per block (a block stored in owned-first orientation runs U_own·V_col,
            // a transposed one U_col·V_own): the same operands as the per-block form below
            pll_shared_step<T, B>(v, sq, ks, i0, j0, swap, acc);
        } else if (ks > 0) {
            if constexpr (sizeof(C) == 4) {
                // v_mfma_f32_32x32x2_f32 = ordered fmaf chain (k0 lanes 0-31, then k1)
                const int kh = v.kmax / 2;
                const float* ua[B];
                const float* vb[B];
#pragma unroll
                for (int b = 0; b < B; b++) {
                    ua[b] = u_rows_f32(v, sq) + ((size_t)(a0[b] >> 5) * 64 + (a0[b] & 31)) * kh;   // row a0; a0+1 at +kh
                    vb[b] = reinterpret_cast<const float*>(sq.Vop) + v.e * v.opstride +
                            ((size_t)(b0[b] >> 5) * 64 + (b0[b] & 31)) * kh;
                }
                for (int s0 = 0; s0 < ks; s0 += 4) {
                    f32x4v ae0[B], ae1[B], ao0[B], ao1[B], be0[B], be1[B], bo0[B], bo1[B];
#pragma unroll
                    for (int b = 0; b < B; b++) {
                        ae0[b] = *reinterpret_cast<const f32x4v*>(ua[b] + s0) * v.us;
                        ae1[b] = *reinterpret_cast<const f32x4v*>(ua[b] + kh + s0) * v.us;
                        ao0[b] = *reinterpret_cast<const f32x4v*>(ua[b] + 32 * kh + s0) * v.us;
                        ao1[b] = *reinterpret_cast<const f32x4v*>(ua[b] + 33 * kh + s0) * v.us;
                        be0[b] = *reinterpret_cast<const f32x4v*>(vb[b] + s0);
                        be1[b] = *reinterpret_cast<const f32x4v*>(vb[b] + kh + s0);
                        bo0[b] = *reinterpret_cast<const f32x4v*>(vb[b] + 32 * kh + s0);
                        bo1[b] = *reinterpret_cast<const f32x4v*>(vb[b] + 33 * kh + s0);
                    }
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        if (s0 + s >= ks) break;
#pragma unroll
                        for (int b = 0; b < B; b++) {
                            acc[b][0] = fmaf(ao0[b][s], bo0[b][s], fmaf(ae0[b][s], be0[b][s], acc[b][0]));
                            acc[b][1] = fmaf(ao0[b][s], bo1[b][s], fmaf(ae0[b][s], be1[b][s], acc[b][1]));
                            acc[b][2] = fmaf(ao1[b][s], bo0[b][s], fmaf(ae1[b][s], be0[b][s], acc[b][2]));
                            acc[b][3] = fmaf(ao1[b][s], bo1[b][s], fmaf(ae1[b][s], be1[b][s], acc[b][3]));
                        }
                    }
                }
            } else {
                // v_mfma_f64_16x16x4_f64 = ordered fma chain over k = 4s..4s+3
                const int kq = v.kmax / 4;
                const double* ua[B];
                const double* vb[B];
#pragma unroll
                for (int b = 0; b < B; b++) {
                    ua[b] = reinterpret_cast<const double*>(sq.Uop) + v.e * v.opstride +
                            ((size_t)(a0[b] >> 5) * 64 + (a0[b] & 15)) * (2 * kq) + ((a0[b] >> 4) & 1) * kq;
                    vb[b] = reinterpret_cast<const double*>(sq.Vop) + v.e * v.opstride +
                            ((size_t)(b0[b] >> 5) * 64 + (b0[b] & 15)) * (2 * kq) + ((b0[b] >> 4) & 1) * kq;
                }
                for (int s = 0; s < ks; s++)
#pragma unroll
                    for (int kk = 0; kk < 4; kk++) {
                        const size_t o = (size_t)16 * kk * 2 * kq + s;
#pragma unroll
                        for (int b = 0; b < B; b++) {
                            const double x0 = ua[b][o], x1 = ua[b][o + 2 * kq];
                            const double y0 = vb[b][o], y1 = vb[b][o + 2 * kq];
                            acc[b][0] = fma(x0, y0, (double)acc[b][0]);
                            acc[b][1] = fma(x0, y1, (double)acc[b][1]);
                            acc[b][2] = fma(x1, y0, (double)acc[b][2]);
                            acc[b][3] = fma(x1, y1, (double)acc[b][3]);
                        }
                    }
            }
#pragma unroll
            for (int b = 0; b < B; b++)
#pragma unroll
                for (int k = 0; k < 4; k++) acc[b][k] = vround<T>(v, acc[b][k]);
        }
        if (cw.z > 0) {
#pragma unroll
            for (int b = 0; b < B; b++) patch_block<T>(v, sq, cw, i0, j0[b], swap[b], acc[b]);
        }
    }
#pragma unroll
    for (int b = 0; b < B; b++) {
        if (swap[b]) {
            out[b][0] = from_domain<T>(acc[b][0], v.ex); out[b][1] = from_domain<T>(acc[b][2], v.ex);
            out[b][2] = from_domain<T>(acc[b][1], v.ex); out[b][3] = from_domain<T>(acc[b][3], v.ex);
        } else {
            out[b][0] = from_domain<T>(acc[b][0], v.ex); out[b][1] = from_domain<T>(acc[b][1], v.ex);
            out[b][2] = from_domain<T>(acc[b][2], v.ex); out[b][3] = from_domain<T>(acc[b][3], v.ex);
        }
    }
}

template <typename T>
__device__ __forceinline__ void pll_block(const PllView<T>& v, int i0, int j0, double out[4])
{
    const int js[1] = {j0};
    double o[1][4];
    pll_blocks<T, 1>(v, i0, js, o);
    out[0] = o[0][0]; out[1] = o[0][1]; out[2] = o[0][2]; out[3] = o[0][3];
}

// The association arithmetic contracts a·b + c only within one source expression, so a
// function inlined into different kernels or phases rounds identically everywhere (the
// speculative and sequential association paths must agree bit for bit).
#pragma clang fp contract(on)

// Uniform per-line package published by the matching thread (LDS).
enum {
    C_S = 0, C_SI = 4, C_V = 8, C_H = 10, C_KR = 13, C_UR = 19, C_WORDS = 25,
};

struct Cand {
    double S[4];
    double Si[4];
    double v[2];
    double h10, h11, h1l;
    double w0, w1, d2;   // S⁻¹v and the distance (cand_amb)
    int pass;
    int singular;
    int amb;   // the decision is within the storage precision of the gate (gate_eta)
};

// The storage precision of the gate (round 5). P as stored differs from the fp64 reference's by
// the roundings of its storage and of the flush's products; eta bounds that difference relative
// to the magnitudes |P_ab| <= sqrt(P_aa·P_bb) of the 5×5 block. With H0 = (0, 0, −1, 1, 0) and
// ‖H1‖² = 2 + h1l², |ΔS_ab| <= eta·s_a·s_b with s_a = Σ_k |H_ak|·√P_kk, and by Cauchy-Schwarz
// s0² <= m0 = 2(|p22| + |daa|), s1² <= m1 = ‖H1‖²·tr|P5|, s0·s1 <= (m0 + m1)/2. The filters add
// these (root-free) bounds to their error bounds (a rejection then
// holds for every P within eta; the decisions themselves are unchanged, so every path still agrees
// bit for bit), and the exact evaluation reports a distance within the first-order bound
// eta·(|w0|·s0 + |w1|·s1)², w = S⁻¹v, of the gate as ambiguous: EKF_ST_PRECISION, the statement
// that this state does not resolve the reference's decision (SURVEY §8d's run-away world, where
// S is the difference of terms 1e10 times larger). fp32 storage: 2^-16 (16 × the
// per-group P bar of 1e-6); fp16: 2^-8; fp64: 2^-44.
template <typename T> constexpr double gate_eta()
{
    return sizeof(T) == 8 ? 0x1p-44 : sizeof(T) == 4 ? 0x1p-16 : 0x1p-8;
}

// 5×5 block {0,1,2, 3+2j, 4+2j} of the current P: robot 3×3 (R33), robot–landmark columns
// (Rs, owned), landmark diagonal block (Dj, owned), and H·P·Hᵀ + R for given H row 1.
struct Block5 {
    double p00, p01, p02, p10, p11, p12, p20, p21, p22;
    double p0a, p1a, p2a, p0b, p1b, p2b;
    double daa, dab, dba, dbb;
};

__device__ __forceinline__ void load_block5(Block5& b, int j, const double* R33, const double* Rs,
                                            int n, const double Dj[4])
{
    const int l0 = 3 + 2 * j;
    b.p00 = R33[0]; b.p01 = R33[1]; b.p02 = R33[2];
    b.p10 = R33[3]; b.p11 = R33[4]; b.p12 = R33[5];
    b.p20 = R33[6]; b.p21 = R33[7]; b.p22 = R33[8];
    const double2 ra = *reinterpret_cast<const double2*>(Rs + l0);
    const double2 rb = *reinterpret_cast<const double2*>(Rs + n + l0);
    const double2 rc = *reinterpret_cast<const double2*>(Rs + 2 * n + l0);
    b.p0a = ra.x; b.p0b = ra.y;
    b.p1a = rb.x; b.p1b = rb.y;
    b.p2a = rc.x; b.p2b = rc.y;
    b.daa = Dj[0]; b.dab = Dj[1]; b.dba = Dj[2]; b.dbb = Dj[3];
}

// S = H·P5·Hᵀ + R in the reference's summation order (Robot.cpp:397-405); also returns the
// intermediate rows hp0 = hr0·P5, hp1 = hr1·P5 (hr0 = (0,0,-1,1,0), hr1 = (h10,h11,0,h1l,1)).
__device__ __forceinline__ void innovation_cov(const Block5& b, double h10, double h11, double h1l,
                                               const double Rm[4], double S[4], double hp0[5],
                                               double hp1[5])
{
    hp0[0] = -b.p20 + b.p0a; hp0[1] = -b.p21 + b.p1a; hp0[2] = -b.p22 + b.p2a;
    hp0[3] = -b.p2a + b.daa; hp0[4] = -b.p2b + b.dab;
    hp1[0] = h10 * b.p00 + h11 * b.p10 + h1l * b.p0a + b.p0b;
    hp1[1] = h10 * b.p01 + h11 * b.p11 + h1l * b.p1a + b.p1b;
    hp1[2] = h10 * b.p02 + h11 * b.p12 + h1l * b.p2a + b.p2b;
    hp1[3] = h10 * b.p0a + h11 * b.p1a + h1l * b.daa + b.dba;
    hp1[4] = h10 * b.p0b + h11 * b.p1b + h1l * b.dab + b.dbb;
    S[0] = -hp0[2] + hp0[3] + Rm[0];
    S[1] = hp0[0] * h10 + hp0[1] * h11 + hp0[3] * h1l + hp0[4] + Rm[1];
    S[2] = -hp1[2] + hp1[3] + Rm[2];
    S[3] = hp1[0] * h10 + hp1[1] * h11 + hp1[3] * h1l + hp1[4] + Rm[3];
}

__device__ __forceinline__ double innovation_angle(double za, double ma, double xp2)
{
    // h0 (Robot.cpp:423-426) and the 2π fold of v0 (Robot.cpp:465-475)
    const double h0 = normalize_radian(ma - xp2);
    double v0 = za - h0;
    if (fabs(v0 - 2.0 * EKF_PI) < fabs(v0)) v0 -= 2.0 * EKF_PI;
    else if (fabs(v0 + 2.0 * EKF_PI) < fabs(v0)) v0 += 2.0 * EKF_PI;
    return v0;
}

// sin/cos of a landmark angle from those of its value at the start of the scan: the angle
// moves by small Kalman corrections within a scan, so sin/cos(ma0 + δ) by the addition formula
// with Taylor series in δ (|δ| <= 1/64: truncation below 1e-19), and the full fp64 sincos
// otherwise. Every path that evaluates a candidate uses this form, so they agree bit for bit.
__device__ __forceinline__ void sincos_near(double ma, double ma0, double s0, double c0, double& sn,
                                            double& cs)
{
    const double dl = ma - ma0;
    if (fabs(dl) <= 0.0009765625) {
        // |δ| <= 2^-10: sin δ = δ − δ³/6 (next term ≤ 8e-18), 1 − cos δ = δ²/2 − δ⁴/24 (≤ 2e-21)
        const double d2 = dl * dl;
        const double sd = dl * (1.0 - d2 * (1.0 / 6.0));
        const double cm = d2 * 0.5 * (1.0 - d2 * (1.0 / 12.0));
        sn = s0 - (s0 * cm - c0 * sd);
        cs = c0 - (c0 * cm + s0 * sd);
    } else if (fabs(dl) <= 0.015625) {
        const double d2 = dl * dl;
        const double sd = dl * (1.0 - d2 * (1.0 / 6.0) * (1.0 - d2 * (1.0 / 20.0) * (1.0 - d2 * (1.0 / 42.0))));
        const double cm = d2 * 0.5 * (1.0 - d2 * (1.0 / 12.0) * (1.0 - d2 * (1.0 / 30.0) * (1.0 - d2 * (1.0 / 56.0))));
        sn = s0 - (s0 * cm - c0 * sd);   // s0·cos δ + c0·sin δ, cos δ = 1 − cm
        cs = c0 - (c0 * cm + s0 * sd);   // c0·cos δ − s0·sin δ
    } else {
        sincos(ma, &sn, &cs);
    }
}

__device__ __forceinline__ int cand_amb(const Block5& b, const Cand& c, double gate, double eta);

// Exact candidate evaluation in fp64 (Robot.cpp:367-489). AMB = false leaves c.amb for cand_amb
// (the replay wave evaluates it after it has published the line's package)
template <bool AMB = true>
__device__ __forceinline__ void eval_candidate(const Block5& b, double ma, double mr, double sn,
                                               double cs, const double xp[3], double za, double zr,
                                               const double Rm[4], double gate, double eta, Cand& c)
{
    c.h10 = -cs;
    c.h11 = -sn;
    c.h1l = xp[0] * sn - xp[1] * cs;
    double hp0[5], hp1[5];
    innovation_cov(b, c.h10, c.h11, c.h1l, Rm, c.S, hp0, hp1);
    const double h1 = mr - (xp[0] * cs + xp[1] * sn);
    c.Si[0] = c.Si[1] = c.Si[2] = c.Si[3] = 0.0;
    c.singular = lu_invert2(c.S, c.Si) ? 0 : 1;
    const double v0 = innovation_angle(za, ma, xp[2]);
    const double v1 = zr - h1;
    c.v[0] = v0;
    c.v[1] = v1;
    // vᵀ·S⁻¹·v (Robot.cpp:479-486); gate (:489): a NaN distance passes, as in the reference
    const double vs0 = v0 * c.Si[0] + v1 * c.Si[2];
    const double vs1 = v0 * c.Si[1] + v1 * c.Si[3];
    const double d2 = vs0 * v0 + vs1 * v1;
    // sqrt(|d2|) > gate decided without the square root where |d2| is more than 2^-40 (relative)
    // away from gate²: sqrt is correctly rounded and monotonic, so such a |d2| gives the same
    // answer; near the gate, and for NaN (which passes), the reference's expression itself
    const double a = fabs(d2), g2 = gate * gate;
    if (a < g2 * (1.0 - 0x1p-40)) c.pass = 1;
    else if (a > g2 * (1.0 + 0x1p-40)) c.pass = 0;
    else c.pass = !(sqrt(a) > gate);
    c.w0 = vs0;
    c.w1 = vs1;
    c.d2 = d2;
    c.amb = AMB ? cand_amb(b, c, gate, eta) : 0;
}

// The storage precision of the gate (gate_eta): |ΔS_ab| <= eta·s_a·s_b with s_a = Σ_k |H_ak|·√P_kk
// (H0 = (0, 0, −1, 1, 0), H1 = (h10, h11, 0, h1l, 1) on rows 0, 1, 2, a, b), so to first order
// |Δd²| <= eta·(|w0|·s0 + |w1|·s1)², w = S⁻¹v (the roots in fp32, 2^-8 of slack)
__device__ __forceinline__ int cand_amb(const Block5& b, const Cand& c, double gate, double eta)
{
    auto rt = [](double x) { return (double)__builtin_amdgcn_sqrtf((float)fabs(x)); };
    const double s0 = rt(b.p22) + rt(b.daa);
    const double s1 = fabs(c.h10) * rt(b.p00) + fabs(c.h11) * rt(b.p11) + fabs(c.h1l) * rt(b.daa) + rt(b.dbb);
    const double wv = fabs(c.w0) * s0 + fabs(c.w1) * s1;
    return !c.singular && !(fabs(c.d2 - gate * gate) > eta * (1.0 + 0x1p-8) * wv * wv);
}

// Certified rejection: true only if the exact evaluation is guaranteed to fail the gate. It
// accepts sin/cos with |error| <= EPS (here the exact ones of sincos_near);
// the resulting error in S and v is bounded explicitly and d² = q/det is bounded from below by
// interval arithmetic. Requires a symmetric R and a determinant that is not tiny relative to
// |S00·S11| + |S01·S10| (so that the reference's LU-based d² is within 1e-9 of q/det).
__device__ __forceinline__ bool certified_reject(const Block5& b, double ma, double mr, double sn,
                                                 double cs, const double xp[3], double za, double zr,
                                                 const double Rm[4], double gate, double eta)
{
    if (!(fabs(ma) <= 8.0) || Rm[1] != Rm[2]) return false;
    const double EPS = 1e-5;
    const double h10 = -cs, h11 = -sn, h1l = xp[0] * sn - xp[1] * cs;
    double S[4], hp0[5], hp1[5];
    innovation_cov(b, h10, h11, h1l, Rm, S, hp0, hp1);
    const double v0 = innovation_angle(za, ma, xp[2]);
    const double v1 = zr - (mr - (xp[0] * cs + xp[1] * sn));
    const double ex = EPS * (fabs(xp[0]) + fabs(xp[1]));
    double Pm = fmax(fmax(fmax(fabs(b.p00), fabs(b.p01)), fmax(fabs(b.p02), fabs(b.p10))),
                     fmax(fmax(fabs(b.p11), fabs(b.p12)), fmax(fabs(b.p20), fabs(b.p21))));
    Pm = fmax(Pm, fmax(fmax(fmax(fabs(b.p22), fabs(b.p0a)), fmax(fabs(b.p1a), fabs(b.p2a))),
                       fmax(fmax(fabs(b.p0b), fabs(b.p1b)), fabs(b.p2b))));
    Pm = fmax(Pm, fmax(fmax(fabs(b.daa), fabs(b.dab)), fmax(fabs(b.dba), fabs(b.dbb))));
    const double dh = (2.0 * EPS + ex) * Pm;                   // |Δ hp1[b]|
    // + the storage precision of the gate (gate_eta)
    const double m0 = eta * 2.0 * (fabs(b.p22) + fabs(b.daa));
    const double m1 = eta * (2.0 + (fabs(h1l) + ex) * (fabs(h1l) + ex)) *
                      (fabs(b.p00) + fabs(b.p11) + fabs(b.p22) + fabs(b.daa) + fabs(b.dbb));
    const double dS00 = m0;
    const double dS01 = EPS * (fabs(hp0[0]) + fabs(hp0[1])) + ex * fabs(hp0[3]) + 0.5 * (m0 + m1);
    const double dS10 = 2.0 * dh + 0.5 * (m0 + m1);
    const double dS11 = dh * (3.0 + fabs(h1l) + ex) + EPS * (fabs(hp1[0]) + fabs(hp1[1])) +
                        ex * fabs(hp1[3]) + m1;
    const double dv1 = ex;
    const double q = v0 * v0 * S[3] - v0 * v1 * (S[1] + S[2]) + v1 * v1 * S[0];
    const double det = S[0] * S[3] - S[1] * S[2];
    const double mag_det = fabs(S[0] * S[3]) + fabs(S[1] * S[2]);
    const double mag_q = v0 * v0 * fabs(S[3]) + fabs(v0 * v1) * (fabs(S[1]) + fabs(S[2])) +
                         v1 * v1 * fabs(S[0]);
    const double av1 = fabs(v1) + dv1;
    const double dq = v0 * v0 * dS11 + fabs(v0) * av1 * (dS01 + dS10) +
                      fabs(v0) * dv1 * fabs(S[1] + S[2]) +
                      (2.0 * fabs(v1) * dv1 + dv1 * dv1) * fabs(S[0]) + av1 * av1 * dS00 + 1e-9 * mag_q;
    const double ddet = fabs(S[0]) * dS11 + fabs(S[3]) * dS00 + fabs(S[1]) * dS10 + fabs(S[2]) * dS01 +
                        dS01 * dS10 + dS00 * dS11 + 1e-9 * mag_det;
    const double det_lo = det - ddet;
    if (!(det_lo > 1e-6 * mag_det)) return false;              // also false for NaN / Inf
    return (q - dq) > gate * gate * (1.0 + 1e-6) * (det + ddet);
}

// Certified cheap rejection (the first filter of the per-line gate: ≈35 fp64 operations, no
// trigonometry). For a symmetric positive definite S, vᵀS⁻¹v ≥ v0²/S00 and vᵀS⁻¹v ≥ v1²/S11, so
// the exact evaluation fails the gate (Robot.cpp:489) if either one-dimensional bound exceeds it:
//  * S00 = H0·P5·H0ᵀ + R00 with the constant row H0 = (0, 0, −1, 1, 0): p22 − 2·p2a + daa + R00
//    (innovation_cov's S[0]); the reference's normalizeRadian (Robot.cpp:62-71) and the 2π fold
//    (:465-475) shift za − (ma − x_pre2) by multiples of 2π only, so |v0| ≥ its circular distance
//    to 0;
//  * S11 = H1·P5·H1ᵀ + R11 ≤ ‖H1‖²·tr(P5) + R11 with ‖H1‖² = 2 + h1l² ≤ 2 + (|x0| + |x1|)² (P5,
//    a principal block of a covariance, is positive semidefinite); v1 = zr − (mr − (x0·cos ma +
//    x1·sin ma)) bounded from below with the scan-start sin/cos of ma0 (|Δcos|, |Δsin| ≤ |ma − ma0|).
// It needs R symmetric with R00, R11 large against the storage rounding of P5 (which could
// otherwise make S indefinite: then it never rejects) and finite inputs (NaN never rejects).
// Margins: 1e-6 relative on the gate plus absolute slack, far above the rounding of the bounds
// and of the exact evaluation.
// s0, c0: sin/cos of ma0 within QR_TRIG_EPS (the fp32 __sincosf of (float)ma0 for |ma0| <= 8:
// argument rounding <= 8·2^-24 plus the instruction's own error, ≈1e-6 together).
constexpr double QR_TRIG_EPS = 4e-6;
__device__ __forceinline__ bool quick_reject(const Block5& b, double ma, double mr, double ma0, double s0,
                                             double c0, const double xp[3], double za, double zr,
                                             const double Rm[4], double gate, double eta)
{
    // every bound evaluated, the tests combined without branches (bitwise on bools): the same
    // values as the early-exit form, fewer exec-mask instructions on the per-line chain
    const double tr5 = b.p00 + b.p11 + b.p22 + b.daa + b.dbb;
    const double X = fabs(xp[0]) + fabs(xp[1]);
    const double H2 = 2.0 + X * X;   // ≥ ‖H1‖²
    const bool ok = (Rm[1] == Rm[2]) & (tr5 >= 0.0) & (Rm[0] > 1e-5 * 2.0 * tr5) & (Rm[3] > 1e-5 * H2 * tr5) &
                    (fabs(ma0) <= 8.0);
    const double g2 = gate * gate * (1.0 + 1e-6);
    // S00 + its storage precision (gate_eta): |Δ(p22 − 2·p2a + daa)| <= 2·eta·(|p22| + |daa|)
    const double S00 = b.p22 - 2.0 * b.p2a + b.daa + Rm[0] + 2.0 * eta * (fabs(b.p22) + fabs(b.daa));
    const double x = za - (ma - xp[2]);
    const double cd = fabs(x - 2.0 * EKF_PI * rint(x * (0.5 / EKF_PI)));
    const double a0 = cd - 1e-12 * (1.0 + fabs(x));
    const bool r0 = (S00 > 0.0) & (a0 > 0.0) & (a0 * a0 > g2 * S00);
    const double v1e = zr - (mr - (xp[0] * c0 + xp[1] * s0));
    const double a1 = fabs(v1e) - X * (fabs(ma - ma0) + QR_TRIG_EPS) - 1e-12 * (1.0 + fabs(zr) + fabs(mr) + X);
    const double S11u = H2 * tr5 * (1.0 + 1e-5 + eta) + Rm[3];
    const bool r1 = (a1 > 0.0) & (a1 * a1 > g2 * S11u);
    return ok & (r0 | r1);
}

// Certified rejection in fp32 (the second filter of the per-line gate; certified_reject in fp64
// and the exact evaluation run only where it cannot decide). Same bound structure as
// certified_reject, with the fp32 roundings added to it: every input rounded to fp32 (relative
// u = 2^-24), the short fp32 sums of S (≤ 12u of the sum of the absolute values of their terms,
// bounded through Pm and Hs = Σ|H row 1|), and q, det (16u of their magnitudes); sin/cos of the
// landmark angle from the fast fp32 path with EPS = 1e-4 allowed. v0 is the exact fp64 value of
// the evaluation (innovation_angle, no trigonometry), rounded once.
__device__ __forceinline__ bool certified_reject_f32(const Block5& b, double ma, double mr, const double xp[3],
                                                     double za, double zr, const double Rm[4], double gate,
                                                     double eta)
{
    if (!(fabs(ma) <= 8.0) || Rm[1] != Rm[2]) return false;
    constexpr float U = 5.9604645e-08f, EPS = 1e-4f;
    float sn, cs;
    __sincosf((float)ma, &sn, &cs);
    const float x0 = (float)xp[0], x1 = (float)xp[1];
    const float p00 = (float)b.p00, p01 = (float)b.p01, p02 = (float)b.p02;
    const float p10 = (float)b.p10, p11 = (float)b.p11, p12 = (float)b.p12;
    const float p20 = (float)b.p20, p21 = (float)b.p21, p22 = (float)b.p22;
    const float p0a = (float)b.p0a, p1a = (float)b.p1a, p2a = (float)b.p2a;
    const float p0b = (float)b.p0b, p1b = (float)b.p1b, p2b = (float)b.p2b;
    const float daa = (float)b.daa, dab = (float)b.dab, dba = (float)b.dba, dbb = (float)b.dbb;
    const float R0 = (float)Rm[0], R1 = (float)Rm[1], R2 = (float)Rm[2], R3 = (float)Rm[3];
    const float h10 = -cs, h11 = -sn, h1l = x0 * sn - x1 * cs;
    // S = H·P5·Hᵀ + R (innovation_cov's expressions)
    const float a0 = -p20 + p0a, a1 = -p21 + p1a, a2 = -p22 + p2a, a3 = -p2a + daa, a4 = -p2b + dab;
    const float c0 = h10 * p00 + h11 * p10 + h1l * p0a + p0b;
    const float c1 = h10 * p01 + h11 * p11 + h1l * p1a + p1b;
    const float c2 = h10 * p02 + h11 * p12 + h1l * p2a + p2b;
    const float c3 = h10 * p0a + h11 * p1a + h1l * daa + dba;
    const float c4 = h10 * p0b + h11 * p1b + h1l * dab + dbb;
    const float S0 = -a2 + a3 + R0;
    const float S1 = a0 * h10 + a1 * h11 + a3 * h1l + a4 + R1;
    const float S2 = -c2 + c3 + R2;
    const float S3 = c0 * h10 + c1 * h11 + c3 * h1l + c4 + R3;
    const float v0 = (float)innovation_angle(za, ma, xp[2]);
    const float v1 = (float)zr - ((float)mr - (x0 * cs + x1 * sn));
    const float ax = fabsf(x0) + fabsf(x1);
    const float ex = EPS * ax;
    float Pm = fmaxf(fmaxf(fmaxf(fabsf(p00), fabsf(p01)), fmaxf(fabsf(p02), fabsf(p10))),
                     fmaxf(fmaxf(fabsf(p11), fabsf(p12)), fmaxf(fabsf(p20), fabsf(p21))));
    Pm = fmaxf(Pm, fmaxf(fmaxf(fmaxf(fabsf(p22), fabsf(p0a)), fmaxf(fabsf(p1a), fabsf(p2a))),
                         fmaxf(fmaxf(fabsf(p0b), fabsf(p1b)), fabsf(p2b))));
    Pm = fmaxf(Pm, fmaxf(fmaxf(fabsf(daa), fabsf(dab)), fmaxf(fabsf(dba), fabsf(dbb))));
    const float Hs = 1.f + fabsf(h10) + fabsf(h11) + fabsf(h1l);
    const float dh = (2.f * EPS + ex) * Pm;
    // + the storage precision of the gate (gate_eta; |h1l| <= ax, 8u for these sums)
    const float fe = (float)eta * (1.f + 8.f * U);
    const float m0 = fe * 2.f * (fabsf(p22) + fabsf(daa));
    const float m1 = fe * (2.f + ax * ax) * (fabsf(p00) + fabsf(p11) + fabsf(p22) + fabsf(daa) + fabsf(dbb));
    const float dS00 = 12.f * U * (4.f * Pm + fabsf(R0)) + m0;
    const float dS01 = EPS * (fabsf(a0) + fabsf(a1)) + ex * fabsf(a3) + 12.f * U * (2.f * Hs * Pm + fabsf(R1)) +
                       0.5f * (m0 + m1);
    const float dS10 = 2.f * dh + 12.f * U * (2.f * Hs * Pm + fabsf(R2)) + 0.5f * (m0 + m1);
    const float dS11 = dh * (3.f + fabsf(h1l) + ex) + EPS * (fabsf(c0) + fabsf(c1)) + ex * fabsf(c3) +
                       12.f * U * (Hs * Hs * Pm + fabsf(R3)) + m1;
    const float dv1 = ex + 8.f * U * ((float)fabs(zr) + (float)fabs(mr) + ax);
    const float q = v0 * v0 * S3 - v0 * v1 * (S1 + S2) + v1 * v1 * S0;
    const float det = S0 * S3 - S1 * S2;
    const float mag_det = fabsf(S0 * S3) + fabsf(S1 * S2);
    const float mag_q = v0 * v0 * fabsf(S3) + fabsf(v0 * v1) * (fabsf(S1) + fabsf(S2)) + v1 * v1 * fabsf(S0);
    const float av1 = fabsf(v1) + dv1;
    const float dq = v0 * v0 * dS11 + fabsf(v0) * av1 * (dS01 + dS10) + fabsf(v0) * dv1 * fabsf(S1 + S2) +
                     (2.f * fabsf(v1) * dv1 + dv1 * dv1) * fabsf(S0) + av1 * av1 * dS00 + 16.f * U * mag_q + 1e-30f;
    const float ddet = fabsf(S0) * dS11 + fabsf(S3) * dS00 + fabsf(S1) * dS10 + fabsf(S2) * dS01 + dS01 * dS10 +
                       dS00 * dS11 + 16.f * U * mag_det + 1e-30f;
    const float det_lo = det - ddet;
    if (!(det_lo > 1e-4f * mag_det)) return false;              // also false for NaN / Inf
    const float g2 = (float)(gate * gate) * (1.f + 1e-4f);
    return (q - dq) > g2 * (det + ddet);
}

// Diagnostic phase timers (thread 0 of each workgroup; only when p.dbg is set).
#define EKF_STAMP(k)                                                            \
    do {                                                                        \
        if (dbg) {                                                              \
            const unsigned long long _t = __builtin_amdgcn_s_memrealtime();     \
            sh_stamp[k] += _t - t_last;                                         \
            t_last = _t;                                                        \
        }                                                                       \
    } while (0)

constexpr int EKF_NSTAMP = 32;   // diagnostic phase-timer slots per instance (EKF_SCAN_STAMPS=1)
constexpr int HIST_LDS = 8;   // matches per scan whose owned U rows stay in LDS
constexpr int HIST_V = 4;     // ... and whose V rows do (sequential path; the rest in Vst)

__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    return v;
}

// The status bits a speculative line can raise (GSL_EDOM, the gate's precision margin, the
// as-written R), three per line (line i at bits 3i .. 3i + 2 of one word, SPEC_L = 8 lines), so that
// a restart after a failed verdict keeps those of the lines before the first violating one
__device__ __forceinline__ int st_line(int st, int i)
{
    return (((st & EKF_ST_SINGULAR) ? 1 : 0) | ((st & EKF_ST_PRECISION_BIT) ? 2 : 0) | ((st & EKF_ST_NSYM) ? 4 : 0))
           << (3 * i);
}
__device__ __forceinline__ int st_lines(int packed, int upto)   // the bits of lines < upto
{
    const int w = upto >= 8 ? packed : packed & ((1 << (3 * upto)) - 1);
    return ((w & 0x249249) ? (int)EKF_ST_SINGULAR : 0) | ((w & 0x492492) ? (int)EKF_ST_PRECISION_BIT : 0) |
           ((w & 0x924924) ? (int)EKF_ST_NSYM : 0);
}

// ---------------------------------------------------------------------------------------
// 1. association + gain chain + augmentation: ⌈N/256⌉ cooperating workgroups per instance
// ---------------------------------------------------------------------------------------
// Thread (g, tid) of instance e OWNS landmark j = 256·g + tid: its gating candidate, its two
// rows of W/K/U/y, its robot-strip columns and its 2×2 diagonal block, all kept in registers
// for the whole scan. The robot 3×3 block and x_pre are uniform and recomputed identically by
// every thread. The instance's workgroups exchange words through a mailbox (one slot per
// workgroup and parity), written with 8-byte agent-scope atomic stores, drained by s_waitcnt
// and a workgroup barrier before a data-tagged word (launch epoch, phase code, payload) that
// the readers poll (MI355X_MICROARCH.md "Valid forms"). Every spin is bounded; a timeout sets a
// status bit.
__device__ __forceinline__ void mb_store(double* p, double v)
{
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ double mb_load(const double* p)
{
    return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// mailbox slot words (the package words double as the LDS package layout)
enum { MB_BEST = 0, MB_S = 1, MB_SI = 5, MB_V = 9, MB_H = 11, MB_KR = 14, MB_UR = 20, MB_VH = 26 };

// tag word: bits 63..32 launch epoch, 31..24 phase code, 23..0 payload. Codes 1..64 are the
// lines of the sequential association; the speculative exchanges use their own codes.
enum { TAG_SPEC_LISTS = 0x81, TAG_SPEC_WINNERS = 0x82, TAG_SPEC_VERDICT = 0x83 };

__device__ __forceinline__ void mb_tag(double* slot, unsigned epoch, unsigned code, unsigned payload)
{
    const unsigned long long want = ((unsigned long long)epoch << 8) | code;
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(slot + MB_BEST), (want << 24) | payload,
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Thread k < G polls workgroup k's tag of the given parity until it carries (epoch, code);
// returns its payload (-1 on timeout, with the status bit set).
// Every wait gives up after 2^spin polls (≈0.5 s at 24) and sets the timeout bit; a thread whose
// status already holds it does not wait again (the launch is rolled back anyway).
__device__ __forceinline__ int mb_poll(const double* mbox, int par, int G, int k, int mbw,
                                       unsigned epoch, unsigned code, int& status, int spin)
{
    const unsigned long long want = ((unsigned long long)epoch << 8) | code;
    const unsigned long long* tw =
        reinterpret_cast<const unsigned long long*>(mbox + ((size_t)par * G + k) * mbw + MB_BEST);
    unsigned long long v = __hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int polls = 0;
    while ((v >> 24) != want) {
        __builtin_amdgcn_s_sleep(1);
        if ((status & EKF_ST_TIMEOUT_BIT) || ++polls > (1 << spin)) {   // a workgroup never arrived
            status |= EKF_ST_TIMEOUT_BIT;
            return -1;
        }
        v = __hip_atomic_load(tw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return (int)(v & 0xffffffu);
}

// Speculative list words carry their own tag: bits 63..40 the launch epoch (mod 2^24), bits
// 39..0 the payload, written with one 8-byte atomic store, so a reader needs one poll of the word
// itself (no separate tag word and second load). They live in the last 16 words of each
// workgroup's parity-0 mailbox slot (MB_LIST_BACK), which nothing else writes, and every
// speculative launch rewrites all SPEC_L of them.
constexpr int LIST_TAG_SHIFT = 40;
constexpr int MB_LIST_BACK = 16;

__device__ __forceinline__ void mb_store_tagged(double* p, unsigned epoch, unsigned long long payload)
{
    const unsigned long long w = ((unsigned long long)(epoch & 0xffffffu) << LIST_TAG_SHIFT) | payload;
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ unsigned long long mb_wait_tagged(const double* p, unsigned epoch, int& status, int spin)
{
    const unsigned long long* w = reinterpret_cast<const unsigned long long*>(p);
    const unsigned long long want = epoch & 0xffffffu;
    unsigned long long v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    int polls = 0;
    while ((v >> LIST_TAG_SHIFT) != want) {
        __builtin_amdgcn_s_sleep(1);
        if ((status & EKF_ST_TIMEOUT_BIT) || ++polls > (1 << spin)) {
            status |= EKF_ST_TIMEOUT_BIT;
            return 0;
        }
        v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return v & ((1ull << LIST_TAG_SHIFT) - 1);
}

// End of a launch (rollback protocol). Every workgroup has written its owned columns of the
// robot strip and mean into the inactive copy; it publishes its completion word (done_word) after
// its loads and stores have returned. The lead (workgroup 0, thread 0) waits for the other G − 1
// words of this epoch, bounded, and returns commit_status over all G: the launch commits (the lead
// flips cur[e] and writes the shared state) only if no timeout is in it. The shared inputs every
// workgroup read at its start (pose, saved, x_pre) are rewritten only after every word arrived,
// i.e. after every workgroup has finished reading them.
__device__ __forceinline__ void publish_done(int* sync, int g, unsigned epoch, int st)
{
    __hip_atomic_store(reinterpret_cast<unsigned*>(&sync[SYNC_WG0 + g]), done_word(epoch, st),
                       __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Run by every thread of workgroup 0 (the words are polled in parallel, thread k word k); the
// folded status of all G words (= commit_status) is returned to every thread.
template <int BLK>   // the workgroup's threads
__device__ __forceinline__ int lead_collect(int* sync, int G, unsigned epoch, int own_status, int spin,
                                            int tid, int* sh_red, int& zg)
{
    // zg: 1 + the highest workgroup whose word carries DONE_NZ (0: none)
    int st = tid == 0 ? commit_fold(0, done_word(epoch, own_status), epoch) : 0;
    int z = (tid == 0 && (own_status & (int)DONE_NZ)) ? 1 : 0;
    const bool late0 = (own_status & EKF_ST_TIMEOUT_BIT) != 0;
    for (int k = 1 + tid; k < G; k += BLK) {
        const unsigned* w = reinterpret_cast<const unsigned*>(&sync[SYNC_WG0 + k]);
        unsigned v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int polls = 0;
        bool late = late0;
        while ((v >> 8) != (epoch & 0xffffffu) && !late) {
            __builtin_amdgcn_s_sleep(1);
            if (++polls > (1 << spin)) late = true;
            v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        st = commit_fold(st, v, epoch);
        if ((v >> 8) == (epoch & 0xffffffu) && (v & DONE_NZ)) z = max(z, k + 1);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) {
        st |= __shfl_xor(st, off, 64);
        z = max(z, __shfl_xor(z, off, 64));
    }
    __syncthreads();
    if ((tid & 63) == 0) sh_red[tid >> 6] = st | (z << 8);
    __syncthreads();
    st = 0;
    z = 0;
#pragma unroll
    for (int w = 0; w < BLK / 64; w++) {
        st |= sh_red[w] & 0xff;
        z = max(z, sh_red[w] >> 8);
    }
    zg = z;
    return st;
}

// rows 0..2 of Fx·P for one landmark's robot-strip columns (Robot.cpp:242)
__device__ __forceinline__ void predict_cols(const double F3[9], double2& rr0, double2& rr1, double2& rr2)
{
    const double2 a0 = rr0, a1 = rr1, a2 = rr2;
    rr0.x = F3[0] * a0.x + F3[1] * a1.x + F3[2] * a2.x;
    rr0.y = F3[0] * a0.y + F3[1] * a1.y + F3[2] * a2.y;
    rr1.x = F3[3] * a0.x + F3[4] * a1.x + F3[5] * a2.x;
    rr1.y = F3[3] * a0.y + F3[4] * a1.y + F3[5] * a2.y;
    rr2.x = F3[6] * a0.x + F3[7] * a1.x + F3[8] * a2.x;
    rr2.y = F3[6] * a0.y + F3[7] * a1.y + F3[8] * a2.y;
}

// R of a line (Robot.cpp:302-304): r_mode 1 reproduces the reference as written (only the
// first four lines' R[3] lands in a zero-initialised 2×2)
__device__ __forceinline__ void line_R(const ekf_line& ln, int i, int r_mode, double Rm[4])
{
    if (r_mode == 1) {
        Rm[0] = i == 0 ? ln.R[3] : 0.0;
        Rm[1] = i == 1 ? ln.R[3] : 0.0;
        Rm[2] = i == 2 ? ln.R[3] : 0.0;
        Rm[3] = i == 3 ? ln.R[3] : 0.0;
    } else {
        Rm[0] = ln.R[0]; Rm[1] = ln.R[1]; Rm[2] = ln.R[2]; Rm[3] = ln.R[3];
    }
}

__device__ __forceinline__ void fill_block5(Block5& b5, const double R33[9], double2 rr0, double2 rr1,
                                            double2 rr2, const double Dj[4])
{
    b5.p00 = R33[0]; b5.p01 = R33[1]; b5.p02 = R33[2];
    b5.p10 = R33[3]; b5.p11 = R33[4]; b5.p12 = R33[5];
    b5.p20 = R33[6]; b5.p21 = R33[7]; b5.p22 = R33[8];
    b5.p0a = rr0.x; b5.p0b = rr0.y;
    b5.p1a = rr1.x; b5.p1b = rr1.y;
    b5.p2a = rr2.x; b5.p2b = rr2.y;
    b5.daa = Dj[0]; b5.dab = Dj[1]; b5.dba = Dj[2]; b5.dbb = Dj[3];
}

// Symmetric downdate operands (fp32 operand storage, every mode but the reference's asymmetric
// R): the landmark block's share of P −= K·S·Kᵀ (Robot.cpp:560-568) is stored as U·Vᵀ with
// V = K·F and U = −2^x·V (x the fp16 storage exponent, else 0), F·Fᵀ = S: the lower Cholesky
// factor of the symmetrised S, in fp32 like the operands themselves (a non-positive pivot
// contributes 0, which happens only where S is singular and K = 0). Every stored element then
// gets the same products whichever orientation is stored (staged_blocks). The scan's own fp64
// chain (gain_rows: W, K, y, the eager robot-strip and diagonal-block downdates, the corrections
// of later lines) keeps K·S·Kᵀ; only the stored operands take this form.
__device__ __forceinline__ void sym_factor_S(const double S[4], float F[3])
{
    const float a = (float)S[0], b = 0.5f * ((float)S[1] + (float)S[2]);
    const float c = (float)S[3];
    // v_rsq_f32 (1 ulp): F need not be correctly rounded, only the same on every thread
    F[0] = F[1] = F[2] = 0.f;
    if (a > 0.f) {
        const float ra = __builtin_amdgcn_rsqf(a);
        F[0] = a * ra;
        F[1] = b * ra;
        const float dd = c - F[1] * F[1];
        F[2] = dd > 0.f ? dd * __builtin_amdgcn_rsqf(dd) : 0.f;
    } else {
        F[2] = c > 0.f ? c * __builtin_amdgcn_rsqf(c) : 0.f;
    }
}

__device__ __forceinline__ void sym_factor(const double* pk, float F[3])
{
    const double S[4] = {pk[MB_S], pk[MB_S + 1], pk[MB_S + 2], pk[MB_S + 3]};
    sym_factor_S(S, F);
}

// The uniform gain package of a match from the matching landmark's state: S, S⁻¹, v, H row 1
// and the robot rows of K = W·S⁻¹ and U = K·S (Robot.cpp:522-602 for rows 0..2).
__device__ __forceinline__ void build_package(const Cand& c, const double R33[9], double2 rr0,
                                              double2 rr1, double2 rr2, double* pk)
{
    const double RL0[3] = {rr0.x, rr1.x, rr2.x};
    const double RL1[3] = {rr0.y, rr1.y, rr2.y};
    pk[MB_S + 0] = c.S[0]; pk[MB_S + 1] = c.S[1];
    pk[MB_S + 2] = c.S[2]; pk[MB_S + 3] = c.S[3];
    pk[MB_SI + 0] = c.Si[0]; pk[MB_SI + 1] = c.Si[1];
    pk[MB_SI + 2] = c.Si[2]; pk[MB_SI + 3] = c.Si[3];
    pk[MB_V + 0] = c.v[0]; pk[MB_V + 1] = c.v[1];
    pk[MB_H + 0] = c.h10; pk[MB_H + 1] = c.h11; pk[MB_H + 2] = c.h1l;
#pragma unroll
    for (int a = 0; a < 3; a++) {
        // W = P·Hᵀ (Robot.cpp:522), K = W·S⁻¹ (:526), U = K·S (:560)
        const double w0 = -R33[a * 3 + 2] + RL0[a];
        const double w1 = c.h10 * R33[a * 3 + 0] + c.h11 * R33[a * 3 + 1] + c.h1l * RL0[a] + RL1[a];
        const double k0 = w0 * c.Si[0] + w1 * c.Si[2];
        const double k1 = w0 * c.Si[1] + w1 * c.Si[3];
        pk[MB_KR + 2 * a] = k0;
        pk[MB_KR + 2 * a + 1] = k1;
        pk[MB_UR + 2 * a] = k0 * c.S[0] + k1 * c.S[2];
        pk[MB_UR + 2 * a + 1] = k0 * c.S[1] + k1 * c.S[3];
    }
}

// The two rows of one landmark for a match: its block of column jstar with the earlier matches
// of the scan applied (Robot.cpp:560-568, in order), W = P·Hᵀ, K = W·S⁻¹, U = K·S, y += K·v
// (Robot.cpp:522-589), and the eager downdate of its robot-strip columns and diagonal block.
// `uq_of(q)` / `vq_of(q)` return the landmark's U rows and jstar's V rows of the scan's match q.
// MAXQ > 0: at most MAXQ earlier matches (the speculative path). (Applying all MAXQ rows
// branch-free on zeroed rows measured slower: DESIGN.md §10.)
// One earlier match q's correction of a landmark's block of a later match's column (Robot.cpp:560-568
// in order): blk −= U_q(own rows)·V_q(column rows)ᵀ, four independent fused chains. Every path that
// corrects a block (gain_rows, all at once; the speculative landmark waves, one match at a time)
// runs this sequence per element, so they agree bit for bit.
__device__ __forceinline__ void correct_block(double blk[4], const double4& uq, const double4& vh)
{
    blk[0] = fma(-uq.x, vh.x, blk[0]);
    blk[1] = fma(-uq.x, vh.z, blk[1]);
    blk[2] = fma(-uq.z, vh.x, blk[2]);
    blk[3] = fma(-uq.z, vh.z, blk[3]);
    blk[0] = fma(-uq.y, vh.y, blk[0]);
    blk[1] = fma(-uq.y, vh.w, blk[1]);
    blk[2] = fma(-uq.w, vh.y, blk[2]);
    blk[3] = fma(-uq.w, vh.w, blk[3]);
}

// The package words the landmark rows of a match read (Robot.cpp:522-589): S, S⁻¹, v, H row 1 and
// the robot rows of U = K·S
struct PkCore {
    double S[4], Si[4], v[2], h[3], Ur[6];
};
__device__ __forceinline__ void gain_core(const PkCore& P, const double blk[4], double2& rr0, double2& rr1,
                                          double2& rr2, double2& yb, double Dj[4], double kk[4], double uu[4]);

template <int MAXQ, typename UQ, typename VQ>
__device__ __forceinline__ void gain_rows(const double* pk, int t, UQ uq_of, VQ vq_of, double blk[4],
                                          double2& rr0, double2& rr1, double2& rr2, double2& yb,
                                          double Dj[4], double kk[4], double uu[4])
{
    // earlier matches of this scan, in order: four independent fused chains (one per entry), the
    // rows of match q + 1 loaded before match q's products (LDS latency off the chain). t is the
    // scan's match count, the same on every lane: a scalar loop
    auto correct = [&](const double4& uq, const double4& vh) __attribute__((always_inline)) {
        correct_block(blk, uq, vh);
    };
    // matches in pairs (both pairs' rows loaded together: one LDS round trip per two matches),
    // then the odd one; the products in q order either way
    const int tu = __builtin_amdgcn_readfirstlane(MAXQ > 0 ? min(t, MAXQ) : t);
    int q = 0;
#pragma unroll 1
    for (; q + 1 < tu; q += 2) {
        const double4 ua = uq_of(q), va = vq_of(q);
        const double4 ub = uq_of(q + 1), vb = vq_of(q + 1);
        correct(ua, va);
        correct(ub, vb);
    }
    if (q < tu) correct(uq_of(q), vq_of(q));
    PkCore P;
#pragma unroll
    for (int a = 0; a < 4; a++) {
        P.S[a] = pk[MB_S + a];
        P.Si[a] = pk[MB_SI + a];
    }
    P.v[0] = pk[MB_V];
    P.v[1] = pk[MB_V + 1];
    P.h[0] = pk[MB_H];
    P.h[1] = pk[MB_H + 1];
    P.h[2] = pk[MB_H + 2];
#pragma unroll
    for (int a = 0; a < 6; a++) P.Ur[a] = pk[MB_UR + a];
    gain_core(P, blk, rr0, rr1, rr2, yb, Dj, kk, uu);
}

// The gain rows from the corrected block (gain_rows without the earlier matches' corrections),
// the package's words in registers: every path computes them with this one expression set
__device__ __forceinline__ void gain_core(const PkCore& P, const double blk[4], double2& rr0, double2& rr1,
                                          double2& rr2, double2& yb, double Dj[4], double kk[4], double uu[4])
{
    const double S0 = P.S[0], S1 = P.S[1], S2 = P.S[2], S3 = P.S[3];
    const double Si0 = P.Si[0], Si1 = P.Si[1], Si2 = P.Si[2], Si3 = P.Si[3];
    const double v0 = P.v[0], v1 = P.v[1];
    const double h10 = P.h[0], h11 = P.h[1], h1l = P.h[2];
#pragma unroll
    for (int pp = 0; pp < 2; pp++) {
        const double pb0 = pp ? rr0.y : rr0.x;
        const double pb1 = pp ? rr1.y : rr1.x;
        const double pb2 = pp ? rr2.y : rr2.x;
        const double pba = blk[pp * 2 + 0], pbb = blk[pp * 2 + 1];
        const double w0 = -pb2 + pba;
        const double w1 = h10 * pb0 + h11 * pb1 + h1l * pba + pbb;
        const double k0 = w0 * Si0 + w1 * Si2;
        const double k1 = w0 * Si1 + w1 * Si3;
        kk[2 * pp] = k0;
        kk[2 * pp + 1] = k1;
        uu[2 * pp] = k0 * S0 + k1 * S2;
        uu[2 * pp + 1] = k0 * S1 + k1 * S3;
        const double dyv = k0 * v0 + k1 * v1;   // y += K·v (Robot.cpp:585-589)
        if (pp) yb.y += dyv; else yb.x += dyv;
    }
    const double* Ur = P.Ur;
    // eager downdate of the robot-strip columns and the diagonal block (Robot.cpp:568)
    rr0.x -= Ur[0] * kk[0] + Ur[1] * kk[1];
    rr0.y -= Ur[0] * kk[2] + Ur[1] * kk[3];
    rr1.x -= Ur[2] * kk[0] + Ur[3] * kk[1];
    rr1.y -= Ur[2] * kk[2] + Ur[3] * kk[3];
    rr2.x -= Ur[4] * kk[0] + Ur[5] * kk[1];
    rr2.y -= Ur[4] * kk[2] + Ur[5] * kk[3];
    Dj[0] -= uu[0] * kk[0] + uu[1] * kk[1];
    Dj[1] -= uu[0] * kk[2] + uu[1] * kk[3];
    Dj[2] -= uu[2] * kk[0] + uu[3] * kk[1];
    Dj[3] -= uu[2] * kk[2] + uu[3] * kk[3];
}

// uniform: robot 3×3 block and x_pre = y[0..2] after a match (Robot.cpp:568, 579-602)
__device__ __forceinline__ void robot_update(double R33[9], double xp[3], const double* pk)
{
    double Kr[6], Ur[6];
#pragma unroll
    for (int q = 0; q < 6; q++) {
        Kr[q] = pk[MB_KR + q];
        Ur[q] = pk[MB_UR + q];
    }
    const double v0 = pk[MB_V], v1 = pk[MB_V + 1];
    double yn[3];
#pragma unroll
    for (int a = 0; a < 3; a++) {
        yn[a] = xp[a] + (Kr[2 * a] * v0 + Kr[2 * a + 1] * v1);
#pragma unroll
        for (int cc = 0; cc < 3; cc++)
            R33[a * 3 + cc] -= Ur[2 * a] * Kr[2 * cc] + Ur[2 * a + 1] * Kr[2 * cc + 1];
    }
    xp[0] = yn[0];
    xp[1] = yn[1];
    xp[2] = normalize_radian(yn[2]);   // Robot.cpp:596
}

// Cheap guess of the exact gate (fp32 sine/cosine, no error bounds). It only steers the
// speculative association; every decision it feeds is re-checked exactly. The landmark's part
// (predicted measurement, H·P·Hᵀ) does not depend on the line and is computed once.
struct Guess {
    float h0, h1, S[4];
};

__device__ __forceinline__ void guess_prep(const Block5& b, double ma, double mr, const double xp[3],
                                           Guess& gs)
{
    float sf, cf;
    __sincosf((float)ma, &sf, &cf);
    const float x0 = (float)xp[0], x1 = (float)xp[1];
    const float h10 = -cf, h11 = -sf, h1l = x0 * sf - x1 * cf;
    const float p00 = (float)b.p00, p01 = (float)b.p01, p02 = (float)b.p02;
    const float p10 = (float)b.p10, p11 = (float)b.p11, p12 = (float)b.p12;
    const float p20 = (float)b.p20, p21 = (float)b.p21, p22 = (float)b.p22;
    const float p0a = (float)b.p0a, p1a = (float)b.p1a, p2a = (float)b.p2a;
    const float p0b = (float)b.p0b, p1b = (float)b.p1b, p2b = (float)b.p2b;
    const float daa = (float)b.daa, dab = (float)b.dab, dba = (float)b.dba, dbb = (float)b.dbb;
    const float a0 = -p20 + p0a, a1 = -p21 + p1a, a2 = -p22 + p2a, a3 = -p2a + daa, a4 = -p2b + dab;
    const float c0 = h10 * p00 + h11 * p10 + h1l * p0a + p0b;
    const float c1 = h10 * p01 + h11 * p11 + h1l * p1a + p1b;
    const float c2 = h10 * p02 + h11 * p12 + h1l * p2a + p2b;
    const float c3 = h10 * p0a + h11 * p1a + h1l * daa + dba;
    const float c4 = h10 * p0b + h11 * p1b + h1l * dab + dbb;
    gs.S[0] = -a2 + a3;
    gs.S[1] = a0 * h10 + a1 * h11 + a3 * h1l + a4;
    gs.S[2] = -c2 + c3;
    gs.S[3] = c0 * h10 + c1 * h11 + c3 * h1l + c4;
    gs.h0 = (float)normalize_radian(ma - xp[2]);
    gs.h1 = (float)mr - (x0 * cf + x1 * sf);
}

__device__ __forceinline__ bool guess_pass(const Guess& gs, double za, double zr, const double Rm[4],
                                           double gate)
{
    constexpr float TWO_PI = 6.283185307179586f;
    float v0 = (float)za - gs.h0;
    if (fabsf(v0 - TWO_PI) < fabsf(v0)) v0 -= TWO_PI;
    else if (fabsf(v0 + TWO_PI) < fabsf(v0)) v0 += TWO_PI;
    const float v1 = (float)zr - gs.h1;
    const float S0 = gs.S[0] + (float)Rm[0], S1 = gs.S[1] + (float)Rm[1];
    const float S2 = gs.S[2] + (float)Rm[2], S3 = gs.S[3] + (float)Rm[3];
    const float q = v0 * v0 * S3 - v0 * v1 * (S1 + S2) + v1 * v1 * S0;
    const float det = S0 * S3 - S1 * S2;
    return !(det > 0.f) || q <= (float)(gate * gate) * det;
}

constexpr int SPEC_L = HIST_LDS;                    // lines
// guessed candidates per line per workgroup: with SPEC_K = SPEC_L every line's guess can be
// resolved (line t needs its first t + 1 candidates at most: only t earlier lines can take one)
constexpr int SPEC_K = 8;
// list words per (workgroup, line): A = local indices 0..3 (8 bits each), the count (bits 32..35)
// and a more bit (36); B = local indices 4..7, written and read only when the count exceeds 4
constexpr int LW_CNT = 32, LW_MORE = 36;
constexpr int SPEC_PB = 2;                          // guessed columns per pass over the pending steps
#ifndef EKF_SPEC_PB64
#define EKF_SPEC_PB64 4
#endif
constexpr int SPEC_PB64 = EKF_SPEC_PB64;            // ... fp64 operands (pll_shared_step: owned rows once per pass)
#ifndef EKF_STAGED_DEPTH
#define EKF_STAGED_DEPTH 1
#endif
constexpr int SPEC_QMAX = 16;                       // pending steps staged in LDS (T = 16: up to 15)
constexpr int SPEC_WD = 14 + 4 * (SPEC_L - 1);      // winner record: rr, Dj, y, sin/cos, column blocks
// speculative package: the words of build_package, then the robot 3×3 block and x_pre after the
// line's update (robot_update), computed once by the replay wave for every landmark wave
constexpr int PK_R33 = MB_VH, PK_XP = MB_VH + 9, PK_F = MB_VH + 12;   // + the symmetric factor (sym_factor)
// 1.0 if the guessed winner passed its exact gate; 0.0: it failed, the line is unmatched unless
// another landmark passes (which the landmark waves flag), and the other words are not written
constexpr int PK_OK = MB_VH + 15;
constexpr int PKW = MB_VH + 16;                     // package words (speculative lines; V rows in sh_wh)

// Blocks (j, cols[t]) for t < SPEC_L and (j, j) (last; only if `diag`) of the landmark block
// with the pending steps applied, fp32 operands, every pending step with ks <= 8: the guessed
// columns' operand rows come from LDS (stg[t][q][U|V][row half][8], staged by the workgroup),
// the owned rows are loaded once per step (the next step's while this one runs). Per element
// the same chain as pll_blocks, kept in the requested orientation: a block stored transposed
// (its column's tile row first) evolves as fma(X_col·V_own) terms, which equal the owned-first
// products bit for bit (fma(a, b, c) == fma(b, a, c)), so every block runs one pattern on
// O = owned U (or owned V when transposed) and X = staged V (or staged U). Every k-step runs:
// past a step's matches the operands hold −0 (U) and +0 (V), whose products leave a chain as it
// is (x + (−0) == x).
// The stored blocks of staged_blocks, in the requested orientation (issued early: their loads
// share a memory round trip with the staging of the guessed columns' rows).
template <typename T>
__device__ __forceinline__ void staged_blocks_load(const PllView<T>& v, int j, const int (&cols)[8],
                                                   typename Stor<T>::C (&r)[9][4])
{
    using C = typename Stor<T>::C;
    const int i0 = 2 * j;
#pragma unroll
    for (int b = 0; b < 9; b++) {
        const int jb = 2 * (b < 8 ? cols[b] : j);
        const bool swap = (i0 >> 5) > (jb >> 5);
        C a[4];
        load_block<T>(v, swap ? jb : i0, swap ? i0 : jb, a);
        r[b][0] = a[0]; r[b][1] = swap ? a[2] : a[1];
        r[b][2] = swap ? a[1] : a[2]; r[b][3] = a[3];
    }
}

template <typename T>
__device__ __forceinline__ void staged_blocks(const PllView<T>& v, int j, const int (&cols)[8],
                                              const float* stg, typename Stor<T>::C (&r)[9][4],
                                              double (&out)[9][4])
{
    using C = typename Stor<T>::C;
    constexpr int NB = 9;
    const int i0 = 2 * j;
    bool swap[NB];
    int jb[NB];
#pragma unroll
    for (int b = 0; b < NB; b++) {
        jb[b] = 2 * (b < 8 ? cols[b] : j);
        swap[b] = (i0 >> 5) > (jb[b] >> 5);
    }
    const int kh = v.kmax / 2;
    // owned rows i0, i0+1 of U_q: [row half][2 × 4 k]. Symmetric operands (U = −2^x·V, x the
    // fp16 storage exponent, 0 otherwise: gain_rows) make every block's chain one pattern on the
    // owned U rows and the column's V rows, whatever the stored orientation: a block stored
    // transposed evolves as fma(V_own, U_col) terms, and V_own·U_col == U_own·V_col exactly
    // (power-of-two scaling; fma(a, b, c) == fma(b, a, c)).
    auto load_rows = [&](int q, f32x4v (&Ux)[4][2]) {
        const Slot& sq = v.pend[q];
        const float* ou = u_rows_f32(v, sq) + ((size_t)(i0 >> 5) * 64 + (i0 & 31)) * kh;
#pragma unroll
        for (int rh = 0; rh < 4; rh++) {
            const int roff = (rh & 1) * kh + (rh >> 1) * 32 * kh;
#pragma unroll
            for (int h = 0; h < 2; h++) Ux[rh][h] = *reinterpret_cast<const f32x4v*>(ou + roff + 4 * h) * v.us;
        }
    };
    const float vscale = -ldexpf(1.0f, -v.ex);   // V_own = U_own · (−2^−x), exact
    // one pending step on the nine blocks, with that step's owned rows
    auto apply_step = [&](int q, const f32x4v (&U)[4][2]) __attribute__((always_inline)) {
        const Slot& sq = v.pend[q];
        const int4 cw = v.ctl[q];
        if (cw.x) {
#pragma unroll
            for (int b = 0; b < NB; b++) r[b][0] = r[b][1] = r[b][2] = r[b][3] = (C)0;
        } else if (cw.y > 0 || cw.z > 0) {   // (ks = 0: no match, or a rolled-back step: nothing to apply)
            // staged V rows of column b, interleaved by row pair (stage_v_index; block b + 1's
            // read from LDS while block b computes); the diagonal block's are the owned V rows
            auto read_x = [&](int b, f32x4v (&X)[2][4]) __attribute__((always_inline)) {
                const float* xs = stg + (((b * SPEC_QMAX + q) * 2 + 1) * 4) * 8;
#pragma unroll
                for (int pr = 0; pr < 2; pr++)
#pragma unroll
                    for (int kc = 0; kc < 4; kc++) X[pr][kc] = *reinterpret_cast<const f32x4v*>(xs + pr * 16 + 4 * kc);
            };
            f32x4v Xa[2][4], Xb[2][4];
            read_x(0, Xa);
#pragma unroll
            for (int b = 0; b < NB; b++) {
                f32x4v (&Xc)[2][4] = (b & 1) ? Xb : Xa;
                f32x4v (&Xn)[2][4] = (b & 1) ? Xa : Xb;
                if (b + 1 < 8) read_x(b + 1, Xn);
                f32x2v r01 = {(float)r[b][0], (float)r[b][1]}, r23 = {(float)r[b][2], (float)r[b][3]};   // fp32 operands only
#pragma unroll
                for (int kp = 0; kp < 8; kp++) {
                    const int h = kp >> 2, s4 = kp & 3;
                    f32x2v x01, x23;   // (column row 0, row 1) at k-pair kp, even and odd k
                    if (b < 8) {
                        x01 = f32x2v{Xc[0][kp >> 1][2 * (kp & 1)], Xc[0][kp >> 1][2 * (kp & 1) + 1]};
                        x23 = f32x2v{Xc[1][kp >> 1][2 * (kp & 1)], Xc[1][kp >> 1][2 * (kp & 1) + 1]};
                    } else {
                        x01 = f32x2v{U[0][h][s4], U[1][h][s4]} * vscale;
                        x23 = f32x2v{U[2][h][s4], U[3][h][s4]} * vscale;
                    }
                    r01 = __builtin_elementwise_fma(f32x2v{U[0][h][s4], U[0][h][s4]}, x01, r01);
                    r01 = __builtin_elementwise_fma(f32x2v{U[2][h][s4], U[2][h][s4]}, x23, r01);
                    r23 = __builtin_elementwise_fma(f32x2v{U[1][h][s4], U[1][h][s4]}, x01, r23);
                    r23 = __builtin_elementwise_fma(f32x2v{U[3][h][s4], U[3][h][s4]}, x23, r23);
                }
                r[b][0] = vround<T>(v, r01[0]); r[b][1] = vround<T>(v, r01[1]);
                r[b][2] = vround<T>(v, r23[0]); r[b][3] = vround<T>(v, r23[1]);
                // one block at a time (bounds the staged rows in registers)
                __builtin_amdgcn_sched_barrier(0);
            }
            if (cw.z > 0) {
#pragma unroll
                for (int b = 0; b < NB; b++) {
                    C a[4] = {r[b][0], swap[b] ? r[b][2] : r[b][1], swap[b] ? r[b][1] : r[b][2], r[b][3]};
                    patch_block<T>(v, sq, cw, i0, jb[b], swap[b], a);
                    r[b][0] = a[0]; r[b][1] = swap[b] ? a[2] : a[1];
                    r[b][2] = swap[b] ? a[1] : a[2]; r[b][3] = a[3];
                }
            }
        }
    };
    // The next step's rows are loaded while this one runs. The loads are issued on every
    // iteration (the last one re-reads its own step): a conditional prefetch makes the compiler's
    // wait-count merge at the loop join wait for ALL outstanding loads (vmcnt(0)) before the
    // body, which serialised every step behind its successor's loads.
    const int np = v.npend;
#if EKF_STAGED_DEPTH >= 2
    // two steps ahead: three register sets, the loop unrolled by three (static names)
    f32x4v UA[4][2], UB[4][2], UC[4][2];
    if (np > 0) {
        load_rows(0, UA);
        load_rows(min(1, np - 1), UB);
        for (int q = 0; q < np; q += 3) {
            load_rows(min(q + 2, np - 1), UC);
            apply_step(q, UA);
            if (q + 1 >= np) break;
            load_rows(min(q + 3, np - 1), UA);
            apply_step(q + 1, UB);
            if (q + 2 >= np) break;
            load_rows(min(q + 4, np - 1), UB);
            apply_step(q + 2, UC);
        }
    }
#else
    // one step ahead: two register sets, the loop unrolled by two (static names, no copies)
    f32x4v UA[4][2], UB[4][2];
    if (np > 0) {
        load_rows(0, UA);
        for (int q = 0; q < np; q += 2) {
            load_rows(min(q + 1, np - 1), UB);
            apply_step(q, UA);
            if (q + 1 >= np) break;
            load_rows(min(q + 2, np - 1), UA);
            apply_step(q + 1, UB);
        }
    }
#endif
#pragma unroll
    for (int b = 0; b < NB; b++)
#pragma unroll
        for (int k = 0; k < 4; k++) out[b][k] = from_domain<T>(r[b][k], v.ex);
}

// Block (2·wa, 2·wb) of the landmark block with the pending steps applied, when both landmarks
// are guessed columns (guess indices ta, tb): both sides' operand rows come from the staged LDS
// image. Per element the same chain as pll_blocks.
template <typename T>
__device__ __forceinline__ void pair_block_load(const PllView<T>& v, int wa, int wb, typename Stor<T>::C (&acc)[4])
{
    const int i0 = 2 * wa, jb = 2 * wb;
    const bool swap = (i0 >> 5) > (jb >> 5);   // stored orientation: (jb, i0)
    load_block<T>(v, swap ? jb : i0, swap ? i0 : jb, acc);
}

template <typename T>
__device__ __forceinline__ void staged_pair_block(const PllView<T>& v, int wa, int ta, int wb, int tb,
                                                  const float* stg, typename Stor<T>::C (&acc)[4],
                                                  double (&out)[4])
{
    using C = typename Stor<T>::C;
    const int i0 = 2 * wa, jb = 2 * wb;
    const bool swap = (i0 >> 5) > (jb >> 5);   // stored orientation: (jb, i0)
    const int tA = swap ? tb : ta, tB = swap ? ta : tb;
    for (int q = 0; q < v.npend; q++) {
        const int4 cw = v.ctl[q];
        if (cw.x) {
            acc[0] = acc[1] = acc[2] = acc[3] = (C)0;
            continue;
        }
        if (cw.y > 0) {   // every k-step (see staged_blocks); ks = 0: nothing (rolled back or no match)
            const float* cu = stg + (((tA * SPEC_QMAX + q) * 2 + 0) * 4) * 8;
            const float* cv = stg + (((tB * SPEC_QMAX + q) * 2 + 1) * 4) * 8;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                f32x4v A[4];
#pragma unroll
                for (int rh = 0; rh < 4; rh++) A[rh] = *reinterpret_cast<const f32x4v*>(cu + rh * 8 + 4 * h);
#pragma unroll
                for (int s = 0; s < 4; s++) {
                    // the V side is interleaved (stage_v_index): rows 0 and 1 of k = 4h + s
                    const f32x2v b01 = *reinterpret_cast<const f32x2v*>(cv + stage_v_index(0, 4 * h + s));
                    const f32x2v b23 = *reinterpret_cast<const f32x2v*>(cv + stage_v_index(2, 4 * h + s));
                    acc[0] = fmaf(A[2][s], b23[0], fmaf(A[0][s], b01[0], acc[0]));
                    acc[1] = fmaf(A[2][s], b23[1], fmaf(A[0][s], b01[1], acc[1]));
                    acc[2] = fmaf(A[3][s], b23[0], fmaf(A[1][s], b01[0], acc[2]));
                    acc[3] = fmaf(A[3][s], b23[1], fmaf(A[1][s], b01[1], acc[3]));
                }
            }
#pragma unroll
            for (int k = 0; k < 4; k++) acc[k] = vround<T>(v, acc[k]);
        }
        if (cw.z > 0) patch_block<T>(v, v.pend[q], cw, i0, jb, swap, acc);
    }
    if (swap) {
        out[0] = from_domain<T>(acc[0], v.ex); out[1] = from_domain<T>(acc[2], v.ex);
        out[2] = from_domain<T>(acc[1], v.ex); out[3] = from_domain<T>(acc[3], v.ex);
    } else {
        out[0] = from_domain<T>(acc[0], v.ex); out[1] = from_domain<T>(acc[1], v.ex);
        out[2] = from_domain<T>(acc[2], v.ex); out[3] = from_domain<T>(acc[3], v.ex);
    }
}

// fp64 MFMA-replay contexts (plain pending steps, kmax = 16): the guessed winners' operand rows of
// up to M64_QMAX pending steps staged in LDS as doubles, [winner t][step q][U, V][row][kk][s] (k =
// 16·kk + s for s < 4: pll_blocks' fp64 k order), 32 KB for eight winners and eight steps.
constexpr int M64_QMAX = 8;
__device__ __forceinline__ int m64_stage_index(int t, int q, int uv, int rr, int kk)
{
    return ((((t * M64_QMAX + q) * 2 + uv) * 2 + rr) * 4 + kk) * 4;
}

// Block (2·wa, 2·wb) with the pending steps applied when both landmarks are guessed winners (guess
// indices ta, tb), from the fp64 stage: per element pll_blocks' chain (per step the k-steps s <
// ks, k-chunks kk, one fma per element and k), operand for operand. acc: the stored block in its
// stored orientation (pair_block_load).
template <typename T>
__device__ __forceinline__ void m64_pair_block(const PllView<T>& v, int wa, int ta, int wb, int tb, const double* stg,
                                               typename Stor<T>::C (&acc)[4], double (&out)[4])
{
    const int i0 = 2 * wa, jb = 2 * wb;
    const bool swap = (i0 >> 5) > (jb >> 5);   // stored orientation: (jb, i0)
    const int tA = swap ? tb : ta, tB = swap ? ta : tb;
    for (int q = 0; q < v.npend; q++) {
        const int ks = v.ctl[q].y;   // (no reset, no augmented rows on this path)
        if (ks <= 0) continue;
        const double* cu = stg + m64_stage_index(tA, q, 0, 0, 0);
        const double* cv = stg + m64_stage_index(tB, q, 1, 0, 0);
        for (int s = 0; s < ks; s++)
#pragma unroll
            for (int kk = 0; kk < 4; kk++) {
                const double x0 = cu[kk * 4 + s], x1 = cu[16 + kk * 4 + s];
                const double y0 = cv[kk * 4 + s], y1 = cv[16 + kk * 4 + s];
                acc[0] = fma(x0, y0, (double)acc[0]);
                acc[1] = fma(x0, y1, (double)acc[1]);
                acc[2] = fma(x1, y0, (double)acc[2]);
                acc[3] = fma(x1, y1, (double)acc[3]);
            }
#pragma unroll
        for (int k = 0; k < 4; k++) acc[k] = vround<T>(v, acc[k]);
    }
    if (swap) {
        out[0] = from_domain<T>(acc[0], v.ex); out[1] = from_domain<T>(acc[2], v.ex);
        out[2] = from_domain<T>(acc[1], v.ex); out[3] = from_domain<T>(acc[3], v.ex);
    } else {
        out[0] = from_domain<T>(acc[0], v.ex); out[1] = from_domain<T>(acc[1], v.ex);
        out[2] = from_domain<T>(acc[2], v.ex); out[3] = from_domain<T>(acc[3], v.ex);
    }
}

// Split-bf16 contexts (ScanParams::mfrep): the pending steps' share of the blocks a scan reads,
// ΔX = Σ_q V_q(rows)·V_q(cols)ᵀ over the active pending steps (amask: ks > 0; rolled-back steps
// have ks = 0), by v_mfma_f32_16x16x32_bf16 on the operand planes the association kernels wrote
// (V = hi + mid + lo exactly, the six part products of the flush). One instruction takes two
// steps: k-groups 0/1 the even/odd k of step qa, 2/3 those of step qb (the same k permutation on
// both operands). NB M-blocks of 16 rows: A row row_a(mb, r), B (16 columns) row row_b(c); a
// negative or out-of-range row is a zero operand. Lane l holds ΔX[4·(l >> 4) + i][l & 15] of
// M-block mb in acc[mb][i]. Not the fp32 chain of the flush (the split-bf16 flush is not one
// either): held to the same parity bar.
typedef __bf16 bf16x8r __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8r __attribute__((ext_vector_type(8)));
// F16 (EKF_ARITH_F16X3): two fp16 planes (hi, lo of 2^σ·V), three products (lo, hi), (hi, lo),
// (hi, hi) on v_mfma_f32_16x16x32_f16; acc then holds 2^(2σ)·ΔX (the caller scales it back)
// BATCH pairs of pending steps per memory round trip: every operand load of the BATCH pairs is
// issued before the first of their MFMAs (the replay wave's 16 winner rows: a few loads per pair,
// latency-bound; the landmark waves' 128 rows keep BATCH = 1). The MFMAs run in the same order for
// every BATCH, so the accumulators are the same bits.
template <int NB, bool F16, int BATCH = 1, typename RA, typename RB>
__device__ __forceinline__ void plane_replay(const Slot* pend, int e, size_t inst_bf, int M, unsigned amask,
                                             int lane, RA row_a, RB row_b, f32x4v (&acc)[NB])
{
    constexpr int NPL = F16 ? 2 : 3;
    using PV = typename std::conditional<F16, f16x8r, bf16x8r>::type;
#pragma unroll
    for (int mb = 0; mb < NB; mb++) acc[mb] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int kg = lane >> 4, h = kg & 1, r16 = lane & 15;
    typedef unsigned u32x4r __attribute__((ext_vector_type(4)));
    const PV zero = __builtin_bit_cast(PV, u32x4r{0u, 0u, 0u, 0u});
    const int rb_ = row_b(r16);
    int ra_[NB];
#pragma unroll
    for (int mb = 0; mb < NB; mb++) ra_[mb] = row_a(mb, r16);
    unsigned m = amask;
    while (m) {
        int qa[BATCH];
        PV B[BATCH][NPL], A[BATCH][NB][NPL];
#pragma unroll
        for (int bb = 0; bb < BATCH; bb++) {
            qa[bb] = m ? __builtin_ctz(m) : -1;
            if (m) m &= m - 1;
            const int qb = m ? __builtin_ctz(m) : -1;
            if (qb >= 0) m &= m - 1;
            const int q0 = qa[bb] >= 0 ? qa[bb] : 0;
            const unsigned short* pa = reinterpret_cast<const unsigned short*>(pend[q0].Bop) + (size_t)e * inst_bf;
            const unsigned short* pb = qb >= 0 ? reinterpret_cast<const unsigned short*>(pend[qb].Bop) + (size_t)e * inst_bf : pa;
            const unsigned short* pq = (kg >= 2) ? pb : pa;
            const bool none = qa[bb] < 0 || (kg >= 2 && qb < 0);
#pragma unroll
            for (int pl = 0; pl < NPL; pl++)
                B[bb][pl] = (!none && rb_ >= 0 && rb_ < M) ? *reinterpret_cast<const PV*>(pq + op_index_pl(rb_, h, pl, NPL)) : zero;
#pragma unroll
            for (int mb = 0; mb < NB; mb++)
#pragma unroll
                for (int pl = 0; pl < NPL; pl++)
                    A[bb][mb][pl] = (!none && ra_[mb] >= 0 && ra_[mb] < M)
                                        ? *reinterpret_cast<const PV*>(pq + op_index_pl(ra_[mb], h, pl, NPL)) : zero;
        }
#pragma unroll
        for (int bb = 0; bb < BATCH; bb++) {
            if (qa[bb] < 0) break;   // (uniform)
            if constexpr (F16) {
#pragma unroll
                for (int pp = 0; pp < 3; pp++) {
                    const int a = pp == 0 ? 1 : 0, b = pp == 1 ? 1 : 0;   // (lo, hi), (hi, lo), (hi, hi)
#pragma unroll
                    for (int mb = 0; mb < NB; mb++)
                        acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_f16(A[bb][mb][a], B[bb][b], acc[mb], 0, 0, 0);
                }
            } else {
#pragma unroll
                for (int pp = 0; pp < 6; pp++) {
                    const int a = (0x102010 >> (4 * (5 - pp))) & 0xf;   // (mid, mid), (hi, lo), (lo, hi),
                    const int b = (0x120100 >> (4 * (5 - pp))) & 0xf;   // (hi, mid), (mid, hi), (hi, hi)
#pragma unroll
                    for (int mb = 0; mb < NB; mb++)
                        acc[mb] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(A[bb][mb][a], B[bb][b], acc[mb], 0, 0, 0);
                }
            }
        }
    }
}

// Split-plane contexts, EKF_OPT_MFMA_REPLAY = 2: the same ΔX = Σ_q V_q(rows)·V_q(cols)ᵀ by
// v_mfma_f32_16x16x4_f32 on the fp32 operand rows V_q themselves (kmax = 16), exact fp32 products
// accumulated in fp32: within a flush group the association kernel reads the landmark block at
// the precision of the EXACT arithmetic, and the split products enter P only at the group's
// flush (≈3 µs per scan more than the plane replay at T = 20: 4× the MFMA cycles).
// Same bytes per row and step as the two fp16 planes (64). Lane l
// loads one 16-byte quarter of a row's operand row: memory lane (row & 31) + 32·b, slots 4a..4a+3
// with (a, b) = (kk >> 1, kk & 1), kk = l >> 4; chunk c takes slot 4a + c, i.e. k = 2·(4a + c) + b
// on both operands (a k permutation: every dot product keeps its terms). acc layout as
// plane_replay's.
template <int NB, typename RA, typename RB>
__device__ __forceinline__ void f32_replay(const Slot* pend, int e, size_t opstride, int M, unsigned amask,
                                           int lane, RA row_a, RB row_b, f32x4v (&acc)[NB])
{
#pragma unroll
    for (int mb = 0; mb < NB; mb++) acc[mb] = f32x4v{0.f, 0.f, 0.f, 0.f};
    const int kk = lane >> 4, r16 = lane & 15;
    const int qoff = 32 * (kk & 1) * 8 + 4 * (kk >> 1);   // floats, within a row's 32-row block
    auto off = [&](int row) __attribute__((always_inline)) {
        return ((size_t)(row >> 5) * 64 + (row & 31)) * 8 + qoff;
    };
    const f32x4v zero = {0.f, 0.f, 0.f, 0.f};
    const int rb_ = row_b(r16);
    const bool bok = rb_ >= 0 && rb_ < M;
    const size_t boff = bok ? off(rb_) : 0;
    size_t aoff[NB];
    bool aok[NB];
#pragma unroll
    for (int mb = 0; mb < NB; mb++) {
        const int ra = row_a(mb, r16);
        aok[mb] = ra >= 0 && ra < M;
        aoff[mb] = aok[mb] ? off(ra) : 0;
    }
    unsigned m = amask;
    while (m) {
        // two steps per round trip: both steps' rows issued before either step's MFMAs
        const int qa = __builtin_ctz(m);
        m &= m - 1;
        const int qb = m ? __builtin_ctz(m) : -1;
        if (qb >= 0) m &= m - 1;
        const float* va = reinterpret_cast<const float*>(pend[qa].Vop) + (size_t)e * opstride;
        const float* vb = reinterpret_cast<const float*>(pend[qb >= 0 ? qb : qa].Vop) + (size_t)e * opstride;
        f32x4v Ba = bok ? *reinterpret_cast<const f32x4v*>(va + boff) : zero;
        f32x4v Bb = (bok && qb >= 0) ? *reinterpret_cast<const f32x4v*>(vb + boff) : zero;
        f32x4v Aa[NB], Ab[NB];
#pragma unroll
        for (int mb = 0; mb < NB; mb++) {
            Aa[mb] = aok[mb] ? *reinterpret_cast<const f32x4v*>(va + aoff[mb]) : zero;
            Ab[mb] = (aok[mb] && qb >= 0) ? *reinterpret_cast<const f32x4v*>(vb + aoff[mb]) : zero;
        }
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int mb = 0; mb < NB; mb++)
                acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(Aa[mb][c], Ba[c], acc[mb], 0, 0, 0);
#pragma unroll
        for (int c = 0; c < 4; c++)
#pragma unroll
            for (int mb = 0; mb < NB; mb++)
                acc[mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(Ab[mb][c], Bb[c], acc[mb], 0, 0, 0);
    }
}

// EKF_ARITH_F16X3: x = 2^σ·v as hi + lo fp16 (hi = fp16(x) round-to-nearest, lo = fp16(x − hi), the
// remainder exact in fp32): 22 significant bits; (a, b) packed into one dword per part, a low
__device__ __forceinline__ void split_pack_f16(float a, float b, int sig, unsigned (&o)[2])
{
    const float xa = ldexpf(a, sig), xb = ldexpf(b, sig);
    const _Float16 ha = (_Float16)xa, hb = (_Float16)xb;
    const _Float16 la = (_Float16)(xa - (float)ha), lb = (_Float16)(xb - (float)hb);
    o[0] = (unsigned)__builtin_bit_cast(unsigned short, ha) | ((unsigned)__builtin_bit_cast(unsigned short, hb) << 16);
    o[1] = (unsigned)__builtin_bit_cast(unsigned short, la) | ((unsigned)__builtin_bit_cast(unsigned short, lb) << 16);
}

// Speculative association (lines <= SPEC_L, G <= SPEC_GMAX): every line's winner is guessed
// from the pre-update state, the guesses' mutual data are exchanged once, every workgroup
// replays the winners' part of the sequential chain to get all gain packages, then every thread
// runs the sequential gating and gain rows against those packages locally and flags any line
// whose exact first passing candidate differs from the guess. Three exchanges per scan instead
// of one per line; on a flag the scan restarts on the sequential path (identical results).

// ST: phase timers (EKF_OPT_SCAN_STAMPS). HOT (1, 2): the launch guarantees symmetric fp32 operands
// with kmax = 16 (the bench and every EKF_R_INTENDED fp32/fp16 context with max_lines <= 8): the
// per-line loops then carry no code for the other operand forms; HOT = 2 also fixes the plane
// arithmetic to EKF_ARITH_F16X3, HOT = 1 to EKF_ARITH_BF16X6 or none. HOT = 0: decided at run time.
// NT: landmarks (threads) per workgroup, 192 by default; 128 and 64 (ScanParams::nt) spread a small
// map's instances over more CUs (the commit's stores and the replay per CU scale with it)
template <typename T, bool ST, int HOT, int NT = ekf::SCAN_THREADS>
__global__ __launch_bounds__(NT + 64) void scan_kernel(ScanParams p)
{
    // (these hide the namespace defaults for the whole kernel body)
    constexpr int SCAN_THREADS = NT;
    constexpr int SCAN_BLOCK = NT + 64;
    const Dims d = p.d;
    const int r_mode = HOT ? (int)EKF_R_INTENDED : p.r_mode;   // (HOT: the launch checked it)
    constexpr double ETA = gate_eta<T>();
    // 1-D grid, instance-minor: block b is workgroup b / E of instance b % E. Workgroups are
    // dealt round-robin over the 8 XCDs, so with 8 instances per launch each instance's
    // workgroups share one XCD (and its L2) in every launch; correctness never depends on it
    const int g = (int)blockIdx.x / p.E;
    const int e = p.e0 + (int)blockIdx.x % p.E;
    const int G = p.G;
    const int tid = threadIdx.x;
    // threads < SCAN_THREADS own landmark j; the last wave (no landmark) replays the guessed
    // winners' chain in the speculative association
    const int j = tid < SCAN_THREADS ? g * SCAN_THREADS + tid : -1 - tid;
    const bool own = tid < SCAN_THREADS && j < d.N;
    const int n = d.n, N = d.N, M = d.M;
    const int b0 = 3 + 2 * j;                   // its first row of P
    // robot strip and mean: read the committed copy, write the other (committed by the lead at
    // the end only if every workgroup completed: a timed-out launch leaves the state untouched)
    const int cb = p.live[e];
    const double* Rs = p.Rs + ((size_t)cb * p.Etot + e) * 3 * n;
    const double* y = p.y + ((size_t)cb * p.Etot + e) * n;
    double* Rsw = p.Rs + ((size_t)(1 - cb) * p.Etot + e) * 3 * n;
    double* yw = p.y + ((size_t)(1 - cb) * p.Etot + e) * n;
    // diagonal landmark blocks after the last committed step (split-bf16 contexts), same two copies
    const double4* Ddr = p.mfrep ? reinterpret_cast<const double4*>(p.Dd) + ((size_t)cb * p.Etot + e) * d.N : nullptr;
    double4* Ddw = p.mfrep ? reinterpret_cast<double4*>(p.Dd) + ((size_t)(1 - cb) * p.Etot + e) * d.N : nullptr;
    int* sync = p.sync + (size_t)e * p.sync_stride;
    double* mbox = p.mbox + (size_t)e * 2 * G * p.mbw;
    const bool lead = (g == 0 && tid == 0);
    if (p.test_drop == e + 1 && G > 1 && g == G - 1) return;   // test hook: a workgroup that never runs

    __shared__ double sh_pkg[MB_VH + 4 * EKF_MAX_LINES];
    __shared__ int sh_red[SCAN_BLOCK / 64];
    __shared__ int sh_best[MAX_GROUPS];
    __shared__ int sh_extra[EKF_MAX_LINES];
    __shared__ int4 sh_ctl[PMAX];
    __shared__ ekf_line sh_lines[EKF_MAX_LINES];
    // U_q rows of the owned landmark for the first HIST_LDS matches of the scan (the rest in Ust)
    __shared__ double4 sh_uhist[HIST_LDS][SCAN_THREADS];
    // V_q rows (sequential path, for the package); owned blocks of the guessed columns as fp32
    // (speculative path with fp32 operands: the values are fp32 numbers)
    __shared__ double4 sh_vhist[HIST_V][SCAN_THREADS];
    static_assert(sizeof(float4) * SPEC_L == sizeof(double4) * HIST_V, "block buffer aliases sh_vhist");
    float4 (*sh_blk)[SCAN_THREADS] = reinterpret_cast<float4 (*)[SCAN_THREADS]>(&sh_vhist[0][0]);
    // fp64 operands: the owned blocks of the guessed columns in fp64 (48 KB; a placeholder otherwise)
    constexpr bool kB64 = sizeof(typename Stor<T>::C) == 8;
    __shared__ double4 sh_blk64[kB64 ? SPEC_L : 1][kB64 ? SCAN_THREADS : 1];
    // speculative association
    __shared__ unsigned long long sh_wl[SPEC_L][SCAN_THREADS / 64];
    __shared__ unsigned long long sh_lists[SPEC_GMAX * SPEC_L];
    __shared__ unsigned long long sh_listsb[SPEC_GMAX * SPEC_L];   // the B words (count > 4)
    __shared__ int sh_glist[SPEC_L][SPEC_K + 1];
    __shared__ int sh_spec[SPEC_L];
    __shared__ int sh_psg[PMAX];      // pending steps' plane exponents (EKF_ARITH_F16X3)
    __shared__ int sh_flag;
    __shared__ int sh_ready;
    __shared__ int sh_rwst;   // status bits of the replay wave (the winners' GSL_EDOM)
    __shared__ int sh_vto;    // a verdict poll of this workgroup timed out
    __shared__ int sh_first[SPEC_L];   // per line the first guessed candidate (speculative path)
    if (tid < SPEC_L) sh_first[tid] = 0x7fffffff;
    // the replay wave's line counter and status words: set before the first barrier below, since
    // on the MFMA-replay path the landmark waves reach their polls with no barrier after the records
    if (tid == 0) {
        sh_ready = 0;
        sh_rwst = 0;
        sh_vto = 0;
    }
    __shared__ double sh_wd[SPEC_L * SPEC_WD];
    __shared__ double4 sh_wh[SPEC_L][SPEC_L][2];
    __shared__ double sh_pk[SPEC_L][PKW];
    __shared__ __attribute__((aligned(16))) float sh_stg[SPEC_L * SPEC_QMAX * 2 * 4 * 8];   // staged pending-step rows
    __shared__ unsigned long long sh_stamp[EKF_NSTAMP];
    // EKF_ARITH_BF16X6 (fp32 storage): the owned rows' V values of this scan's matches (k-major
    // per row), split into bf16 planes and stored once at the end
    // fp32 operand storage (fp32 and fp16 P): the split-bf16 planes, the MFMA replay
    constexpr bool kPlanes = sizeof(typename Stor<T>::C) == 4;
    __shared__ __attribute__((aligned(16))) float sh_vpl[kPlanes ? SCAN_THREADS * 32 : 4];
    // plane arithmetic (HOT fixes it at compile time): EKF_ARITH_F16X3 planes hold hi + lo fp16 of
    // 2^σ·V. σ follows the largest landmark variance vmax (pvmax[e]) but changes only at the first
    // scan of a flush group (every workgroup of the instance computes it from pvmax), so that a
    // group's steps share one σ and the flush takes its pipelined path; mid-group only a reset
    // (σ empty) or a new landmark 64× above the variance σ was set for (then at the step that adds
    // it: that group and every pending replay over it take the exact forms). The MFMA replay of
    // plain pending steps returns 2^(2σ)·ΔX.
    const bool pf16 = kPlanes && (HOT == 2 || (HOT == 0 && p.bf == 2));
    const int npl = pf16 ? 2 : 3;
    const int psig = !pf16 ? 0 : p.npend == 0 ? plane_sigma(p.pvmax[e]) : p.psig[e];
    const double rsc = pf16 ? ldexp(1.0, -2 * psig) : 1.0;
    // the on-read replay of plain pending steps (EKF_OPT_MFMA_REPLAY): 1 the split products on
    // the planes (plane_replay: 2^(2σ)·ΔX for EKF_ARITH_F16X3), 2 fp32 MFMA on the fp32 operand
    // rows (f32_replay: ΔX unscaled); 1 also takes f32_replay when a pending step's planes were
    // written at another exponent or could not carry the instance's range (PLANE_SIGMA_EXACT),
    // instead of the exact per-element forms (below; the flush still takes the exact forms)
    bool f32rep = kPlanes && p.mfrep == 2;
    double rrsc = f32rep ? 1.0 : rsc;
    // phase timers only in the ST instantiation (EKF_SCAN_STAMPS=1): the product kernel carries
    // no timer code at all (its uniform branches and registers cost ≈2 µs per scan)
    unsigned long long* const pdbg = ST ? p.dbg : nullptr;
    unsigned long long* dbg = (pdbg && lead) ? pdbg + (size_t)e * EKF_NSTAMP : nullptr;
    if (pdbg && tid < EKF_NSTAMP) sh_stamp[tid] = 0;
    unsigned long long t_last = dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
    const unsigned long long t_first = t_last;

    // owned state, in registers for the whole scan
    double2 rr0, rr1, rr2, yb;
    double R33[9], xp[3];
    double F3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    // (re)load the owned state and apply the predict (Robot.cpp:130-286, SIMULATIONOFF == true:
    // `rot` unused); the inputs stay untouched until the commit, so a restart is exact
    auto init_state = [&]() {
        rr0 = make_double2(0, 0); rr1 = rr0; rr2 = rr0; yb = rr0;
        if (own) {
            rr0 = *reinterpret_cast<const double2*>(Rs + b0);
            rr1 = *reinterpret_cast<const double2*>(Rs + n + b0);
            rr2 = *reinterpret_cast<const double2*>(Rs + 2 * n + b0);
            yb = *reinterpret_cast<const double2*>(y + b0);
        }
#pragma unroll
        for (int a = 0; a < 9; a++) R33[a] = Rs[(a / 3) * n + (a % 3)];
        if (p.phase & PHASE_PREDICT) {
            const double x0 = p.pose[3 * e + 0], y0 = p.pose[3 * e + 1], t0 = p.pose[3 * e + 2];
            const double* enc = p.enc + 3 * e;
            const double u2 = t0 - enc[2];
            const double dx = x0 - enc[0], dy = y0 - enc[1];
            const double u0 = sqrt(dx * dx + dy * dy);
            const double c = u2 / 2.0 + t0;
            double sc, cc;
            sincos(c, &sc, &cc);
            F3[2] = -u0 * sc;
            F3[5] = u0 * cc;
            // cos/sin(t0 + u2/2) of Robot.cpp:150-151: the same angle as c (addition commutes)
            xp[0] = x0 + u0 * cc;
            xp[1] = y0 + u0 * sc;
            xp[2] = t0 + u2;
            predict_cols(F3, rr0, rr1, rr2);
            // 3×3 block: F3·P33·F3ᵀ + Fu3·Q·Fu3ᵀ (Robot.cpp:178-258)
            const double Fu3[9] = {cc, 0, -u0 * sc / 2.0, sc, 1, u0 * cc / 2.0, 0, 0, 1};
            const double qs = (-1.0 / (1 + fabs(u0)) + 1);
            const double Q[9] = {p.enc_noise * qs, 0, 0, 0, 2 * p.enc_noise * qs, 0, 0, 0,
                                 p.enc_noise * qs};
            double FP[9], FuQ[9];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) {
                    double s = 0.0, t = 0.0;
                    for (int k = 0; k < 3; k++) {
                        s += F3[a * 3 + k] * R33[k * 3 + b];
                        t += Fu3[a * 3 + k] * Q[k * 3 + b];
                    }
                    FP[a * 3 + b] = s;
                    FuQ[a * 3 + b] = t;
                }
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) {
                    double s = 0.0, t = 0.0;
                    for (int k = 0; k < 3; k++) {
                        s += FP[a * 3 + k] * F3[b * 3 + k];
                        t += FuQ[a * 3 + k] * Fu3[b * 3 + k];
                    }
                    R33[a * 3 + b] = s + t;
                }
        } else {
            xp[0] = p.xpre[3 * e + 0];
            xp[1] = p.xpre[3 * e + 1];
            xp[2] = p.xpre[3 * e + 2];
        }
    };
    // the owned diagonal block as last flushed (the staged speculative path guesses from it),
    // issued with the owned-state loads: the scan's inputs arrive in one memory round trip
    typename Stor<T>::C dj0[4] = {0, 0, 0, 0};
    double4 djb = make_double4(0, 0, 0, 0);   // the kept diagonal block (split-bf16 contexts)
    if (own && (p.phase & PHASE_UPDATE)) {
        PllView<T> v0;
        v0.X = reinterpret_cast<const T*>(p.Pread) + (size_t)e * d.ntiles * TILE_ELEMS;
        v0.nb = d.nb;
        v0.rnd = 1;
        load_block<T>(v0, 2 * j, 2 * j, dj0);
        if (Ddr && p.npend > 0) djb = Ddr[j];
    }
    // the scan's other inputs, issued with the state loads (one memory round trip): the pending
    // steps' control words, the line count, savedLineCount and the line words
    int4 ctl_pre = make_int4(0, 0, 0, 0);
    int psg_pre = 0;
    if ((p.phase & PHASE_UPDATE) && tid < p.npend) {
        const int* r = p.pend[tid].res + (size_t)e * RES_STRIDE;
        ctl_pre = make_int4(r[RES_RESET], r[RES_KSTEPS], r[RES_NADD], r[RES_SAVED_IN]);
        psg_pre = r[RES_PSIG];
    }
    const int L_pre = p.nlines[e];
    const int s_pre = (p.phase & PHASE_UPDATE) ? p.saved[e] : 0;
    constexpr int LW_PER = (EKF_MAX_LINES * 6 + SCAN_BLOCK - 1) / SCAN_BLOCK;
    double lw_pre[LW_PER];
    {
        const double* src = reinterpret_cast<const double*>(p.lines + (size_t)e * d.max_lines);
#pragma unroll
        for (int k = 0; k < LW_PER; k++) {
            const int idx = tid + k * SCAN_BLOCK;
            lw_pre[k] = ((p.phase & PHASE_UPDATE) && idx < d.max_lines * 6) ? src[idx] : 0.0;
        }
    }
    init_state();
    // the owned landmark's angle at the start of the scan and its sin/cos (sincos_near)
    // sin/cos of the owned landmark's scan-start angle: fp32 now (the quick filter's bound and the
    // guess), the exact fp64 ones (sincos_near) only where a lane needs the exact evaluation
    double ma0 = yb.x, s0j = 0.0, c0j = 1.0;
    bool sc_exact = false;
    float s0f = 0.f, c0f = 1.f;
    if (own && (p.phase & PHASE_UPDATE)) __sincosf((float)ma0, &s0f, &c0f);
    auto exact_sc = [&]() {
        if (!sc_exact) {
            sincos(ma0, &s0j, &c0j);
            sc_exact = true;
        }
    };

    if (!(p.phase & PHASE_UPDATE)) {
        // predict only: the predicted robot strip (and the mean, unchanged) into the other copy,
        // the 3×3 block and x_pre by the lead once every workgroup completed
        if (own) {
            *reinterpret_cast<double2*>(Rsw + b0) = rr0;
            *reinterpret_cast<double2*>(Rsw + n + b0) = rr1;
            *reinterpret_cast<double2*>(Rsw + 2 * n + b0) = rr2;
            *reinterpret_cast<double2*>(yw + b0) = yb;
            if (Ddr) Ddw[j] = Ddr[j];
        }
        if (tid == 0 && g != 0) publish_done(sync, g, p.epoch, 0);
        if (g == 0) {
            int zg_unused = 0;
            const int st = lead_collect<SCAN_BLOCK>(sync, G, p.epoch, 0, p.spin_log2, tid, sh_red, zg_unused);
            if (lead) sync[SYNC_WG0] = (int)done_word(p.epoch, st);
            if (lead && !(st & EKF_ST_TIMEOUT_BIT)) {
                for (int a = 0; a < 9; a++) Rsw[(a / 3) * n + (a % 3)] = R33[a];
                yw[0] = y[0]; yw[1] = y[1]; yw[2] = y[2];
                p.xpre[3 * e + 0] = xp[0];
                p.xpre[3 * e + 1] = xp[1];
                p.xpre[3 * e + 2] = xp[2];
                p.live[e] = 1 - cb;
            }
        }
        return;
    }
    EKF_STAMP(0);

    // ---------------- association / update (Robot.cpp:288-904) ----------------
    const size_t opstride = (size_t)d.nb * 64 * (d.kmax / 2);
    double* Ust = p.Ust + (size_t)e * d.max_lines * n * 2;
    double* Vst = p.Vst + (size_t)e * d.max_lines * n * 2;
    using C = typename Stor<T>::C;   // operand (compute) type
    C* Uop = reinterpret_cast<C*>(p.cur.Uop) + (size_t)e * opstride;
    C* Vop = reinterpret_cast<C*>(p.cur.Vop) + (size_t)e * opstride;
    // split-plane arithmetics: V's planes for the split flush (null otherwise)
    unsigned short* Bop = p.cur.Bop ? reinterpret_cast<unsigned short*>(p.cur.Bop) + (size_t)e * opstride * npl
                                    : nullptr;
    // (staged in LDS, sh_vpl, and written once at the end: per-match 2-byte global stores cost
    // ≈4 µs of the chain, since on CDNA every store counts in vmcnt and each later load wait
    // then also waited for them)
    double* patch = p.cur.patch + (size_t)e * d.max_lines * 2 * M;
    double* pdiag = p.cur.patch_diag + (size_t)e * d.max_lines * 4;
    int* res = p.cur.res + (size_t)e * RES_STRIDE;

    PllView<T> pv;
    pv.X = reinterpret_cast<const T*>(p.Pread) + (size_t)e * d.ntiles * TILE_ELEMS;
    pv.nb = d.nb;
    pv.kmax = d.kmax;
    pv.M = M;
    pv.max_lines = d.max_lines;
    pv.e = e;
    pv.ex = storage_exp<T>(p.pexp, e);
    pv.opstride = opstride;
    pv.usym = p.usym;
    pv.us = p.usym ? -ldexpf(1.0f, pv.ex) : 1.0f;
    pv.npend = p.npend;
    pv.pend = p.pend;
    pv.ctl = sh_ctl;
    pv.rnd = !p.bf;
    if (tid < p.npend) {
        sh_ctl[tid] = ctl_pre;
        sh_psg[tid] = psg_pre;
    }

    int L = L_pre;
    L = L < 0 ? 0 : (L > d.max_lines ? d.max_lines : L);
    const int s = s_pre;
#pragma unroll
    for (int k = 0; k < LW_PER; k++) {
        const int idx = tid + k * SCAN_BLOCK;
        if (idx < L * 6) reinterpret_cast<double*>(sh_lines)[idx] = lw_pre[k];
    }
    __syncthreads();   // sh_lines, sh_ctl

    const bool spec_ok = p.spec && L > 0 && L <= SPEC_L && s > 0 && G <= SPEC_GMAX;
    // symmetric downdate operands (sym_factor): fp32 operand storage, every mode but the
    // reference's asymmetric R
    const bool sym = HOT || (r_mode != 1 && sizeof(typename Stor<T>::C) == 4);
    // symmetric fp32 operands with kmax = 16: staged in LDS (sh_vpl) and written at the end
    const bool stage_ops = HOT || (sym && d.kmax == 16);
    // speculative path with fp32 operands and few pending steps: the pending steps' rows of the
    // guessed columns are staged in LDS and one pass per step updates all owned blocks
    bool staged = false;
    // split-bf16 contexts with plain pending steps (no reset, no augmented rows): the pending
    // steps are applied by bf16 MFMA on the operand planes (plane_replay) and the diagonal blocks
    // come from Dd (the last committed step's, exact); fp32 storage
    bool mf = false;
    int rpath = 0;   // diagnostic (RES_DBG): 64 the pending replay took an exact form, 128 a pending
                     // reset, 256 a pending plane exponent other than this scan's
    bool aug_pend = false;   // some pending step adds landmarks (uniform)
    unsigned amask = 0;   // pending steps with a downdate (ks > 0)
    // (the MFMA replay reads the planes, not the LDS stage: any number of pending steps)
    if (spec_ok && sym && sizeof(typename Stor<T>::C) == 4 && d.kmax / 2 >= 8) {
        __syncthreads();   // sh_ctl
        bool st = true;
        for (int q = 0; q < p.npend; q++) st &= sh_ctl[q].y <= 8;
        // pending steps that add landmarks stay on the MFMA replay: a block touching a landmark
        // added at step q* starts from q*'s patch (its V rows are zero before), below; a reset or
        // a plane exponent other than this scan's takes the exact forms
        bool m = st && p.mfrep && kPlanes;
        if (pf16 && p.mfrep == 1) {
            for (int q = 0; q < p.npend; q++) f32rep |= sh_psg[q] != psig;
            rrsc = f32rep ? 1.0 : rsc;
        }
        for (int q = 0; q < p.npend; q++) {
            // (the planes of a step written with another exponent: only the plane replay minds)
            const bool sgx = pf16 && !f32rep && sh_psg[q] != psig;
            m &= !sh_ctl[q].x && !sgx;
            rpath |= (sh_ctl[q].x ? 128 : 0) | (pf16 && sh_psg[q] != psig ? 256 : 0);
            aug_pend |= sh_ctl[q].z > 0;
            if (sh_ctl[q].y > 0) amask |= 1u << q;
        }
        staged = st && (p.npend <= SPEC_QMAX || m);
        mf = m && staged;
    }
    // fp64 storage, plain pending steps (no reset, no augmented rows): the owned rows' blocks of
    // the guessed columns and the owned diagonal blocks by v_mfma_f64_16x16x4f64 over the pending
    // steps' operand rows, the flush's own instruction on its own operands (below, phase (e))
    bool m64 = false;
    if constexpr (sizeof(typename Stor<T>::C) == 8)
        if (spec_ok && p.mfrep64 && d.kmax == 16 && p.npend > 0) {
            bool m = true;
            for (int q = 0; q < p.npend; q++) m &= !sh_ctl[q].x && sh_ctl[q].z == 0;
            m64 = m;
        }
    if (p.npend > 0 && !mf && !m64) rpath |= 64;
    double Dj[4] = {0, 0, 0, 0};   // owned diagonal block
    if (own && j < s) {
        if (mf && p.npend > 0) {
            Dj[0] = djb.x; Dj[1] = djb.y; Dj[2] = djb.z; Dj[3] = djb.w;
        } else if (staged || m64) {
            // the guess only needs it approximately: the last flushed value (exact one below)
#pragma unroll
            for (int a = 0; a < 4; a++) Dj[a] = from_domain<T>(dj0[a], pv.ex);
        } else {
            pll_block(pv, 2 * j, 2 * j, Dj);
        }
    }
    EKF_STAMP(1);

    // writes a match's owned rows: U/V history and the MFMA downdate operands
    // F: the line's symmetric operand factor (sym_factor; unused otherwise)
    bool nzr = false;   // this thread wrote a nonzero operand row (DONE_NZ, RES_ZMAX)
    // the scan's downdate of the owned 2×2 diagonal block, trace (Σ over matches and both rows of
    // −U·V ≥ 0): with the block after the scan it measures the update's cancellation (EKF_ST_PRECISION)
    double dsq = 0.0;
    // uhist: keep the U rows for later corrections (the sequential path; the speculative landmark
    // waves apply each match to the later blocks at once and keep only the last one, in registers)
    auto store_rows = [&](int t, const double kk[4], const double uu[4], bool vhist, const float F[3], bool uhist) {
        nzr = nzr || kk[0] != 0.0 || kk[1] != 0.0 || kk[2] != 0.0 || kk[3] != 0.0 || uu[0] != 0.0 ||
              uu[1] != 0.0 || uu[2] != 0.0 || uu[3] != 0.0;
        if (!uhist) {
        } else if (t < HIST_LDS)
            sh_uhist[t][tid] = make_double4(uu[0], uu[1], uu[2], uu[3]);
        else
            *reinterpret_cast<double4*>(Ust + ((size_t)t * n + b0) * 2) = make_double4(uu[0], uu[1], uu[2], uu[3]);
        if (vhist) {
            if (t < HIST_V)
                sh_vhist[t][tid] = make_double4(kk[0], kk[1], kk[2], kk[3]);
            else
                *reinterpret_cast<double4*>(Vst + ((size_t)t * n + b0) * 2) = make_double4(kk[0], kk[1], kk[2], kk[3]);
        }
#pragma unroll
        for (int pp = 0; pp < 2; pp++) {
            const int lr = 2 * j + pp;
            if constexpr (sizeof(C) == 4) {
                double o0 = uu[2 * pp], o1 = uu[2 * pp + 1], v0 = kk[2 * pp], v1 = kk[2 * pp + 1];
                if (sym) {   // V = K·F, U = −2^x·V (sym_factor)
                    v0 = kk[2 * pp] * (double)F[0] + kk[2 * pp + 1] * (double)F[1];
                    v1 = kk[2 * pp + 1] * (double)F[2];
                    o0 = (double)(float)v0;
                    o1 = (double)(float)v1;
                }
                dsq += o0 * v0 + o1 * v1;   // (row pp's diagonal entry falls by it)
                if (stage_ops) {
                    // staged in LDS: the operand rows (U, V, the bf16 planes) go out once at the end
                    // of the scan as whole 16-byte lane rows
                    if constexpr (kPlanes)
                        *reinterpret_cast<f32x2v*>(sh_vpl + tid * 32 + pp * 16 + 2 * t) = f32x2v{(float)v0, (float)v1};
                } else {
                    if (!p.usym) {   // (symmetric operands: U = −2^x·V, read from V)
                        Uop[op_index_f32(lr, 2 * t, d.kmax)] = to_domain<T>(-o0, pv.ex);
                        Uop[op_index_f32(lr, 2 * t + 1, d.kmax)] = to_domain<T>(-o1, pv.ex);
                    }
                    Vop[op_index_f32(lr, 2 * t, d.kmax)] = (C)v0;
                    Vop[op_index_f32(lr, 2 * t + 1, d.kmax)] = (C)v1;
                }
            } else {
                Uop[op_index_f64(lr, 2 * t, d.kmax)] = (C)(-uu[2 * pp]);
                Uop[op_index_f64(lr, 2 * t + 1, d.kmax)] = (C)(-uu[2 * pp + 1]);
                Vop[op_index_f64(lr, 2 * t, d.kmax)] = (C)kk[2 * pp];
                Vop[op_index_f64(lr, 2 * t + 1, d.kmax)] = (C)kk[2 * pp + 1];
            }
        }
    };
    auto uq_owned = [&](int q) -> double4 {
        return q < HIST_LDS ? sh_uhist[q][tid] : *reinterpret_cast<const double4*>(Ust + ((size_t)q * n + b0) * 2);
    };
    // symmetric operands from their LDS stage (stage_ops): per owned row and k parity h one 16-byte
    // half of the 32-byte lane row, half 0 = k slots 0..3 (matches 0..3), half 1 = slots 4..7; V and
    // U = −2^x·V (exact); k past the matches +0 (V) and −0 (U), so that a flush running every
    // k-step leaves every value as it is (flush_f32_wave_kernel; the other forms and the on-read
    // replay stop at ks). Half 0 is final after the fourth match: the speculative path stores it
    // then, during the later lines (the commit's stores are issue-bound, ≈10 B/clk per CU)
    int ops_early = 0;
    auto store_ops_half = [&](int half, int mm) {   // mm: the matches
        if constexpr (kPlanes) {
            const float us = -ldexpf(1.0f, pv.ex);
            const bool su = !p.usym;   // (usym: U = us·V is not stored; the readers scale V)
#pragma unroll
            for (int pp = 0; pp < 2; pp++) {
                const f32x4v* src = reinterpret_cast<const f32x4v*>(sh_vpl + tid * 32 + pp * 16) + 2 * half;
                float v[8];
#pragma unroll
                for (int i = 0; i < 2; i++) {
                    const f32x4v x = src[i];
#pragma unroll
                    for (int u = 0; u < 4; u++) v[4 * i + u] = (8 * half + 4 * i + u) < 2 * mm ? x[u] : 0.f;
                }
#pragma unroll
                for (int h = 0; h < 2; h++) {
                    const size_t o = op_index_f32(2 * j + pp, h, d.kmax) + 4 * half;   // k = h: s = 0
                    const f32x4v vh = {v[h], v[2 + h], v[4 + h], v[6 + h]};
                    *reinterpret_cast<f32x4v*>(Vop + o) = vh;
                    if (su) *reinterpret_cast<f32x4v*>(Uop + o) = vh * us;
                }
            }
        }
    };

    bool matched = false;
    int m = 0, nextra = 0, status = 0, tstatus = 0;
    int dpath = 0;   // diagnostic: 1 fast guess, 2 collision-resolved guess, 4 unresolved, 8 verdict failed,
                     // 32 a guessed winner failed its exact gate and its line stayed unmatched (16: sequential;
                     // 64-256: rpath)
    int par0 = 0;   // mailbox parity of line 0 on the sequential path
    bool sequential = true;
    // a restart after a failed verdict keeps the lines before the first violating one: every
    // workgroup replays them from the speculative packages (no gate, no exchange; the state, rows
    // and status bits the sequential path computes for them), then the sequential path takes over
    int keep = 0;
    // a restart after a failed verdict: the owned blocks of the guessed columns as the speculative
    // pass computed them (scan start, pending steps applied) serve the lines whose winner was guessed
    bool blk_cached = false;
    float4 (*const sh_cblk)[SCAN_THREADS] = reinterpret_cast<float4 (*)[SCAN_THREADS]>(sh_stg);

    if (spec_ok) {
        // ---- (a) guesses: per line, does the owned landmark pass under the predicted state ----
        unsigned gp = 0;
        if (own && j < s) {
            Block5 b5;
            fill_block5(b5, R33, rr0, rr1, rr2, Dj);
            Guess gs;
            guess_prep(b5, yb.x, yb.y, xp, gs);
#pragma unroll
            for (int t = 0; t < SPEC_L; t++) {
                if (t >= L) break;
                const ekf_line ln = sh_lines[t];
                double Rm[4];
                line_R(ln, t, r_mode, Rm);
                if (guess_pass(gs, ln.alpha, ln.r, Rm, p.gate)) gp |= 1u << t;
            }
            if (p.spec == 2 && L > 1)   // test hook: every guess taken from the next line
                gp = ((gp >> 1) | (gp << (L - 1))) & ((1u << L) - 1u);
            if (p.spec == 3 && L > 3) {
                // test hook: the guesses of lines L/2 .. L − 1 taken from the next of them (the
                // lines before stay right: a failed verdict keeps them)
                const int h = L / 2, nh = L - h;
                const unsigned hi = (gp >> h) & ((1u << nh) - 1u);
                gp = (gp & ((1u << h) - 1u)) | ((((hi >> 1) | (hi << (nh - 1))) & ((1u << nh) - 1u)) << h);
            }
        }
        // per wave and line the guessed candidates (ballot), then the workgroup's first SPEC_K
        // in landmark order: word A = 8-bit local indices 0..3 | count << 32 | more << 36, word B =
        // local indices 4..7
        for (int t = 0; t < L; t++) {
            const unsigned long long mk = __ballot((gp >> t) & 1u);
            if ((tid & 63) == 0 && tid < SCAN_THREADS) sh_wl[t][tid >> 6] = mk;
        }
        __syncthreads();
        if (tid < L) {
            unsigned long long word = 0, wordb = 0;
            int cnt = 0, more = 0;
            for (int w = 0; w < SCAN_THREADS / 64 && !more; w++) {
                unsigned long long mk = sh_wl[tid][w];
                while (mk) {
                    if (cnt == SPEC_K) { more = 1; break; }
                    const int b = __builtin_ctzll(mk);
                    mk &= mk - 1;
                    if (cnt < 4) word |= (unsigned long long)(w * 64 + b) << (8 * cnt);
                    else wordb |= (unsigned long long)(w * 64 + b) << (8 * (cnt - 4));
                    cnt++;
                }
            }
            word |= ((unsigned long long)cnt << LW_CNT) | ((unsigned long long)more << LW_MORE);
            sh_lists[g * SPEC_L + tid] = word;
            sh_listsb[g * SPEC_L + tid] = wordb;
        }
        __syncthreads();
        EKF_STAMP(5);
        // ---- (b) exchange 1 (parity 0): every workgroup's lists ----
        if (G > 1) {
            // self-tagged words per (workgroup, line), polled directly by their readers: A always,
            // B (at SPEC_L words further) only when A's count says it is there
            const int lb = p.mbw - MB_LIST_BACK;
            double* slot = mbox + (size_t)g * p.mbw + lb;
            if (tid < SPEC_L) {
                const unsigned long long wa = tid < L ? sh_lists[g * SPEC_L + tid] : 0ull;
                if (((wa >> LW_CNT) & 15) > 4) mb_store_tagged(slot + SPEC_L + tid, p.epoch, sh_listsb[g * SPEC_L + tid]);
                mb_store_tagged(slot + tid, p.epoch, wa);
            }
            for (int k = tid; k < G * L; k += SCAN_BLOCK) {
                const int gq = k / L, t = k - gq * L;
                if (gq != g) {
                    const double* src = mbox + (size_t)gq * p.mbw + lb;
                    const unsigned long long wa = mb_wait_tagged(src + t, p.epoch, tstatus, p.spin_log2);
                    sh_lists[gq * SPEC_L + t] = wa;
                    if (((wa >> LW_CNT) & 15) > 4)
                        sh_listsb[gq * SPEC_L + t] = mb_wait_tagged(src + SPEC_L + t, p.epoch, tstatus, p.spin_log2);
                }
            }
            __syncthreads();
        }
        EKF_STAMP(2);
        // ---- (c) guessed winners (every workgroup computes the same). Fast form: per line the
        // instance's first guessed candidate (workgroups are in landmark order); if those are
        // distinct they are the winners. Otherwise, per line the first SPEC_K guessed candidates,
        // and in line order the first one not taken by an earlier line. ----
        // per line the first guessed candidate over all workgroups: one list word per thread, an LDS
        // atomic minimum per line (sh_first, reset at the start of the kernel)
        for (int k = tid; k < G * SPEC_L; k += SCAN_BLOCK) {
            const int gq = k / SPEC_L, t = k - gq * SPEC_L;
            const unsigned long long w = sh_lists[gq * SPEC_L + t];
            if (t < L && ((w >> LW_CNT) & 15)) atomicMin(&sh_first[t], gq * SCAN_THREADS + (int)(w & 255));
        }
        __syncthreads();
        {
            int first[SPEC_L];
#pragma unroll
            for (int t = 0; t < SPEC_L; t++) first[t] = sh_first[t];
            if (tid == 0) {
                bool distinct = true;
#pragma unroll
                for (int t = 0; t < SPEC_L; t++)
#pragma unroll
                    for (int q = 0; q < t; q++)
                        distinct &= !(t < L && first[t] != 0x7fffffff && first[t] == first[q]);
#pragma unroll
                for (int t = 0; t < SPEC_L; t++) sh_spec[t] = first[t] == 0x7fffffff ? -1 : first[t];
                sh_flag = distinct ? 0 : 2;
            }
        }
        __syncthreads();
        dpath = sh_flag == 2 ? 2 : 1;
        if (sh_flag == 2) {
            if (tid < L) {
                int cnt = 0, more = 0;
                for (int gq = 0; gq < G && cnt < SPEC_K; gq++) {
                    const unsigned long long w = sh_lists[gq * SPEC_L + tid];
                    const unsigned long long wb = sh_listsb[gq * SPEC_L + tid];
                    const int c = (int)((w >> LW_CNT) & 15);
                    for (int k = 0; k < c; k++) {
                        const int loc = (int)(((k < 4 ? w : wb) >> (8 * (k & 3))) & 255);
                        if (cnt < SPEC_K) sh_glist[tid][cnt++] = gq * SCAN_THREADS + loc;
                        else more = 1;
                    }
                    if ((w >> LW_MORE) & 1) more = 1;
                }
                sh_glist[tid][SPEC_K] = cnt | (more << 8);
            }
            __syncthreads();
            if (tid == 0) {
                int spec[SPEC_L];
                int unresolved = 0;
    #pragma unroll
                for (int t = 0; t < SPEC_L; t++) {
                    spec[t] = -1;
                    if (t < L) {
                        const int info = sh_glist[t][SPEC_K];
                        const int cnt = info & 255;
                        int w = -1;
    #pragma unroll
                        for (int k = 0; k < SPEC_K; k++) {
                            const int cand = sh_glist[t][k];
                            bool taken = false;
    #pragma unroll
                            for (int q = 0; q < t; q++) taken |= (spec[q] == cand);
                            if (k < cnt && w < 0 && !taken) w = cand;
                        }
                        if (w < 0 && (info >> 8)) unresolved = 1;
                        spec[t] = w;
                    }
                }
    #pragma unroll
                for (int t = 0; t < SPEC_L; t++) sh_spec[t] = spec[t];
                sh_flag = unresolved;
            }
            __syncthreads();
        }
        EKF_STAMP(10);

        if (!sh_flag) {
            sequential = false;
            // ---- (d) the winners' records straight from memory, as their owners hold them:
            // predicted robot-strip columns and mean, diagonal block, blocks of the earlier
            // winners' columns; and (staged replay) the guessed columns' rows of the pending
            // steps' operands ----
            // staged path: everything below is issued before one barrier, so that the stored
            // blocks of the owned row (landmark waves), the winners' records and mutual blocks
            // (replay wave) and the staged operand rows arrive in one memory round trip
            int cols[SPEC_L];
#pragma unroll
            for (int t = 0; t < SPEC_L; t++) {
                const int w = t < L ? sh_spec[t] : -1;
                cols[t] = w >= 0 ? w : j;
            }
            // per guessed winner t (lane t of every wave): the latest pending step that added it,
            // or -1; read with __shfl, so that no wave waits for another's (the MFMA-replay path
            // has no barrier between the records and the waves' replays)
            int addq_l = -1;
            if (mf && aug_pend) {
                const int lt = tid & 63;
                const int w = lt < L ? sh_spec[lt] : -1;
                if (w >= 0)
                    for (int q = 0; q < p.npend; q++)
                        if (w >= sh_ctl[q].w && w < sh_ctl[q].w + sh_ctl[q].z) addq_l = q;
            }
            C srow[SPEC_L + 1][4];
            if ((staged || m64) && own) staged_blocks_load<T>(pv, j, cols, srow);
            int pu = 0, pt = 0;   // replay-wave lane → mutual block (pu, pt), pt <= pu
            C pacc[4] = {0, 0, 0, 0};
            const int lane_r = tid - SCAN_THREADS;
            // fp64 MFMA-replay contexts: the winners' mutual blocks from their U and V rows of every
            // pending step staged in LDS (m64s, below) instead of a memory round trip per step
            const bool m64s = m64 && p.npend <= M64_QMAX;
            if ((staged || m64s) && tid >= SCAN_THREADS && lane_r < L * (L + 1) / 2) {
                pt = lane_r;
                while (pt > pu) { pt -= pu + 1; pu++; }
                if (sh_spec[pu] >= 0 && sh_spec[pt] >= 0) pair_block_load<T>(pv, sh_spec[pu], sh_spec[pt], pacc);
            }
            if constexpr (sizeof(C) == 8)
                if (m64s) {
                    // rows 2w, 2w + 1 of U_q and V_q of every guessed winner w and pending step q,
                    // all loads in flight together: pieces of 4 doubles (k = 16·kk + s, s < 4, as
                    // pll_blocks reads them), [t][q][U, V][row][kk][s] (m64_stage_index), in history
                    // slots 1.. (unused until the line loop's second match; slot 0 holds the
                    // landmark waves' diagonal blocks meanwhile, the fp32 stage is not allocated here)
                    static_assert((HIST_LDS - 1) * SCAN_THREADS * sizeof(double4) >= SPEC_L * M64_QMAX * 64 * sizeof(double),
                                  "fp64 winners' stage");
                    double* stg64 = reinterpret_cast<double*>(&sh_uhist[1][0]);
                    typedef double d64x2 __attribute__((ext_vector_type(2)));
                    const int nld = L * p.npend * 16;
                    for (int k = tid; k < nld; k += SCAN_BLOCK) {
                        const int piece = k & 15, tq = k >> 4, q = tq % p.npend, t = tq / p.npend;
                        const int w = sh_spec[t];
                        if (w < 0 || sh_ctl[q].y <= 0) continue;
                        const int uv = piece >> 3, rr = (piece >> 2) & 1, kk = piece & 3;
                        const int r = 2 * w + rr;
                        const double* base = reinterpret_cast<const double*>(uv ? p.pend[q].Vop : p.pend[q].Uop) + e * opstride;
                        const d64x2* src = reinterpret_cast<const d64x2*>(
                            base + ((size_t)(r >> 5) * 64 + (r & 15)) * 8 + ((r >> 4) & 1) * 4 + 128 * kk);
                        d64x2* dst = reinterpret_cast<d64x2*>(stg64 + m64_stage_index(t, q, uv, rr, kk));
                        dst[0] = src[0];
                        dst[1] = src[1];
                    }
                }
            if (!staged && !m64s && tid < L * (L + 1) / 2) {
                int u = 0, t = tid;
                while (t > u) { t -= u + 1; u++; }
                const int wu = sh_spec[u], wt = sh_spec[t];
                if (wu >= 0 && wt >= 0) {
                    double bk[4];
                    pll_block(pv, 2 * wu, 2 * wt, bk);
                    double* r = sh_wd + u * SPEC_WD + (t == u ? 6 : 14 + 4 * t);
                    r[0] = bk[0]; r[1] = bk[1]; r[2] = bk[2]; r[3] = bk[3];
                }
            }
            if (tid >= SCAN_THREADS && tid < SCAN_THREADS + L) {
                const int u = tid - SCAN_THREADS, wu = sh_spec[u];
                if (wu >= 0) {
                    const int bw = 3 + 2 * wu;
                    double2 q0 = *reinterpret_cast<const double2*>(Rs + bw);
                    double2 q1 = *reinterpret_cast<const double2*>(Rs + n + bw);
                    double2 q2 = *reinterpret_cast<const double2*>(Rs + 2 * n + bw);
                    const double2 qy = *reinterpret_cast<const double2*>(y + bw);
                    if (p.phase & PHASE_PREDICT) predict_cols(F3, q0, q1, q2);
                    double* r = sh_wd + u * SPEC_WD;
                    r[0] = q0.x; r[1] = q0.y; r[2] = q1.x; r[3] = q1.y; r[4] = q2.x; r[5] = q2.y;
                    r[10] = qy.x; r[11] = qy.y;   // (sin/cos of the angle: by the replay wave, after the barrier)
                }
            }
            if (staged && !mf) {
                // rows 2w, 2w+1 of U_q and V_q of every guessed column w, pending step q (4 row
                // halves × 8 k each; the V side interleaved, stage_v_index): 16 pieces of 4 floats
                const int kh = d.kmax / 2;
                const int nld = L * p.npend * 16;
                for (int k = tid; k < nld; k += SCAN_BLOCK) {
                    const int piece = k & 15, tq = k >> 4, q = tq % p.npend, t = tq / p.npend;
                    const int w = sh_spec[t];
                    if (w < 0) continue;
                    const size_t rowb = ((size_t)((2 * w) >> 5) * 64 + ((2 * w) & 31)) * kh;
                    float* dst = sh_stg + ((t * SPEC_QMAX + q) * 2) * 32;
                    if (piece < 8) {   // U: row half rh, 4 k
                        const int half = piece & 1, rh = piece >> 1;
                        const float* base = u_rows_f32(pv, p.pend[q]) + rowb;
                        const int roff = (rh & 1) * kh + (rh >> 1) * 32 * kh;
                        *reinterpret_cast<f32x4v*>(dst + rh * 8 + half * 4) =
                            *reinterpret_cast<const f32x4v*>(base + roff + half * 4) * pv.us;
                    } else {           // V: rows of pair pr, k-pairs 2kc, 2kc + 1, interleaved
                        const int pr = (piece - 8) >> 2, kc = (piece - 8) & 3;
                        const float* base = reinterpret_cast<const float*>(p.pend[q].Vop) + e * opstride + rowb;
                        const f32x2v a = *reinterpret_cast<const f32x2v*>(base + (2 * pr) / 2 * 32 * kh + 2 * kc);
                        const f32x2v c = *reinterpret_cast<const f32x2v*>(base + kh + pr * 32 * kh + 2 * kc);
                        *reinterpret_cast<f32x4v*>(dst + 32 + pr * 16 + 4 * kc) = f32x4v{a[0], c[0], a[1], c[1]};
                    }
                }
            }
            // the guessed winners' addition steps of this lane's mutual block (the replay wave), and of
            // every guessed column (the landmark waves): shuffles with the whole wave active
            const int qs_pair = mf && aug_pend ? max(__shfl(addq_l, pu, 64), __shfl(addq_l, pt, 64)) : -1;
            int addq_t[SPEC_L];
#pragma unroll
            for (int t = 0; t < SPEC_L; t++) addq_t[t] = mf && aug_pend ? __shfl(addq_l, t, 64) : -1;
            // MFMA replay (mf): no barrier here. Each wave reads only what it wrote itself or what
            // an earlier barrier published — the replay wave its winners' records (sh_wd), the
            // landmark waves their owned rows' blocks — so the landmark waves replay the pending
            // steps while the replay wave loads the records and replays the winners' mutual blocks,
            // and its chain starts without waiting for them (the packages and the winners' V rows
            // then reach the landmark waves through sh_ready, release / acquire)
            if (!mf) __syncthreads();
            if (mf && tid >= SCAN_THREADS) {
              if constexpr (kPlanes) {
                // the winners' mutual blocks: X minus the pending steps' ΔX of the 16 winner rows
                // against themselves (one M-block of plane_replay), by the replay wave itself
                auto wrow = [&](int c) {
                    const int t = c >> 1;
                    const int w = t < L ? sh_spec[t] : -1;
                    return w >= 0 ? 2 * w + (c & 1) : -1;
                };
                f32x4v dacc[1];
                if (f32rep)
                    f32_replay<1>(p.pend, e, opstride, M, amask, lane_r, [&](int, int r) { return wrow(r); }, wrow, dacc);
                else if (HOT == 2 || (HOT == 0 && pf16))
                    plane_replay<1, true, 4>(p.pend, e, opstride * 2, M, amask, lane_r, [&](int, int r) { return wrow(r); }, wrow, dacc);
                else
                    plane_replay<1, false, 4>(p.pend, e, opstride * 3, M, amask, lane_r, [&](int, int r) { return wrow(r); }, wrow, dacc);
                float* scr = sh_stg;   // (not staged in this mode) 16 × 16 floats
#pragma unroll
                for (int i = 0; i < 4; i++) scr[(4 * (lane_r >> 4) + i) * 16 + (lane_r & 15)] = dacc[0][i];
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                if (lane_r < L * (L + 1) / 2 && sh_spec[pu] >= 0 && sh_spec[pt] >= 0) {
                    const bool swap = ((2 * sh_spec[pu]) >> 5) > ((2 * sh_spec[pt]) >> 5);
                    C xr[4] = {pacc[0], swap ? pacc[2] : pacc[1], swap ? pacc[1] : pacc[2], pacc[3]};
                    const int qs = qs_pair;   // (as for the landmark waves' blocks)
                    if (qs >= 0) patch_block<T>(pv, p.pend[qs], sh_ctl[qs], 2 * sh_spec[pu], 2 * sh_spec[pt], false, xr);
                    double* r = sh_wd + pu * SPEC_WD + (pt == pu ? 6 : 14 + 4 * pt);
#pragma unroll
                    for (int a = 0; a < 4; a++)
                        r[a] = from_domain<T>(xr[a], pv.ex) - (double)scr[(2 * pu + (a >> 1)) * 16 + 2 * pt + (a & 1)] * rrsc;
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
              }
            } else if ((staged || m64s) && tid >= SCAN_THREADS) {
                // the winners' mutual blocks from the staged rows, by the replay wave itself
                // (only it reads them): the landmark waves go straight on
                if (lane_r < L * (L + 1) / 2 && sh_spec[pu] >= 0 && sh_spec[pt] >= 0) {
                    double bk[4];
                    if constexpr (sizeof(C) == 8)
                        m64_pair_block<T>(pv, sh_spec[pu], pu, sh_spec[pt], pt,
                                          reinterpret_cast<const double*>(&sh_uhist[1][0]), pacc, bk);
                    else
                        staged_pair_block<T>(pv, sh_spec[pu], pu, sh_spec[pt], pt, sh_stg, pacc, bk);
                    double* r = sh_wd + pu * SPEC_WD + (pt == pu ? 6 : 14 + 4 * pt);
                    r[0] = bk[0]; r[1] = bk[1]; r[2] = bk[2]; r[3] = bk[3];
                }
                __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                __builtin_amdgcn_wave_barrier();
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            }
            EKF_STAMP(12);
            __shared__ unsigned long long sh_trec;   // diagnostics: the records' end (thread 0, WG 0)
            if (dbg) sh_trec = t_last;
            // ---- (f) the winners' part of the sequential chain, in the last wave (lane u carries
            // winner u's rows): per line the winner's lane evaluates it and writes the package,
            // then the later winners' lanes apply their gain rows. Meanwhile (g) the landmark
            // waves run every line as soon as its package is published (sh_ready). ----
            int viol = 0;
            int vline = L;   // the line of this thread's violation
            int stp = 0;     // its status bits per line (st_line)
            if (tid >= SCAN_THREADS) {
                const int u = tid - SCAN_THREADS;
                const unsigned long long t_l0 = __builtin_amdgcn_s_memrealtime();
                const bool act = u < L && sh_spec[u] >= 0;
                double R33l[9], xpl[3];
#pragma unroll
                for (int a = 0; a < 9; a++) R33l[a] = R33[a];
                xpl[0] = xp[0]; xpl[1] = xp[1]; xpl[2] = xp[2];
                double2 w0 = make_double2(0, 0), w1 = w0, w2 = w0, wy = w0;
                double wD[4] = {0, 0, 0, 0};
                double wma0 = 0.0, ws0 = 0.0, wc0 = 1.0;
                if (act) {
                    const double* r = sh_wd + u * SPEC_WD;
                    w0 = make_double2(r[0], r[1]); w1 = make_double2(r[2], r[3]);
                    w2 = make_double2(r[4], r[5]); wy = make_double2(r[10], r[11]);
                    wD[0] = r[6]; wD[1] = r[7]; wD[2] = r[8]; wD[3] = r[9];
                    wma0 = r[10];
                    sincos(wma0, &ws0, &wc0);   // sincos_near's scan-start values (as the owner's)
                }
                int ml = 0;
                const bool lst = pdbg && g == 0 && u == 0;
                unsigned long long tl = lst ? __builtin_amdgcn_s_memrealtime() : 0ull;
                // lane u evaluates line u: its line in registers, and the lines with a winner as a
                // wave-uniform mask (no LDS read on the chain)
                ekf_line lnu = {};
                if (u < L) lnu = sh_lines[u];
                const unsigned long long wmask = __ballot(act);
                for (int t = 0; t < L; t++) {
                    if (!((wmask >> t) & 1ull)) continue;
                    double* pk = sh_pk[t];
                    int okl = 1;
                    Cand c;
                    Block5 b5;
                    if (u == t) {
                        const ekf_line ln = lnu;
                        double Rm[4];
                        line_R(ln, t, r_mode, Rm);
                        fill_block5(b5, R33l, w0, w1, w2, wD);
                        double sn, cs;
                        sincos_near(wy.x, wma0, ws0, wc0, sn, cs);
                        // (its storage-precision margin and GSL_EDOM status after the package is out)
                        eval_candidate<false>(b5, wy.x, wy.y, sn, cs, xpl, ln.alpha, ln.r, Rm, p.gate, ETA, c);
                        okl = c.pass ? 1 : 0;
                        pk[PK_OK] = okl ? 1.0 : 0.0;
                    }
                    // the guessed winner failed its exact gate: no update from this line (the
                    // landmark waves check that no other landmark passes it)
                    const int ok = __builtin_amdgcn_readlane(okl, t);
                    if (ok && u == t) {
                        // the package in registers, the robot block after the line from it (for
                        // every lane and every landmark wave), then all of it to LDS
                        double pkl[PKW];
                        build_package(c, R33l, w0, w1, w2, pkl);   // its V rows stay in sh_wh[t]
                        robot_update(R33l, xpl, pkl);
#pragma unroll
                        for (int a = 0; a < 9; a++) pkl[PK_R33 + a] = R33l[a];
                        pkl[PK_XP + 0] = xpl[0]; pkl[PK_XP + 1] = xpl[1]; pkl[PK_XP + 2] = xpl[2];
                        // (the robot rows of K stay in registers: only robot_update, here, reads them;
                        // the symmetric operand factor is the landmark waves' own, from S)
#pragma unroll
                        for (int a = MB_S; a < PK_F; a++)
                            if (a < MB_KR || a >= MB_KR + 6) pk[a] = pkl[a];
                    }
                    // the package is complete: to the other lanes of this wave, and to the
                    // landmark waves (release of lane t's LDS writes, then the line counter)
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    if (u == 0) __hip_atomic_store(&sh_ready, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
                    if (u == t) {
                        // GSL_EDOM of the winner (the reference evaluated it: Robot.cpp:454) and the
                        // gate's storage precision (gate_eta), off the line's chain
                        if (c.singular) atomicOr(&sh_rwst, st_line(EKF_ST_SINGULAR, t));
                        if (cand_amb(b5, c, p.gate, ETA)) atomicOr(&sh_rwst, st_line(EKF_ST_PRECISION_BIT, t));
                    }
                    if (!ok) continue;   // (ml counts matches: unchanged)
                    if (u != t) {   // (lane t has them)
#pragma unroll
                        for (int a = 0; a < 9; a++) R33l[a] = pk[PK_R33 + a];
                        xpl[0] = pk[PK_XP + 0]; xpl[1] = pk[PK_XP + 1]; xpl[2] = pk[PK_XP + 2];
                    }
                    if (lst) { const unsigned long long t2 = __builtin_amdgcn_s_memrealtime(); sh_stamp[3] += t2 - tl; tl = t2; }
                    if (act && u > t) {
                        const double* r = sh_wd + u * SPEC_WD + 14 + 4 * t;
                        double blk[4] = {r[0], r[1], r[2], r[3]};
                        double kk[4], uu[4];
                        gain_rows<SPEC_L>(pk, ml, [&](int q) { return sh_wh[u][q][0]; },
                                          [&](int q) { return sh_wh[t][q][1]; }, blk, w0, w1, w2, wy, wD, kk, uu);
                        sh_wh[u][ml][0] = make_double4(uu[0], uu[1], uu[2], uu[3]);
                        sh_wh[u][ml][1] = make_double4(kk[0], kk[1], kk[2], kk[3]);
                    }
                    ml++;
                    if (lst) { const unsigned long long t2 = __builtin_amdgcn_s_memrealtime(); sh_stamp[4] += t2 - tl; tl = t2; }
                }
                if (u == 0) {
                    sh_flag = 0;   // (a failed guessed winner is settled per line by the landmark waves)
                    if (pdbg && g == 0) {
                        const unsigned long long te = __builtin_amdgcn_s_memrealtime();
                        sh_stamp[13] += te - t_l0;
                        sh_stamp[29] += t_l0 - sh_trec;   // the replay wave's chain starts ...
                        sh_stamp[30] += te - sh_trec;     // ... and ends, after the records
                    }
                }
            } else {
                // ---- (e) owned blocks of the guessed columns (Robot.cpp:560 operands), while the
                // last wave runs (f) ----
                if (mf) {
                  if constexpr (kPlanes) {
                    // the owned rows' blocks of the guessed columns: X minus the pending steps' ΔX
                    // of the wave's 128 rows (8 M-blocks) against the 16 winner rows, transposed
                    // through this wave's part of sh_vpl (8 KB; the planes are staged there later)
                    const int l = tid & 63;
                    const int rbase = 2 * (g * SCAN_THREADS + (tid & ~63));
                    auto wrow = [&](int c) {
                        const int t = c >> 1;
                        const int w = t < L ? sh_spec[t] : -1;
                        return w >= 0 ? 2 * w + (c & 1) : -1;
                    };
                    f32x4v dacc[8];
                    if (f32rep)
                        f32_replay<8>(p.pend, e, opstride, M, amask, l,
                                      [&](int mb, int r) { return rbase + 16 * mb + r; }, wrow, dacc);
                    else if (HOT == 2 || (HOT == 0 && pf16))
                        plane_replay<8, true>(p.pend, e, opstride * 2, M, amask, l,
                                              [&](int mb, int r) { return rbase + 16 * mb + r; }, wrow, dacc);
                    else
                        plane_replay<8, false>(p.pend, e, opstride * 3, M, amask, l,
                                               [&](int mb, int r) { return rbase + 16 * mb + r; }, wrow, dacc);
                    float* scr = sh_vpl + (tid & ~63) * 32;
#pragma unroll
                    for (int mb = 0; mb < 8; mb++)
#pragma unroll
                        for (int i = 0; i < 4; i++) scr[(mb * 16 + 4 * (l >> 4) + i) * 16 + (l & 15)] = dacc[mb][i];
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    if (own) {
                        const float* r0 = scr + ((l >> 3) * 16 + ((2 * l) & 15)) * 16;
                        f32x4v d0[4], d1[4];
#pragma unroll
                        for (int k = 0; k < 4; k++) {
                            d0[k] = *reinterpret_cast<const f32x4v*>(r0 + 4 * k);
                            d1[k] = *reinterpret_cast<const f32x4v*>(r0 + 16 + 4 * k);
                        }
                        // a block touching a landmark added during the pending steps starts from
                        // the patch of the step that added the later of its two landmarks (the
                        // higher index: landmarks are appended); the replay's ΔX holds only the
                        // steps after it (their V rows are zero before)
                        int qj = -1;
                        if (aug_pend)
                            for (int q = 0; q < p.npend; q++)
                                if (j >= sh_ctl[q].w && j < sh_ctl[q].w + sh_ctl[q].z) qj = q;
#pragma unroll
                        for (int t = 0; t < SPEC_L; t++)
                            if (t < L && sh_spec[t] >= 0) {
                                C b[4] = {srow[t][0], srow[t][1], srow[t][2], srow[t][3]};
                                const int qs = max(qj, addq_t[t]);
                                if (qs >= 0) patch_block<T>(pv, p.pend[qs], sh_ctl[qs], 2 * j, 2 * sh_spec[t], false, b);
                                const int c0 = 2 * t;
                                sh_blk[t][tid] = make_float4(
                                    (float)(from_domain<T>(b[0], pv.ex) - (double)d0[c0 >> 2][c0 & 3] * rrsc),
                                    (float)(from_domain<T>(b[1], pv.ex) - (double)d0[c0 >> 2][(c0 & 3) + 1] * rrsc),
                                    (float)(from_domain<T>(b[2], pv.ex) - (double)d1[c0 >> 2][c0 & 3] * rrsc),
                                    (float)(from_domain<T>(b[3], pv.ex) - (double)d1[c0 >> 2][(c0 & 3) + 1] * rrsc));
                            }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                  }
                } else if (m64) {
                  if constexpr (sizeof(C) == 8) {
                    // fp64: the wave's 128 owned rows (8 M-blocks of 16) against the 16 winner rows
                    // and against themselves (their diagonal blocks), one v_mfma_f64_16x16x4f64 per
                    // M-block and k-chunk on the flush's operand rows in the flush's k order: per
                    // element the flush's own chain, bit for bit. A block stored transposed (the
                    // winner's tile row first) evolves as U_col·V_own: each k-chunk runs both
                    // products with the other one's winner column zeroed (it adds ±0). The chains
                    // start from the stored blocks (srow), handed from the owner threads to the MFMA
                    // lanes and back through LDS: sh_blk64 (winners) and sh_uhist[0] (diagonal
                    // blocks).
                    typedef double d64x2 __attribute__((ext_vector_type(2)));
                    typedef double d64x4 __attribute__((ext_vector_type(4)));
                    constexpr int KH = 8;   // doubles per lane and row block (kmax = 16)
                    const int l = tid & 63;
                    const int wb = tid & ~63;                          // the wave's first thread
                    const int rb0 = (2 * (g * SCAN_THREADS + wb)) >> 5;   // its first tile row (4 of them)
                    double4* dg = sh_uhist[0];   // (this wave's part: free until its first match)
                    if (own) {
#pragma unroll
                        for (int t = 0; t < SPEC_L; t++) sh_blk64[t][tid] = make_double4(srow[t][0], srow[t][1], srow[t][2], srow[t][3]);
                        dg[tid] = make_double4(srow[SPEC_L][0], srow[SPEC_L][1], srow[SPEC_L][2], srow[SPEC_L][3]);
                    } else {
#pragma unroll
                        for (int t = 0; t < SPEC_L; t++) sh_blk64[t][tid] = make_double4(0, 0, 0, 0);
                        dg[tid] = make_double4(0, 0, 0, 0);
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    // this lane's winner column c = l % 16: row wr of winner t = c / 2 (B operands
                    // hold column l % 16 at k-offset l / 16, A operands row l % 16)
                    const int c = l & 15, t = c >> 1;
                    const int wsp = t < L ? sh_spec[t] : -1;
                    const int wr = wsp >= 0 ? 2 * wsp + (c & 1) : 0;
                    const size_t coff = (size_t)(wr >> 5) * 64 * KH + ((wr & 15) + 16 * (l >> 4)) * KH + ((wr >> 4) & 1) * 4;
                    auto comp = [](double4& v, int k) -> double& { return reinterpret_cast<double*>(&v)[k]; };
                    // two tile rows per pass, the pending steps inside: each step's operand loads of
                    // both row blocks are in flight together (a memory round trip per step and pair,
                    // not per step and tile row); per accumulator the same MFMA sequence
#pragma unroll 1
                    for (int r2 = 0; r2 < 4; r2 += 2) {
                        // (the last workgroup's waves may reach past the landmark block: no rows,
                        // no operand rows there)
                        if (rb0 + r2 >= d.nb) break;
                        const bool two = rb0 + r2 + 1 < d.nb;   // (uniform)
                        bool sw[2], nsw[2];
                        d64x4 acc[2][2], dac[2][2];
#pragma unroll
                        for (int x = 0; x < 2; x++) {
                            const int r4 = r2 + x, rb = rb0 + r4;
                            sw[x] = wsp >= 0 && rb > (wr >> 5);   // stored transposed
                            nsw[x] = wsp >= 0 && !sw[x];
#pragma unroll
                            for (int h = 0; h < 2; h++)
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const int rl = 32 * r4 + 16 * h + 4 * i + (l >> 4);   // row in the wave (tile_off_f64)
                                    const int ow = wb + (rl >> 1);
                                    acc[x][h][i] = comp(sh_blk64[t][ow], (rl & 1) * 2 + (c & 1));
                                    const int cl = 32 * r4 + 16 * h + c;
                                    dac[x][h][i] = (rl >> 1) == (cl >> 1) ? comp(dg[ow], (rl & 1) * 2 + (cl & 1)) : 0.0;
                                }
                        }
                        for (int q = 0; q < p.npend; q++) {
                            if (sh_ctl[q].y <= 0) continue;   // no match, or rolled back: nothing
                            const double* Uq = reinterpret_cast<const double*>(p.pend[q].Uop) + e * opstride;
                            const double* Vq = reinterpret_cast<const double*>(p.pend[q].Vop) + e * opstride;
                            d64x2 ua[2][4], va[2][4], cu[2], cv[2];
#pragma unroll
                            for (int x = 0; x < 2; x++) {
                                // (a second row block past the landmark block re-reads the first)
                                const int rb = rb0 + r2 + (two ? x : 0);
                                const d64x2* uo = reinterpret_cast<const d64x2*>(Uq + (size_t)rb * 64 * KH + l * KH);
                                const d64x2* vo = reinterpret_cast<const d64x2*>(Vq + (size_t)rb * 64 * KH + l * KH);
#pragma unroll
                                for (int k = 0; k < 4; k++) { ua[x][k] = uo[k]; va[x][k] = vo[k]; }
                            }
#pragma unroll
                            for (int k = 0; k < 2; k++) {
                                cu[k] = reinterpret_cast<const d64x2*>(Uq + coff)[k];
                                cv[k] = reinterpret_cast<const d64x2*>(Vq + coff)[k];
                            }
#pragma unroll
                            for (int x = 0; x < 2; x++)
#pragma unroll
                                for (int s4 = 0; s4 < 4; s4++) {
                                    const double bv = nsw[x] ? cv[s4 >> 1][s4 & 1] : 0.0;
                                    const double bu = sw[x] ? cu[s4 >> 1][s4 & 1] : 0.0;
#pragma unroll
                                    for (int h = 0; h < 2; h++) {
                                        const double au = ua[x][2 * h + (s4 >> 1)][s4 & 1];
                                        const double av = va[x][2 * h + (s4 >> 1)][s4 & 1];
                                        acc[x][h] = __builtin_amdgcn_mfma_f64_16x16x4f64(au, bv, acc[x][h], 0, 0, 0);
                                        acc[x][h] = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bu, acc[x][h], 0, 0, 0);
                                        dac[x][h] = __builtin_amdgcn_mfma_f64_16x16x4f64(au, av, dac[x][h], 0, 0, 0);
                                    }
                                }
                        }
                        __builtin_amdgcn_wave_barrier();   // (every lane read its starting values)
#pragma unroll
                        for (int x = 0; x < 2; x++) {
                            if (x == 1 && !two) break;
                            const int r4 = r2 + x;
#pragma unroll
                            for (int h = 0; h < 2; h++)
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const int rl = 32 * r4 + 16 * h + 4 * i + (l >> 4);
                                    const int ow = wb + (rl >> 1);
                                    comp(sh_blk64[t][ow], (rl & 1) * 2 + (c & 1)) = acc[x][h][i];
                                    const int cl = 32 * r4 + 16 * h + c;
                                    if ((rl >> 1) == (cl >> 1)) comp(dg[ow], (rl & 1) * 2 + (cl & 1)) = dac[x][h][i];
                                }
                        }
                    }
                    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
                    __builtin_amdgcn_wave_barrier();
                    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
                    if (own && j < s) {
                        const double4 dd = dg[tid];
                        Dj[0] = dd.x; Dj[1] = dd.y; Dj[2] = dd.z; Dj[3] = dd.w;
                    }
                  }
                } else if (own) {
                    if (staged) {
                        double blk[SPEC_L + 1][4];
                        staged_blocks<T>(pv, j, cols, sh_stg, srow, blk);
#pragma unroll
                        for (int t = 0; t < SPEC_L; t++)
                            if (t < L && sh_spec[t] >= 0)
                                sh_blk[t][tid] = make_float4((float)blk[t][0], (float)blk[t][1], (float)blk[t][2], (float)blk[t][3]);
                        if (j < s) {
                            Dj[0] = blk[SPEC_L][0]; Dj[1] = blk[SPEC_L][1];
                            Dj[2] = blk[SPEC_L][2]; Dj[3] = blk[SPEC_L][3];
                        }
                    } else if constexpr (sizeof(typename Stor<T>::C) == 4) {
                        for (int t0 = 0; t0 < L; t0 += SPEC_PB) {
                            int cols[SPEC_PB];
                            double bk[SPEC_PB][4];
#pragma unroll
                            for (int b = 0; b < SPEC_PB; b++) {
                                const int w = (t0 + b < L) ? sh_spec[t0 + b] : -1;
                                cols[b] = 2 * (w >= 0 ? w : j);
                            }
                            pll_blocks<T, SPEC_PB>(pv, 2 * j, cols, bk);
#pragma unroll
                            for (int b = 0; b < SPEC_PB; b++)
                                if (t0 + b < L && sh_spec[t0 + b] >= 0)
                                    sh_blk[t0 + b][tid] = make_float4((float)bk[b][0], (float)bk[b][1], (float)bk[b][2], (float)bk[b][3]);
                        }
                    } else {
                        // fp64 operands: the same blocks in fp64, ahead of the line loop (they used
                        // to be read, pending steps replayed, inside it: a memory round trip per
                        // line on the landmark waves' chain)
                        for (int t0 = 0; t0 < L; t0 += SPEC_PB64) {
                            int cols[SPEC_PB64];
                            double bk[SPEC_PB64][4];
#pragma unroll
                            for (int b = 0; b < SPEC_PB64; b++) {
                                const int w = (t0 + b < L) ? sh_spec[t0 + b] : -1;
                                cols[b] = 2 * (w >= 0 ? w : j);
                            }
                            pll_blocks<T, SPEC_PB64>(pv, 2 * j, cols, bk);
#pragma unroll
                            for (int b = 0; b < SPEC_PB64; b++)
                                if (t0 + b < L && sh_spec[t0 + b] >= 0)
                                    sh_blk64[t0 + b][tid] = make_double4(bk[b][0], bk[b][1], bk[b][2], bk[b][3]);
                        }
                    }
                }
                EKF_STAMP(11);
                // ---- (g) the landmark waves: the sequential gating and gain rows against the
                // packages ----
                unsigned long long tq = dbg ? __builtin_amdgcn_s_memrealtime() : 0ull;
                auto sub = [&](int k) {
                    if (dbg) {
                        const unsigned long long t2 = __builtin_amdgcn_s_memrealtime();
                        sh_stamp[k] += t2 - tq;
                        tq = t2;
                    }
                };
                for (int i = 0; i < L && !viol; ++i) {
                    const ekf_line ln = sh_lines[i];
                    double Rm[4];
                    line_R(ln, i, r_mode, Rm);
                    const int w = __builtin_amdgcn_readfirstlane(sh_spec[i]);   // uniform: scalar branches, m scalar
                    int deep = 0;   // diagnostics: 1 past the quick filter, 2 past the fp32 one, 3 past the fp64 one
                    // the gate of line i on the state before it (the guessed winner itself, j == w, is
                    // evaluated exactly by the replay wave, which reports the result in the package
                    // (PK_OK) and its GSL_EDOM in sh_rwst; a failed winner leaves the line unmatched
                    // unless another landmark passes, which flags a violation). Its first filter runs in one block with the line's gain rows,
                    // which do not depend on it: two independent chains for the scheduler to interleave
                    const bool cand = own && j < s && !matched && j != w;
                    Block5 b5;
                    fill_block5(b5, R33, rr0, rr1, rr2, Dj);
                    const double ybx = yb.x, yby = yb.y;
                    const double xpg[3] = {xp[0], xp[1], xp[2]};
                    bool deeper = false;
                    const double* pk = nullptr;
                    bool wok = true;   // the guessed winner passed its exact gate (PK_OK)
                    if (w >= 0) {
                        int polls = 0;
                        while (__hip_atomic_load(&sh_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= i) {
                            __builtin_amdgcn_s_sleep(1);
                            if ((tstatus & EKF_ST_TIMEOUT_BIT) || ++polls > (1 << p.spin_log2)) { tstatus |= EKF_ST_TIMEOUT_BIT; viol = 1; vline = i; break; }
                        }
                        sub(17);
                        pk = sh_pk[i];
                        wok = __builtin_amdgcn_readfirstlane(pk[PK_OK] != 0.0 ? 1 : 0) != 0;
                        if (r_mode == 1 && (i == 1 || i == 2) && wok) stp |= st_line(EKF_ST_NSYM, i);
                        if (own) {
                            // the quick filter and the gain rows in one block (independent chains);
                            // the gain rows take effect only if the guessed winner passed (wok,
                            // uniform; otherwise the package words are not written)
                            deeper = cand && !quick_reject(b5, ybx, yby, ma0, s0f, c0f, xpg, ln.alpha, ln.r, Rm, p.gate, ETA);
                            double blk[4];
                            if constexpr (sizeof(typename Stor<T>::C) == 4) {
                                const float4 bk = sh_blk[i][tid];
                                blk[0] = bk.x; blk[1] = bk.y; blk[2] = bk.z; blk[3] = bk.w;
                            } else {
                                const double4 bk = sh_blk64[i][tid];
                                blk[0] = bk.x; blk[1] = bk.y; blk[2] = bk.z; blk[3] = bk.w;
                            }
                            double kk[4], uu[4];
                            double2 g0 = rr0, g1 = rr1, g2 = rr2, gy = yb;
                            double gD[4] = {Dj[0], Dj[1], Dj[2], Dj[3]};
                            gain_rows<SPEC_L>(pk, m, [&](int q) { return sh_uhist[q][tid]; },   // m < SPEC_L = HIST_LDS
                                              [&](int q) { return sh_wh[i][q][1]; }, blk, g0, g1, g2, gy, gD, kk, uu);
                            if (wok) {
                                rr0 = g0; rr1 = g1; rr2 = g2; yb = gy;
                                Dj[0] = gD[0]; Dj[1] = gD[1]; Dj[2] = gD[2]; Dj[3] = gD[3];
                                float F[3];
                                sym_factor(pk, F);   // (the same bits as the replay wave's S gives)
                                store_rows(m, kk, uu, false, F, true);
                            }
                        }
                        sub(18);
                    } else {
                        deeper = cand && !quick_reject(b5, ybx, yby, ma0, s0f, c0f, xpg, ln.alpha, ln.r, Rm, p.gate, ETA);
                    }
                    if (deeper) {   // rare: the certified fp32 and fp64 filters, then the exact evaluation
                        deep = 1;
                        bool pass = false;
                        double sn = 0.0, cs = 1.0;
                        if (!certified_reject_f32(b5, ybx, yby, xpg, ln.alpha, ln.r, Rm, p.gate, ETA) &&
                            (deep = 2, exact_sc(), sincos_near(ybx, ma0, s0j, c0j, sn, cs),
                             !certified_reject(b5, ybx, yby, sn, cs, xpg, ln.alpha, ln.r, Rm, p.gate, ETA))) {
                            deep = 3;
                            Cand c;
                            eval_candidate(b5, ybx, yby, sn, cs, xpg, ln.alpha, ln.r, Rm, p.gate, ETA, c);
                            // GSL_EDOM counts only for candidates the reference evaluates: the
                            // unmatched ones up to the winner (Robot.cpp:313-498 stops there)
                            if (c.singular && (w < 0 || !wok || j <= w)) stp |= st_line(EKF_ST_SINGULAR, i);
                            if (c.amb && (w < 0 || !wok || j <= w)) stp |= st_line(EKF_ST_PRECISION_BIT, i);
                            pass = c.pass;
                        }
                        // the guess must be the first passing unmatched landmark; a guessed
                        // winner that failed leaves the line unmatched only if none passes
                        if (pass && (w < 0 || !wok || j < w)) {
                            viol = 1;
                            vline = i;
                        }
                    }
                    if (pdbg && g == 0) {   // waves of workgroup 0 whose lanes went deeper
                        const bool d1 = __any(deep >= 1), d2 = __any(deep >= 2), d3 = __any(deep >= 3);
                        if ((tid & 63) == 0) {
                            if (d1) atomicAdd(&sh_stamp[20], 1ull);
                            if (d2) atomicAdd(&sh_stamp[21], 1ull);
                            if (d3) atomicAdd(&sh_stamp[23], 1ull);
                            atomicAdd(&sh_stamp[22], 1ull);
                        }
                    }
                    sub(16);
                    if (w < 0 || !wok) {
                        // no match: the line goes to extraLines (Robot.cpp:308-310, 492-496)
                        if (w >= 0) dpath |= 32;   // diagnostics: a guessed winner failed, line unmatched
                        if (lead) {
                            res[RES_MATCH + i] = -1;
                            res[RES_EXTRA + nextra] = i;
                        }
                        if (tid == 0) sh_extra[nextra] = i;
                        nextra++;
                        continue;
                    }
                    // = robot_update(R33, xp, pk), computed by the replay wave
#pragma unroll
                    for (int a = 0; a < 9; a++) R33[a] = pk[PK_R33 + a];
                    xp[0] = pk[PK_XP + 0]; xp[1] = pk[PK_XP + 1]; xp[2] = pk[PK_XP + 2];
                    sub(19);
                    if (j == w) matched = true;
                    if (lead) res[RES_MATCH + i] = w;
                    m++;
                    if (stage_ops && own && m == 4) {
                        store_ops_half(0, m);
                        ops_early = 1;
                    }
                }
            }
            if (dbg) sh_stamp[31] += __builtin_amdgcn_s_memrealtime() - sh_trec;   // landmark wave 0 done
            __syncthreads();
            if (sh_flag) vline = 0;
            const int rwp = sh_rwst;
            EKF_STAMP(14);
            // ---- (h) verdict (exchange 3, parity 0): the first violating line over the workgroups
            // (payload line + 1, 0: none); a violation restarts on the sequential path from there ----
            const int wv = wave_min(tid < SCAN_THREADS ? vline : L);
            __syncthreads();
            if ((tid & 63) == 0 && tid < SCAN_THREADS) sh_red[tid >> 6] = wv;
            __syncthreads();
            int first = L;
#pragma unroll
            for (int w = 0; w < SCAN_THREADS / 64; w++) first = min(first, sh_red[w]);
            if (G > 1) {
                if (tid == 0) mb_tag(mbox + (size_t)g * p.mbw, p.epoch, TAG_SPEC_VERDICT, (unsigned)(first < L ? first + 1 : 0));
                if (tid < G) {
                    int v = mb_poll(mbox, 0, G, tid, p.mbw, p.epoch, TAG_SPEC_VERDICT, tstatus, p.spin_log2);
                    if (p.test_verdict == e + 1 && g == 1 && tid == 0) {   // test hook: this poll timed out
                        tstatus |= EKF_ST_TIMEOUT_BIT;
                        v = -1;
                    }
                    sh_best[tid] = v > 0 ? v - 1 : L;
                    if (v < 0) sh_vto = 1;
                }
                __syncthreads();
                for (int k = 0; k < G; k++) first = min(first, sh_best[k]);
                if (sh_vto) {
                    // a verdict that never arrived: this workgroup does not restart (its peers
                    // may have committed their halves already); it finishes with the timeout bit
                    // in its completion word, and the lead, which collects every word, rolls the
                    // instance's call back
                    tstatus |= EKF_ST_TIMEOUT_BIT;
                    first = L;
                }
            }
            EKF_STAMP(6);
            if (first >= L) {
                status |= st_lines(stp, L) | st_lines(rwp, L);
            } else {
                dpath |= (first > 0 ? 8 | 512 : 8) | (first << 10);   // (512: lines kept; bits 10..12 the line)
                if (dbg) sh_stamp[15] += 1;
                sequential = true;
                keep = first;
                // the first kept line's exchange on parity 1: the verdict tags (parity 0) may still
                // be polled until every workgroup has passed it
                par0 = (first + 1) & 1;
                init_state();
                Dj[0] = Dj[1] = Dj[2] = Dj[3] = 0.0;
                if (own && j < s) {
                    if (mf && p.npend > 0) {
                        // the diagonal block the speculative pass started from (Dd, exact), which
                        // the kept lines' packages were computed against
                        const double4 b = Ddr[j];
                        Dj[0] = b.x; Dj[1] = b.y; Dj[2] = b.z; Dj[3] = b.w;
                    } else {
                        pll_block(pv, 2 * j, 2 * j, Dj);
                    }
                }
                // fp32 operands: out of sh_blk, which aliases the V history the restart writes, into
                // the stage (free once the speculative pass is over); fp64: sh_blk64 as it is
                if constexpr (!kB64)
                    if (own)
#pragma unroll
                        for (int t = 0; t < SPEC_L; t++)
                            if (t < L && sh_spec[t] >= 0) sh_cblk[t][tid] = sh_blk[t][tid];
                blk_cached = true;
                matched = false;
                m = nextra = 0;
                status = st_lines(stp, first) | st_lines(rwp, first);
                dsq = 0.0;
                ops_early = 0;   // (the sequential path rewrites every operand row)
                __syncthreads();   // sh_extra, sh_vhist reuse
            }
        } else {
            par0 = 1;   // the lists' parity-0 words may still be read
            // unresolved guesses: straight to the sequential path, which needs the exact owned
            // diagonal block (the staged path only loaded the last flushed one, for the guess)
            if ((staged || m64) && own && j < s) pll_block(pv, 2 * j, 2 * j, Dj);
        }
    }

    for (int i = 0; sequential && i < L; ++i) {
        if (i < keep) {
            // a kept line (restart): its guessed winner and package, verified by the verdict
            const int w = __builtin_amdgcn_readfirstlane(sh_spec[i]);
            const double* pk = sh_pk[i];
            if (w < 0 || __builtin_amdgcn_readfirstlane(pk[PK_OK] != 0.0 ? 1 : 0) == 0) {
                if (lead) {
                    res[RES_MATCH + i] = -1;
                    res[RES_EXTRA + nextra] = i;
                }
                if (tid == 0) sh_extra[nextra] = i;
                nextra++;
                continue;
            }
            if (own) {
                // the owned block of column w: the speculative pass's (scan start, pending steps
                // applied), as the sequential lines take it (owned_block, blk_cached)
                double blk[4];
                if constexpr (kB64) {
                    const double4 b = sh_blk64[i][tid];
                    blk[0] = b.x; blk[1] = b.y; blk[2] = b.z; blk[3] = b.w;
                } else {
                    const float4 b = sh_cblk[i][tid];
                    blk[0] = b.x; blk[1] = b.y; blk[2] = b.z; blk[3] = b.w;
                }
                double kk[4], uu[4];
                gain_rows<0>(pk, m, uq_owned, [&](int q) { return sh_wh[i][q][1]; }, blk, rr0, rr1, rr2, yb, Dj, kk, uu);
                float F[3] = {0.f, 0.f, 0.f};
                if (sym) sym_factor(pk, F);
                store_rows(m, kk, uu, true, F, true);
            }
            // = robot_update(R33, xp, pk), computed by the replay wave
#pragma unroll
            for (int a = 0; a < 9; a++) R33[a] = pk[PK_R33 + a];
            xp[0] = pk[PK_XP + 0]; xp[1] = pk[PK_XP + 1]; xp[2] = pk[PK_XP + 2];
            if (j == w) matched = true;
            if (lead) res[RES_MATCH + i] = w;
            m++;
            continue;
        }
        const ekf_line ln = sh_lines[i];
        double Rm[4];
        line_R(ln, i, r_mode, Rm);
        // gating of the owned candidate (Robot.cpp:313-498); the first passing unmatched j wins
        int best = 0x7fffffff;
        bool sing = false, amb = false;
        Cand c;
        if (own && j < s && !matched) {
            Block5 b5;
            fill_block5(b5, R33, rr0, rr1, rr2, Dj);
            double sn, cs;
            if (!quick_reject(b5, yb.x, yb.y, ma0, s0f, c0f, xp, ln.alpha, ln.r, Rm, p.gate, ETA) &&
                (exact_sc(), sincos_near(yb.x, ma0, s0j, c0j, sn, cs),
                 !certified_reject(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA))) {
                eval_candidate(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA, c);
                sing = c.singular;
                amb = c.amb;
                if (c.pass) best = j;
            }
        }
        EKF_STAMP(2);
        const int wbest = wave_min(best);
        if ((tid & 63) == 0 && tid < SCAN_THREADS) sh_red[tid >> 6] = wbest;
        __syncthreads();
        int gbest = sh_red[0];
#pragma unroll
        for (int w = 1; w < SCAN_THREADS / 64; w++) gbest = min(gbest, sh_red[w]);
        const int par = (i + par0) & 1;
        double* slot = mbox + ((size_t)par * G + g) * p.mbw;
        const int npk = MB_VH + 4 * m;
        if (best != 0x7fffffff && best == gbest) {
            // this workgroup's candidate: the uniform gain package and the V rows of the
            // candidate for the earlier matches of this scan (Robot.cpp:560-568 corrections),
            // staged in LDS
            build_package(c, R33, rr0, rr1, rr2, sh_pkg);
            for (int q = 0; q < m; q++) {
                const double4 vq = q < HIST_V ? sh_vhist[q][tid]
                                                : *reinterpret_cast<const double4*>(Vst + ((size_t)q * n + b0) * 2);
                sh_pkg[MB_VH + 4 * q + 0] = vq.x;
                sh_pkg[MB_VH + 4 * q + 1] = vq.y;
                sh_pkg[MB_VH + 4 * q + 2] = vq.z;
                sh_pkg[MB_VH + 4 * q + 3] = vq.w;
            }
        }
        __syncthreads();   // the staged package
        int jstar = gbest, gstar = 0;
        if (G > 1) {
            // to the mailbox, one word per lane; drained and ordered by the barrier before the
            // tagged best word (payload best + 1, 0: no candidate); every workgroup polls all G
            if (gbest != 0x7fffffff)
                for (int k = 1 + tid; k < npk; k += SCAN_BLOCK) mb_store(slot + k, sh_pkg[k]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
            if (tid == 0) mb_tag(slot, p.epoch, (unsigned)(i + 1), (unsigned)(gbest == 0x7fffffff ? 0 : gbest + 1));
            EKF_STAMP(3);
            for (int k = tid; k < G; k += SCAN_BLOCK) {
                const int bq = mb_poll(mbox, par, G, k, p.mbw, p.epoch, (unsigned)(i + 1), tstatus, p.spin_log2);
                sh_best[k] = bq <= 0 ? 0x7fffffff : bq - 1;
            }
            __syncthreads();
            jstar = 0x7fffffff;
            for (int k = 0; k < G; k++) {
                const int v = sh_best[k];
                if (v < jstar) { jstar = v; gstar = k; }
            }
        } else {
            EKF_STAMP(3);   // one workgroup: the package never leaves LDS
        }
        EKF_STAMP(4);
        // GSL_EDOM counts only for the candidates the reference evaluates (up to the winner)
        if (sing && j <= jstar) status |= EKF_ST_SINGULAR;
        if (amb && j <= jstar) status |= EKF_ST_PRECISION_BIT;
        if (jstar == 0x7fffffff) {
            // no match (or s == 0): the line goes to extraLines (Robot.cpp:308-310, 492-496)
            if (lead) {
                res[RES_MATCH + i] = -1;
                res[RES_EXTRA + nextra] = i;
            }
            if (tid == 0) sh_extra[nextra] = i;
            nextra++;
            continue;
        }
        // ---- match (Robot.cpp:500-641) ----
        // the winner's package and this thread's block of column jstar are independent: issue both
        // loads before waiting on either (another workgroup's winner: every workgroup reloads, its
        // own staged candidate included)
        double blk[4] = {0.0, 0.0, 0.0, 0.0};
        int tsc = -1;   // the winner's guess index, when its blocks are cached (blk_cached)
        if (blk_cached)
#pragma unroll
            for (int t = 0; t < SPEC_L; t++)
                if (t < L && sh_spec[t] == jstar) tsc = t;
        auto owned_block = [&]() {
            if (tsc >= 0) {
                if constexpr (kB64) {
                    const double4 b = sh_blk64[tsc][tid];
                    blk[0] = b.x; blk[1] = b.y; blk[2] = b.z; blk[3] = b.w;
                } else {
                    const float4 b = sh_cblk[tsc][tid];
                    blk[0] = b.x; blk[1] = b.y; blk[2] = b.z; blk[3] = b.w;
                }
            } else {
                pll_block(pv, 2 * j, 2 * jstar, blk);
            }
        };
        if (G > 1) {
            // (every thread passed the poll barrier after its mailbox stores read sh_pkg)
            const double* ps = mbox + ((size_t)par * G + gstar) * p.mbw;
            double pk0 = 0.0, pk1 = 0.0;
            if (tid < npk) pk0 = mb_load(ps + tid);
            if (tid + SCAN_BLOCK < npk) pk1 = mb_load(ps + tid + SCAN_BLOCK);
            if (own) owned_block();
            if (tid < npk) sh_pkg[tid] = pk0;
            if (tid + SCAN_BLOCK < npk) sh_pkg[tid + SCAN_BLOCK] = pk1;
            __syncthreads();
        } else if (own) {
            owned_block();
        }
        if (r_mode == 1 && (i == 1 || i == 2)) status |= EKF_ST_NSYM;
        if (own) {
            double kk[4], uu[4];
            gain_rows<0>(sh_pkg, m, uq_owned,
                         [&](int q) {
                             const double* vh = sh_pkg + MB_VH + 4 * q;
                             return make_double4(vh[0], vh[1], vh[2], vh[3]);
                         },
                         blk, rr0, rr1, rr2, yb, Dj, kk, uu);
            float F[3] = {0.f, 0.f, 0.f};
            if (sym) sym_factor(sh_pkg, F);
            store_rows(m, kk, uu, true, F, true);
        }
        robot_update(R33, xp, sh_pkg);
        if (j == jstar) matched = true;
        if (lead) res[RES_MATCH + i] = jstar;
        m++;
        EKF_STAMP(6);
    }
    status |= tstatus;

    // ---------------- commit (Robot.cpp:702-716) ----------------
    __syncthreads();   // sh_extra
    double pose[3] = {xp[0], xp[1], xp[2]};
    if (L == 0 || m == 0) pose[2] = normalize_radian(xp[2]);   // y[2] stays un-normalised
    const int nadd = min(nextra, N - s);
    const int reset = (s + nadd > N - p.reset_margin) ? 1 : 0;

    // ---------------- augmentation (Robot.cpp:776-866) ----------------
    double vnew = 0.0;   // the lead: the largest variance of the new landmarks (EKF_ARITH_F16X3's σ)
    if (!reset) {
        // the new landmarks' world-frame line and its sin/cos (Robot.cpp:787-803), lane q of every
        // wave for new landmark q (nadd <= max_lines <= 64), then read from that lane: one set of
        // fp64 trigonometry per wave instead of one per new landmark
        double a_r = 0.0, a_al = 0.0, a_sa = 0.0, a_ca = 1.0;
        {
            const int ql = threadIdx.x & 63;
            if (ql < nadd) {
                const ekf_line lq = sh_lines[sh_extra[ql]];
                double alfa = lq.alpha;
                a_r = lq.r + (pose[0] * cos(alfa) + pose[1] * sin(alfa));
                alfa += pose[2];
                sincos(alfa, &a_sa, &a_ca);
                a_al = alfa;
            }
        }
        for (int q = 0; q < nadd; q++) {
            const ekf_line ln = sh_lines[sh_extra[q]];
            const int sq = s + q;
            const double r = __shfl(a_r, q, 64);
            const double alfa = __shfl(a_al, q, 64);
            const double sa = __shfl(a_sa, q, 64), ca = __shfl(a_ca, q, 64);
            if (own && j < sq) {
                // landmark columns of P[l0:l0+2, 0:l0] = Gx·P[0:3, 0:l0] (Robot.cpp:852-862)
                double* prow = patch + (size_t)(q * 2) * M;
                *reinterpret_cast<double2*>(prow + 2 * j) = rr2;
                double2 gx;
                gx.x = ca * rr0.x + sa * rr1.x;
                gx.y = ca * rr0.y + sa * rr1.y;
                *reinterpret_cast<double2*>(prow + M + 2 * j) = gx;
            }
            if (j == sq) {
                // the new landmark: robot part of the same product (its robot-strip columns) and
                // its mean (Robot.cpp:801-803)
                rr0 = make_double2(R33[6], ca * R33[0] + sa * R33[3]);
                rr1 = make_double2(R33[7], ca * R33[1] + sa * R33[4]);
                rr2 = make_double2(R33[8], ca * R33[2] + sa * R33[5]);
                yb = make_double2(normalize_radian(alfa), r);
            }
            if (lead || j == sq) {
                // P_ll = Gx·Prr·Gxᵀ + Gl·R·Glᵀ (Robot.cpp:813-847); Gx = [[0,0,1],[ca,sa,0]],
                // Gl = [[1,0],[y1·ca − y0·sa, 1]]
                const double Gx[6] = {0, 0, 1, ca, sa, 0};
                const double Gl[4] = {1.0, 0, xp[1] * ca - xp[0] * sa, 1};
                double GP[6], GlR[4];
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 3; b++) {
                        double acc = 0.0;
                        for (int k = 0; k < 3; k++) acc += Gx[a * 3 + k] * R33[k * 3 + b];
                        GP[a * 3 + b] = acc;
                    }
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++)
                        GlR[a * 2 + b] = Gl[a * 2 + 0] * ln.R[0 * 2 + b] + Gl[a * 2 + 1] * ln.R[1 * 2 + b];
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) {
                        double gsum = 0.0;
                        for (int k = 0; k < 3; k++) gsum += GP[a * 3 + k] * Gx[b * 3 + k];
                        const double h = GlR[a * 2 + 0] * Gl[b * 2 + 0] + GlR[a * 2 + 1] * Gl[b * 2 + 1];
                        if (j == sq) Dj[a * 2 + b] = gsum + h;   // the new landmark's kept diagonal block
                        if (!lead) continue;
                        pdiag[q * 4 + a * 2 + b] = gsum + h;
                        if (a == b) vnew = fmax(vnew, gsum + h);
                        // fp16 storage: the new landmark's variances bound its whole row and
                        // column (|P_ij| <= sqrt(P_ii P_jj)), and downdates only shrink them
                        if (Stor<T>::half && fabs(ldexp(gsum + h, pv.ex)) > F16_RANGE_WARN)
                            status |= EKF_ST_RANGE_BIT;
                        // fp32 storage: within 2^8 of fp32's range (a diverged filter; SURVEY §8d's
                        // world reaches P ≈ 1e43 after 200 scans)
                        if (sizeof(typename Stor<T>::C) == 4 && !Stor<T>::half && !(fabs(gsum + h) <= F32_RANGE_WARN))
                            status |= EKF_ST_RANGE_BIT;
                    }
            }
        }
    }
    EKF_STAMP(27);
    // fp32 storage: an update that cancels more than 4 of fp32's 24 significant bits of a
    // landmark's variance (trace before / after > PREC_CANCEL = 2^4: the result no longer
    // guaranteed to 2^-20, the P bar), or leaves it non-positive, is flagged EKF_ST_PRECISION; the
    // result still commits (a diverging filter: SURVEY §8d's world)
    if constexpr (sizeof(C) == 4 && !Stor<T>::half)
        if (own && !reset && j < s && dsq > 0.0) {
            const double ta = Dj[0] + Dj[3];
            if (!(ta > 0.0) || ta + dsq > PREC_CANCEL * ta) status |= EKF_ST_PRECISION_BIT;
        }
    // EKF_ARITH_F16X3: an active landmark whose variance sits below the planes' dynamic range at
    // this scan's σ (a filter whose largest variance is ≥ 2^28 times its smallest: SURVEY §8d's
    // world in steady state) makes the step's flush exact (PLANE_SIGMA_EXACT, DONE_PLOSS)
    if (pf16 && own && !reset && j < s + nadd && ldexp(fmin(Dj[0], Dj[3]), 2 * psig) < PLANE_VAR_MIN)
        status |= (int)DONE_PLOSS;
    // write back the owned state (reset: Robot.cpp:893-904 zeroes landmark entries of y and P)
    if (own) {
        if (reset) {
            rr0 = rr1 = rr2 = yb = make_double2(0.0, 0.0);
        }
        *reinterpret_cast<double2*>(Rsw + b0) = rr0;
        *reinterpret_cast<double2*>(Rsw + n + b0) = rr1;
        *reinterpret_cast<double2*>(Rsw + 2 * n + b0) = rr2;
        *reinterpret_cast<double2*>(yw + b0) = yb;
        if (Ddw) Ddw[j] = reset || j >= s + nadd ? make_double4(0, 0, 0, 0) : make_double4(Dj[0], Dj[1], Dj[2], Dj[3]);
    }
    EKF_STAMP(28);
    if (own) {
        if (stage_ops) {
            if (!ops_early) store_ops_half(0, m);
            store_ops_half(1, m);
        } else if (sizeof(C) == 4) {
            // f32 operands: the k columns past the matches hold −0 (U) and +0 (V), so a flush
            // that runs every k-step unconditionally adds −0 there, which leaves every value as
            // it is (flush_f32_wave_kernel; the other forms and the on-read replay stop at ks)
            for (int k = 2 * m; k < d.kmax; k++)
#pragma unroll
                for (int pp = 0; pp < 2; pp++) {
                    if (!p.usym) Uop[op_index_f32(2 * j + pp, k, d.kmax)] = (C)(-0.0f);
                    Vop[op_index_f32(2 * j + pp, k, d.kmax)] = (C)0.0f;
                }
        }
        if (sizeof(C) == 8) {
            // f64 operands: the same −0 (U) / +0 (V) padding past the matches, so that the f64
            // wave flush may run every k-step (flush_f64_wave_kernel) while downdate_f64_kernel
            // and the on-read replay stop at the last 4-wide k-step holding a match
            for (int k = 2 * m; k < d.kmax; k++)
#pragma unroll
                for (int pp = 0; pp < 2; pp++) {
                    Uop[op_index_f64(2 * j + pp, k, d.kmax)] = (C)(-0.0);
                    Vop[op_index_f64(2 * j + pp, k, d.kmax)] = (C)0.0;
                }
        }
    }
    EKF_STAMP(24);
    // status bits seen by this workgroup's threads → its status word (read by ekf_read_results)
    int wgst = 0;
    {
        int st = status;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) st |= __shfl_xor(st, off, 64);
        __shared__ int sh_m;
        if (tid == 0) sh_m = m;   // the matches, as a landmark wave counted them
        __syncthreads();
        if constexpr (kPlanes)
            if (Bop && own) {
                // the owned rows' planes: per row and k parity h (k = 2s + h, s = 0..7) one
                // 16-byte lane row per part; k past the matches +0 (stored early, as the U and V
                // halves are, their split arithmetic lands on the per-line chain: scan +0.8 µs)
                const int m = sh_m;
                typedef unsigned u32x4v __attribute__((ext_vector_type(4)));
#pragma unroll
                for (int pp = 0; pp < 2; pp++) {
                    const f32x4v* src = reinterpret_cast<const f32x4v*>(sh_vpl + tid * 32 + pp * 16);
                    float v[16];
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const f32x4v x = src[i];
#pragma unroll
                        for (int u = 0; u < 4; u++) v[4 * i + u] = (4 * i + u) < 2 * m ? x[u] : 0.f;
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        if (HOT == 2 || (HOT == 0 && pf16)) {   // EKF_ARITH_F16X3: hi, lo of 2^σ·V
                            unsigned w[2][4];
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                unsigned o[2];
                                split_pack_f16(v[4 * q + h], v[4 * q + 2 + h], psig, o);
                                w[0][q] = o[0];
                                w[1][q] = o[1];
                            }
#pragma unroll
                            for (int pl = 0; pl < 2; pl++)
                                *reinterpret_cast<u32x4v*>(Bop + op_index_pl(2 * j + pp, h, pl, 2)) =
                                    u32x4v{w[pl][0], w[pl][1], w[pl][2], w[pl][3]};
                        }
                        if (HOT == 1 || (HOT == 0 && !pf16)) {   // EKF_ARITH_BF16X6: hi, mid, lo
                            unsigned w[3][4];
#pragma unroll
                            for (int q = 0; q < 4; q++) {
                                unsigned o[3];
                                split_pack(v[4 * q + h], v[4 * q + 2 + h], o);
#pragma unroll
                                for (int pl = 0; pl < 3; pl++) w[pl][q] = o[pl];
                            }
#pragma unroll
                            for (int pl = 0; pl < 3; pl++)
                                *reinterpret_cast<u32x4v*>(Bop + op_index_bf(2 * j + pp, h, pl)) =
                                    u32x4v{w[pl][0], w[pl][1], w[pl][2], w[pl][3]};
                        }
                    }
                }
            }
        if (__ballot(nzr) != 0ull) st |= (int)DONE_NZ;
        if ((tid & 63) == 0 && tid < SCAN_THREADS) sh_red[tid >> 6] = st;
        __syncthreads();
#pragma unroll
        for (int w = 0; w < SCAN_THREADS / 64; w++) wgst |= sh_red[w];
    }
    // completion (rollback protocol, publish_done / lead_collect): the lead commits the launch —
    // flips the instance to the copy of the robot strip and mean written above, writes the shared
    // state and the step's result record — only if every workgroup completed without a timeout.
    // Otherwise the instance keeps its state from before the call, and the step's record applies
    // nothing (no downdate, rows or reset: the flush and later on-read replays skip it).
    // The lead collects on the speculative path too: a workgroup's own verdict poll can time out
    // while the lead's succeeds (the two polls race the spin bound), and that workgroup then
    // finishes with the timeout bit (above); only its completion word tells the lead.
    EKF_STAMP(25);
    if (tid == 0 && g != 0) publish_done(sync, g, p.epoch, wgst);
    int zg = (wgst & (int)DONE_NZ) ? 1 : 0;
    if (g == 0 && (sequential || G > 1)) wgst = lead_collect<SCAN_BLOCK>(sync, G, p.epoch, wgst, p.spin_log2, tid, sh_red, zg);
    const bool ploss = (wgst & (int)DONE_PLOSS) != 0;
    wgst &= ~(int)(DONE_NZ | DONE_PLOSS);
    EKF_STAMP(26);
    if (lead) {
        sync[SYNC_WG0] = (int)done_word(p.epoch, wgst);
        const bool commit = !(wgst & EKF_ST_TIMEOUT_BIT);
        res[RES_NLINES] = L;
        res[RES_SAVED_IN] = s;
        res[RES_DBG] = dpath | rpath | (sequential ? 16 : 0);
        for (int t = 0; t < 5; t++) res[RES_DBG + 1 + t] = t < SPEC_L ? sh_spec[t] : -2;
        if (commit) {
            yw[0] = xp[0];
            yw[1] = xp[1];
            yw[2] = xp[2];
            for (int a = 0; a < 9; a++) Rsw[(a / 3) * n + (a % 3)] = R33[a];
            p.pose[3 * e + 0] = pose[0];
            p.pose[3 * e + 1] = pose[1];
            p.pose[3 * e + 2] = pose[2];
            res[RES_STATUS] = ((nextra > nadd) ? EKF_ST_CAP : 0);
            res[RES_M] = m;
            res[RES_NEXTRA] = nextra;
            res[RES_SAVED] = reset ? 0 : s + nadd;
            res[RES_RESET] = reset;
            res[RES_NADD] = reset ? 0 : nadd;
            res[RES_KSTEPS] = (sizeof(C) == 4) ? m : (m + 1) / 2;
            res[RES_ROLLBACK] = 0;
            res[RES_PSIG] = ploss ? PLANE_SIGMA_EXACT : psig;
            // nonzero operand rows only below zg workgroups' landmarks; new rows below s + nadd
            res[RES_ZMAX] = max(min(zg * SCAN_THREADS, N), reset ? 0 : s + nadd);
            if (p.res_host) {
                // the synchronous call's result without a copy: the words ekf_result takes (the
                // status with every workgroup's bits, as the host's fold of the completion words
                // would give: the lead collected them), the pose and the robot block, then the
                // epoch. A rollback writes none of it (the host then reads the device copies)
                int* rh = p.res_host + (size_t)e * RES_STRIDE;
                rh[RES_NLINES] = L;
                rh[RES_STATUS] = res[RES_STATUS] | (wgst & DONE_STATUS_MASK);
                rh[RES_M] = m;
                rh[RES_NEXTRA] = nextra;
                rh[RES_SAVED] = reset ? 0 : s + nadd;
                rh[RES_RESET] = reset;
                for (int i = 0; i < L; i++) rh[RES_MATCH + i] = res[RES_MATCH + i];
                p.pose_host[3 * e + 0] = pose[0];
                p.pose_host[3 * e + 1] = pose[1];
                p.pose_host[3 * e + 2] = pose[2];
                for (int a = 0; a < 9; a++) p.r33_host[9 * e + a] = R33[a];
                __threadfence_system();
                __hip_atomic_store(p.ep_host + e, p.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
            }
            p.saved[e] = reset ? 0 : s + nadd;
            p.live[e] = 1 - cb;
            if (pf16) {
                // the plane exponent of the later steps: |V_ik| <= sqrt(P_ii) <= sqrt(vmax), and
                // |2^σ·V| <= 2^12 at σ = plane_sigma(vmax). A larger vmax waits for the next group
                // (the first scan of a group recomputes σ) while |2^σ·V| stays <= 2^15 (fp16's
                // range is 2^16): σ at most 3 above plane_sigma(vmax)
                if (reset) {
                    p.pvmax[e] = 0.0;
                    p.psig[e] = PLANE_SIGMA_EMPTY;
                } else {
                    const double vm = fmax(p.pvmax[e], vnew);
                    const int target = plane_sigma(vm);
                    p.pvmax[e] = vm;
                    p.psig[e] = target < psig - 3 ? target : psig;
                }
            }
        } else {
            res[RES_STATUS] = 0;
            res[RES_M] = 0;
            res[RES_NEXTRA] = 0;
            res[RES_SAVED] = s;
            res[RES_RESET] = 0;
            res[RES_NADD] = 0;
            res[RES_KSTEPS] = 0;
            res[RES_ROLLBACK] = 1;
            res[RES_ZMAX] = 0;
            for (int i = 0; i < L; i++) res[RES_MATCH + i] = -1;
        }
    }
    EKF_STAMP(7);
    if (dbg) {
        // (phase times accumulate in LDS: a global read-modify-write per stamp would add a
        // memory round trip to every phase it measures)
        for (int k = 0; k < EKF_NSTAMP; k++) dbg[k] += sh_stamp[k];
        dbg[8] += t_last - t_first;
        dbg[9] += 1;
    }
}

// ---------------------------------------------------------------------------------------
// One instance with its landmark block partitioned over ranks (ShardParams): the
// scan kernel's sequential association path phase by phase over every landmark, one thread per
// landmark, every expression the scan kernel's (the same inline functions in this contract(on)
// region), so that a sharded run is bit-identical to a single-context one. Between phases the
// caller sums the [N][4] exchange buffer over the ranks (each fills the blocks its tiles hold).
// Predict (Robot.cpp:130-286) as the scan kernel's init_state: F3, x_pre and the 3×3 block
__device__ __forceinline__ void shard_predict(const double pose[3], const double enc[3], double enc_noise,
                                              double F3[9], double R33[9], double xp[3])
{
    const double x0 = pose[0], y0 = pose[1], t0 = pose[2];
    const double u2 = t0 - enc[2];
    const double dx = x0 - enc[0], dy = y0 - enc[1];
    const double u0 = sqrt(dx * dx + dy * dy);
    const double c = u2 / 2.0 + t0;
    double sc, cc;
    sincos(c, &sc, &cc);
    F3[2] = -u0 * sc;
    F3[5] = u0 * cc;
    xp[0] = x0 + u0 * cc;
    xp[1] = y0 + u0 * sc;
    xp[2] = t0 + u2;
    const double Fu3[9] = {cc, 0, -u0 * sc / 2.0, sc, 1, u0 * cc / 2.0, 0, 0, 1};
    const double qs = (-1.0 / (1 + fabs(u0)) + 1);
    const double Q[9] = {enc_noise * qs, 0, 0, 0, 2 * enc_noise * qs, 0, 0, 0, enc_noise * qs};
    double FP[9], FuQ[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0.0, t = 0.0;
            for (int k = 0; k < 3; k++) {
                s += F3[a * 3 + k] * R33[k * 3 + b];
                t += Fu3[a * 3 + k] * Q[k * 3 + b];
            }
            FP[a * 3 + b] = s;
            FuQ[a * 3 + b] = t;
        }
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0.0, t = 0.0;
            for (int k = 0; k < 3; k++) {
                s += FP[a * 3 + k] * F3[b * 3 + k];
                t += FuQ[a * 3 + k] * Fu3[b * 3 + k];
            }
            R33[a * 3 + b] = s + t;
        }
}

// One phase of the partitioned instance's scan for landmark j (every rank runs every landmark):
// shard_kernel runs one phase over a grid, shard_run_kernel the per-line phases of the
// speculative path in one workgroup (its ctl, robot and package words in LDS).
template <typename T>
__device__ __forceinline__ void shard_step(const ShardParams& p, const int phase, const int line, const int j,
                                           const PllView<T>& pv)
{
    using C = typename Stor<T>::C;
    constexpr double ETA = gate_eta<T>();
    const Dims d = p.d;
    const int n = d.n;
    const bool own = j < d.N;
    int* ctl = p.ctl;
    // block (j, w) of the landmark block is this rank's if the tile that stores it is
    auto local_blk = [&](int ja, int wb) {
        const int ba = (2 * ja) >> 5, bb = (2 * wb) >> 5;
        const long long t = tile_index(ba < bb ? ba : bb, ba < bb ? bb : ba, d.nb);
        return t >= p.t0 && t < p.t1;
    };
    const bool sym = p.r_mode != 1 && sizeof(C) == 4;
    const int b0 = 3 + 2 * j;
    double* rc = p.rec + (size_t)j * SH_REC;
    double R33[9], xp[3];
    if (phase != SH_BEGIN) {
#pragma unroll
        for (int a = 0; a < 9; a++) R33[a] = p.rob[a];
        xp[0] = p.rob[9]; xp[1] = p.rob[10]; xp[2] = p.rob[11];
    }
    if (phase == SH_ROBOT) {
        // after line `line` (one thread): the robot block and x_pre after its match (Robot.cpp:560-602),
        // the match list, and the winner word reset for the next line's gate
        if (j == 0) {
            const int jstar = ctl[SC_WIN];
            if (jstar != 0x7fffffff) {
                robot_update(R33, xp, p.pkg);
#pragma unroll
                for (int a = 0; a < 9; a++) p.rob[a] = R33[a];
                p.rob[9] = xp[0]; p.rob[10] = xp[1]; p.rob[11] = xp[2];
                ctl[SC_MATCH + line] = jstar;
                ctl[SC_M] += 1;
            } else {
                ctl[SC_MATCH + line] = -1;
                ctl[SC_EXTRA + ctl[SC_NEXTRA]] = line;
                ctl[SC_NEXTRA] += 1;
            }
            ctl[SC_WIN] = 0x7fffffff;
        }
        return;
    }

    if (phase == SH_BEGIN) {
        // the committed robot block and pose, predicted (every thread the same), every landmark's
        // strip columns predicted (Robot.cpp:242) and scan-start angle; the rank's diagonal blocks
        // with the pending steps applied into the exchange buffer (zero where another rank's)
        const int s = p.saved[0];
#pragma unroll
        for (int a = 0; a < 9; a++) R33[a] = p.Rs[(a / 3) * n + (a % 3)];
        double F3[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
        shard_predict(p.pose, p.enc_v, p.enc_noise, F3, R33, xp);
        if (j == 0) {
            // the scan's inputs, handed over as kernel arguments (no host staging copy), for the
            // later phases
            double* enc = const_cast<double*>(p.enc);
            enc[0] = p.enc_v[0]; enc[1] = p.enc_v[1]; enc[2] = p.enc_v[2];
            ekf_line* lines = const_cast<ekf_line*>(p.lines);
            for (int i = 0; i < d.max_lines; i++) lines[i] = p.lines_v[i];
#pragma unroll
            for (int a = 0; a < 9; a++) p.rob[a] = R33[a];
            p.rob[9] = xp[0]; p.rob[10] = xp[1]; p.rob[11] = xp[2];
            ctl[SC_WIN] = 0x7fffffff;
            ctl[SC_STATUS] = 0;
            ctl[SC_M] = 0;
            ctl[SC_NEXTRA] = 0;
            ctl[SC_S] = s;
            ctl[SC_NEXT] = 0;
            for (int i = 0; i < EKF_MAX_LINES; i++) ctl[SC_GUESS + i] = 0x7fffffff;
        }
        if (!own) return;
        double2 rr0 = *reinterpret_cast<const double2*>(p.Rs + b0);
        double2 rr1 = *reinterpret_cast<const double2*>(p.Rs + n + b0);
        double2 rr2 = *reinterpret_cast<const double2*>(p.Rs + 2 * n + b0);
        const double2 yb = *reinterpret_cast<const double2*>(p.y + b0);
        predict_cols(F3, rr0, rr1, rr2);
        double Dj[4] = {0, 0, 0, 0};
        if (j < s && local_blk(j, j)) pll_block(pv, 2 * j, 2 * j, Dj);
        double s0j, c0j;
        sincos(yb.x, &s0j, &c0j);
        float s0f, c0f;
        __sincosf((float)yb.x, &s0f, &c0f);
        const double v[SH_REC] = {rr0.x, rr0.y, rr1.x, rr1.y, rr2.x, rr2.y, yb.x, yb.y, 0, 0, 0, 0,
                                  yb.x, s0j, c0j, (double)s0f, (double)c0f, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < SH_REC; k++) rc[k] = v[k];
        *reinterpret_cast<double4*>(p.col + 4 * (size_t)j) = make_double4(Dj[0], Dj[1], Dj[2], Dj[3]);
        p.flags[j] = 0;
        return;
    }
    if (!own) return;
    const bool fused_diag = phase == SH_GUESS && p.diag_first;
    double4 dj = make_double4(0, 0, 0, 0);
    if (phase == SH_DIAG || fused_diag) {
        // the summed diagonal blocks (every rank contributed its own); the guesses may follow in
        // the same launch, which reads them from the sum (its grid row 0 stores them)
        dj = *reinterpret_cast<const double4*>(p.col + 4 * (size_t)j);
        if (phase == SH_DIAG || line == 0) {
            rc[8] = dj.x; rc[9] = dj.y; rc[10] = dj.z; rc[11] = dj.w;
        }
        if (phase == SH_DIAG) return;
    }
    const int s = ctl[SC_S];
    double2 rr0 = make_double2(rc[0], rc[1]), rr1 = make_double2(rc[2], rc[3]), rr2 = make_double2(rc[4], rc[5]);
    double2 yb = make_double2(rc[6], rc[7]);
    double Dj[4] = {rc[8], rc[9], rc[10], rc[11]};
    if (fused_diag) {
        Dj[0] = dj.x; Dj[1] = dj.y; Dj[2] = dj.z; Dj[3] = dj.w;
    }
    const double ma0 = rc[12], s0j = rc[13], c0j = rc[14];
    const double s0f = rc[15], c0f = rc[16];
    int fl = p.flags[j];
    ekf_line ln = p.lines[line < 0 ? 0 : line];
    double Rm[4];
    line_R(ln, line, p.r_mode, Rm);

    // the gate of one landmark exactly as the sequential path (Robot.cpp:313-498)
    auto gate_of = [&](Cand& c, bool& pass, bool& sing, bool& amb) {
        Block5 b5;
        fill_block5(b5, R33, rr0, rr1, rr2, Dj);
        double sn, cs;
        pass = sing = amb = false;
        if (!quick_reject(b5, yb.x, yb.y, ma0, s0f, c0f, xp, ln.alpha, ln.r, Rm, p.gate, ETA) &&
            (sincos_near(yb.x, ma0, s0j, c0j, sn, cs),
             !certified_reject(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA))) {
            eval_candidate(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA, c);
            sing = c.singular;
            amb = c.amb;
            pass = c.pass;
        }
    };

    if (phase == SH_GUESS) {
        // every line's first passing landmark at the scan's start (no line applied yet): the
        // speculative path fetches these columns in one exchange; shard_run_kernel checks each
        // line's real winner against its guess
        // (one line per grid row)
        if (!(j < s)) return;
        Cand c;
        bool pass, sing, amb;
        gate_of(c, pass, sing, amb);
        if (pass) atomicMin(ctl + SC_GUESS + line, j);
        return;
    }
    if (phase == SH_SPEC_COLS) {
        // the rank's blocks of the guessed column of line `line` (one line per grid row), pending
        // steps applied (SH_COLUMN's blocks)
        {
            const int i = line;
            const int w = ctl[SC_GUESS + i];
            double blk[4] = {0, 0, 0, 0};
            if (w != 0x7fffffff && local_blk(j, w)) pll_block(pv, 2 * j, 2 * w, blk);
            *reinterpret_cast<double4*>(p.cols + 4 * ((size_t)i * d.N + j)) = make_double4(blk[0], blk[1], blk[2], blk[3]);
        }
        return;
    }
    if (phase == SH_PACKAGE) {   // (the winner's thread) SH_COLUMN's package, without the column
        Cand c;
        bool pass, sing, amb;
        gate_of(c, pass, sing, amb);
        build_package(c, R33, rr0, rr1, rr2, p.pkg);
        const int m = ctl[SC_M];
        for (int q = 0; q < m; q++) {
            const double* h = p.hist + ((size_t)j * d.max_lines + q) * 8 + 4;
            p.pkg[MB_VH + 4 * q + 0] = h[0];
            p.pkg[MB_VH + 4 * q + 1] = h[1];
            p.pkg[MB_VH + 4 * q + 2] = h[2];
            p.pkg[MB_VH + 4 * q + 3] = h[3];
        }
        return;
    }

    if (phase == SH_GATE) {
        // the first passing unmatched landmark of the line: every rank finds the same one
        if (!(j < s) || (fl & 1)) {
            p.flags[j] = fl & 1;
            return;
        }
        Cand c;
        bool pass, sing, amb;
        gate_of(c, pass, sing, amb);
        p.flags[j] = (fl & 1) | (sing ? 2 : 0) | (amb ? 4 : 0);
        if (pass) {
            atomicMin(ctl + SC_WIN, j);
            if (p.pkg_slot) {   // (shard_run_kernel) SH_PACKAGE's package from this evaluation
                double* slot = p.pkg_slot + (size_t)threadIdx.x * SH_PKG_WORDS;
                build_package(c, R33, rr0, rr1, rr2, slot);
                const int m = ctl[SC_M];
                for (int q = 0; q < m; q++) {
                    const double* h = p.hist + ((size_t)j * d.max_lines + q) * 8 + 4;
                    slot[MB_VH + 4 * q + 0] = h[0];
                    slot[MB_VH + 4 * q + 1] = h[1];
                    slot[MB_VH + 4 * q + 2] = h[2];
                    slot[MB_VH + 4 * q + 3] = h[3];
                }
            }
        }
        return;
    }

    if (phase == SH_COLUMN) {
        // the winner's gain package (its thread) and the rank's blocks of its column, with the
        // pending steps applied, into the exchange buffer (zero where another rank's)
        const int jstar = ctl[SC_WIN];
        double blk[4] = {0, 0, 0, 0};
        if (jstar != 0x7fffffff) {
            if (local_blk(j, jstar)) pll_block(pv, 2 * j, 2 * jstar, blk);
            if (j == jstar) {
                Cand c;
                bool pass, sing, amb;
                gate_of(c, pass, sing, amb);
                build_package(c, R33, rr0, rr1, rr2, p.pkg);
                const int m = ctl[SC_M];
                for (int q = 0; q < m; q++) {   // the winner's V rows of the earlier matches (Robot.cpp:560-568)
                    const double* h = p.hist + ((size_t)j * d.max_lines + q) * 8 + 4;
                    p.pkg[MB_VH + 4 * q + 0] = h[0];
                    p.pkg[MB_VH + 4 * q + 1] = h[1];
                    p.pkg[MB_VH + 4 * q + 2] = h[2];
                    p.pkg[MB_VH + 4 * q + 3] = h[3];
                }
            }
        }
        *reinterpret_cast<double4*>(p.col + 4 * (size_t)j) = make_double4(blk[0], blk[1], blk[2], blk[3]);
        return;
    }

    if (phase == SH_APPLY) {
        const int jstar = ctl[SC_WIN];
        // GSL_EDOM counts only for the candidates the reference evaluates (up to the winner)
        int st = (fl & 2) && j <= jstar ? (int)EKF_ST_SINGULAR : 0;
        if ((fl & 4) && j <= jstar) st |= EKF_ST_PRECISION_BIT;   // (gate_eta)
        if (p.r_mode == 1 && (line == 1 || line == 2)) st |= EKF_ST_NSYM;
        if (st) atomicOr(ctl + SC_STATUS, st);
        if (jstar == 0x7fffffff) return;
        const double4 cb = *reinterpret_cast<const double4*>(p.col + 4 * (size_t)j);   // summed over ranks
        double blk[4] = {cb.x, cb.y, cb.z, cb.w};
        const double* pk = p.pkg;
        const int m = ctl[SC_M];
        double kk[4], uu[4];
        gain_rows<0>(pk, m,
                     [&](int q) {
                         const double* h = p.hist + ((size_t)j * d.max_lines + q) * 8;
                         return make_double4(h[0], h[1], h[2], h[3]);
                     },
                     [&](int q) {
                         const double* vh = pk + MB_VH + 4 * q;
                         return make_double4(vh[0], vh[1], vh[2], vh[3]);
                     },
                     blk, rr0, rr1, rr2, yb, Dj, kk, uu);
        float F[3] = {0.f, 0.f, 0.f};
        if (sym) sym_factor(pk, F);
        // store_rows (the scan kernel's non-staged form: the same values)
        double* h = p.hist + ((size_t)j * d.max_lines + m) * 8;
        h[0] = uu[0]; h[1] = uu[1]; h[2] = uu[2]; h[3] = uu[3];
        h[4] = kk[0]; h[5] = kk[1]; h[6] = kk[2]; h[7] = kk[3];
        C* Uop = reinterpret_cast<C*>(p.cur.Uop);
        C* Vop = reinterpret_cast<C*>(p.cur.Vop);
#pragma unroll
        for (int pp = 0; pp < 2; pp++) {
            const int lr = 2 * j + pp;
            if constexpr (sizeof(C) == 4) {
                double o0 = uu[2 * pp], o1 = uu[2 * pp + 1], v0 = kk[2 * pp], v1 = kk[2 * pp + 1];
                if (sym) {
                    v0 = kk[2 * pp] * (double)F[0] + kk[2 * pp + 1] * (double)F[1];
                    v1 = kk[2 * pp + 1] * (double)F[2];
                    o0 = (double)(float)v0;
                    o1 = (double)(float)v1;
                }
                Uop[op_index_f32(lr, 2 * m, d.kmax)] = to_domain<T>(-o0, pv.ex);
                Uop[op_index_f32(lr, 2 * m + 1, d.kmax)] = to_domain<T>(-o1, pv.ex);
                Vop[op_index_f32(lr, 2 * m, d.kmax)] = (C)v0;
                Vop[op_index_f32(lr, 2 * m + 1, d.kmax)] = (C)v1;
            } else {
                Uop[op_index_f64(lr, 2 * m, d.kmax)] = (C)(-uu[2 * pp]);
                Uop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (C)(-uu[2 * pp + 1]);
                Vop[op_index_f64(lr, 2 * m, d.kmax)] = (C)kk[2 * pp];
                Vop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (C)kk[2 * pp + 1];
            }
        }
        if (j == jstar) fl |= 1;
        p.flags[j] = fl & 1;
        const double v[12] = {rr0.x, rr0.y, rr1.x, rr1.y, rr2.x, rr2.y, yb.x, yb.y, Dj[0], Dj[1], Dj[2], Dj[3]};
#pragma unroll
        for (int k = 0; k < 12; k++) rc[k] = v[k];
        return;
    }

    // SH_END: augmentation (Robot.cpp:776-866) as the scan kernel's commit: the new landmarks' rows
    // to the step's patch buffer (every rank all of them: its flush takes the columns of its tiles),
    // the new landmarks' strip columns and mean, the 2×2 diagonal blocks; the capacity reset
    // (Robot.cpp:893-904)
    if (p.end_gate) {
        // (ekf_shard_localize) launched behind the speculative run before the host has read the
        // agreement: a run that stopped short or failed on some rank leaves everything untouched
        const double a0 = p.end_gate[0], a1 = p.end_gate[1];
        if (j == 0) {
            p.end_gate_host[0] = a0;
            p.end_gate_host[1] = a1;
            __threadfence_system();
        }
        if (a0 > 0.0 || a1 != (double)p.L) return;
    }
    const int m = ctl[SC_M], nextra = ctl[SC_NEXTRA];
    double pose[3] = {xp[0], xp[1], xp[2]};
    if (p.L == 0 || m == 0) pose[2] = normalize_radian(xp[2]);
    const int N = d.N, M = d.M;
    const int nadd = min(nextra, N - s);
    const int reset = (s + nadd > N - p.reset_margin) ? 1 : 0;
    double* patch = p.cur.patch;
    double* pdiag = p.cur.patch_diag;
    if (!reset) {
        for (int q = 0; q < nadd; q++) {
            const ekf_line lq = p.lines[ctl[SC_EXTRA + q]];
            const int sq = s + q;
            double alfa = lq.alpha;
            const double r = lq.r + (pose[0] * cos(alfa) + pose[1] * sin(alfa));
            alfa += pose[2];
            double sa, ca;
            sincos(alfa, &sa, &ca);
            if (j < sq) {
                double* prow = patch + (size_t)(q * 2) * M;
                *reinterpret_cast<double2*>(prow + 2 * j) = rr2;
                double2 gx;
                gx.x = ca * rr0.x + sa * rr1.x;
                gx.y = ca * rr0.y + sa * rr1.y;
                *reinterpret_cast<double2*>(prow + M + 2 * j) = gx;
            }
            if (j == sq) {
                rr0 = make_double2(R33[6], ca * R33[0] + sa * R33[3]);
                rr1 = make_double2(R33[7], ca * R33[1] + sa * R33[4]);
                rr2 = make_double2(R33[8], ca * R33[2] + sa * R33[5]);
                yb = make_double2(normalize_radian(alfa), r);
            }
            if (j == 0) {
                const double Gx[6] = {0, 0, 1, ca, sa, 0};
                const double Gl[4] = {1.0, 0, xp[1] * ca - xp[0] * sa, 1};
                double GP[6], GlR[4];
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 3; b++) {
                        double acc = 0.0;
                        for (int k = 0; k < 3; k++) acc += Gx[a * 3 + k] * R33[k * 3 + b];
                        GP[a * 3 + b] = acc;
                    }
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++)
                        GlR[a * 2 + b] = Gl[a * 2 + 0] * lq.R[0 * 2 + b] + Gl[a * 2 + 1] * lq.R[1 * 2 + b];
                for (int a = 0; a < 2; a++)
                    for (int b = 0; b < 2; b++) {
                        double gsum = 0.0;
                        for (int k = 0; k < 3; k++) gsum += GP[a * 3 + k] * Gx[b * 3 + k];
                        const double hh = GlR[a * 2 + 0] * Gl[b * 2 + 0] + GlR[a * 2 + 1] * Gl[b * 2 + 1];
                        pdiag[q * 4 + a * 2 + b] = gsum + hh;
                    }
            }
        }
    }
    if (reset) rr0 = rr1 = rr2 = yb = make_double2(0.0, 0.0);
    // the strip columns and mean, the operand padding past the matches
    *reinterpret_cast<double2*>(p.Rs + b0) = rr0;
    *reinterpret_cast<double2*>(p.Rs + n + b0) = rr1;
    *reinterpret_cast<double2*>(p.Rs + 2 * n + b0) = rr2;
    *reinterpret_cast<double2*>(p.y + b0) = yb;
    C* Uop = reinterpret_cast<C*>(p.cur.Uop);
    C* Vop = reinterpret_cast<C*>(p.cur.Vop);
    for (int k = 2 * m; k < d.kmax; k++)
#pragma unroll
        for (int pp = 0; pp < 2; pp++) {
            if constexpr (sizeof(C) == 4) {
                Uop[op_index_f32(2 * j + pp, k, d.kmax)] = (C)(-0.0f);
                Vop[op_index_f32(2 * j + pp, k, d.kmax)] = (C)0.0f;
            } else {
                Uop[op_index_f64(2 * j + pp, k, d.kmax)] = (C)(-0.0);
                Vop[op_index_f64(2 * j + pp, k, d.kmax)] = (C)0.0;
            }
        }
    if (j == 0) {
        // commit (Robot.cpp:702-716)
        for (int a = 0; a < 9; a++) p.Rs[(a / 3) * n + (a % 3)] = R33[a];
        p.y[0] = xp[0]; p.y[1] = xp[1]; p.y[2] = xp[2];
        p.pose[0] = pose[0]; p.pose[1] = pose[1]; p.pose[2] = pose[2];
        int* res = p.cur.res;
        res[RES_NLINES] = p.L;
        res[RES_SAVED_IN] = s;
        res[RES_DBG] = 16;
        res[RES_STATUS] = ((nextra > nadd) ? EKF_ST_CAP : 0) | ctl[SC_STATUS];
        res[RES_M] = m;
        res[RES_NEXTRA] = nextra;
        res[RES_SAVED] = reset ? 0 : s + nadd;
        res[RES_RESET] = reset;
        res[RES_NADD] = reset ? 0 : nadd;
        res[RES_KSTEPS] = (sizeof(C) == 4) ? m : (m + 1) / 2;
        res[RES_ROLLBACK] = 0;
        for (int i = 0; i < p.L; i++) res[RES_MATCH + i] = ctl[SC_MATCH + i];
        for (int q = 0; q < nextra; q++) res[RES_EXTRA + q] = ctl[SC_EXTRA + q];
        p.saved[0] = reset ? 0 : s + nadd;
        if (p.res_host) {
            // the words ekf_result takes, for the host to read after this kernel without a copy
            // (each store crosses to host memory: only these, not the whole record)
            int* rh = p.res_host;
            rh[RES_NLINES] = res[RES_NLINES];
            rh[RES_STATUS] = res[RES_STATUS];
            rh[RES_M] = res[RES_M];
            rh[RES_NEXTRA] = res[RES_NEXTRA];
            rh[RES_SAVED] = res[RES_SAVED];
            rh[RES_RESET] = res[RES_RESET];
            for (int i = 0; i < p.L; i++) rh[RES_MATCH + i] = res[RES_MATCH + i];
            p.pose_host[0] = pose[0]; p.pose_host[1] = pose[1]; p.pose_host[2] = pose[2];
            __threadfence_system();
        }
    }
}

template <typename T>
__global__ __launch_bounds__(SH_THREADS) void shard_kernel(ShardParams p)
{
    __shared__ int4 sh_ctl[PMAX];
    for (int q = threadIdx.x; q < p.npend; q += blockDim.x) {
        const int* r = p.pend[q].res;
        sh_ctl[q] = make_int4(r[RES_RESET], r[RES_KSTEPS], r[RES_NADD], r[RES_SAVED_IN]);
    }
    __syncthreads();
    const Dims d = p.d;
    PllView<T> pv;
    pv.X = reinterpret_cast<const T*>(p.Pread);
    pv.nb = d.nb;
    pv.kmax = d.kmax;
    pv.M = d.M;
    pv.max_lines = d.max_lines;
    pv.e = 0;
    pv.ex = storage_exp<T>(p.pexp, 0);
    pv.opstride = (size_t)d.nb * 64 * (d.kmax / 2);
    pv.usym = 0;   // (the partitioned instance stores its U rows)
    pv.us = 1.0f;
    pv.npend = p.npend;
    pv.pend = p.pend;
    pv.ctl = sh_ctl;
    pv.rnd = 1;
    // (SH_GUESS, SH_SPEC_COLS: grid row y = the line)
    shard_step<T>(p, p.phase, (p.phase == SH_SPEC_COLS || p.phase == SH_GUESS) ? (int)blockIdx.y : p.line,
                  (int)(blockIdx.x * blockDim.x + threadIdx.x), pv);
}

// The speculative path's lines (ekf_shard_run): G cooperating workgroups run lines 0 .. L − 1 of
// the sequential association exactly as the per-line phases do (gate of every landmark, the
// winner's package, gain rows, robot update), taking each winner's column from the exchanged
// guessed columns (p.cols) instead of a per-line exchange between ranks. Landmark j belongs to
// thread j mod SHR_THREADS of workgroup ⌊j / SHR_THREADS⌋ mod G for the whole run (its records,
// U/V history and flags are only ever touched by that thread). Every workgroup holds its own
// copy of the control words, the robot block and the package in LDS and updates them itself
// (SH_ROBOT: the same bits in every workgroup). Per line one exchange among the workgroups, the
// scan kernel's sequential-path mailbox: each publishes its first passing landmark and, when it has
// one, that landmark's package (built before the exchange), then polls every workgroup's tag; all
// take the smallest landmark and its package, the reference's first passing one
// (Robot.cpp:313-498). A line whose winner is not its guess stops the run there (*next_out = that
// line; L + 1 when a workgroup's exchange timed out: the scan is abandoned): the caller continues
// with the per-line phases from the state after the lines before it. Every rank holds the same
// replicated state, so every rank stops at the same line.
template <typename T>
__global__ __launch_bounds__(SHR_THREADS) void shard_run_kernel(ShardParams p)
{
    __shared__ int sh_cw[SC_WORDS];
    __shared__ double sh_rob[12];
    __shared__ double sh_pkg[MB_WORDS_FIXED + 4 * EKF_MAX_LINES];
    __shared__ int sh_best[SHR_GMAX];
    __shared__ int sh_to;
    __shared__ int sh_bad;   // workgroup 0: some workgroup timed out, never arrived or stopped elsewhere
    __shared__ double sh_slot[SHR_THREADS][SH_PKG_WORDS];   // each thread's package of its passing landmark
    const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x;
    for (int k = tid; k < SC_WORDS; k += SHR_THREADS) sh_cw[k] = p.ctl[k];
    if (tid < 12) sh_rob[tid] = p.rob[tid];
    if (tid == 0) sh_to = sh_bad = 0;
    __syncthreads();
    ShardParams q = p;
    q.ctl = sh_cw;
    q.rob = sh_rob;
    q.pkg = sh_pkg;
    PllView<T> pv = {};   // (unused by the per-line phases)
    const int N = p.d.N;
    const int stride = G * SHR_THREADS;
    // one landmark per thread: every passing landmark builds its package during the gate (the
    // owner's slot is the package); otherwise the owner rebuilds it after the gate (SH_PACKAGE)
    const bool fused = N <= stride;
    q.pkg_slot = fused ? &sh_slot[0][0] : nullptr;   // (only SH_GATE reads it: its thread's row)
    int status = 0, i = 0;
    for (; i < p.L; i++) {
        for (int j = g * SHR_THREADS + tid; j < N; j += stride) shard_step<T>(q, SH_GATE, i, j, pv);
        __syncthreads();
        const int lw = sh_cw[SC_WIN];   // this workgroup's first passing landmark
        const int m = sh_cw[SC_M];
        const double* lpk = sh_pkg;
        if (fused) {
            if (lw != 0x7fffffff) lpk = sh_slot[lw % SHR_THREADS];
        } else {
            if (lw != 0x7fffffff && lw % SHR_THREADS == tid) shard_step<T>(q, SH_PACKAGE, i, lw, pv);
            __syncthreads();
        }
        // to the mailbox (parity i & 1: a workgroup one line ahead never overwrites a slot that
        // another still reads), drained and ordered by the barrier before the tagged word
        double* slot = p.mbox + ((size_t)(i & 1) * G + g) * p.mbw;
        const int npk = MB_VH + 4 * m;
        if (lw != 0x7fffffff)
            for (int k = 1 + tid; k < npk; k += SHR_THREADS) mb_store(slot + k, lpk[k]);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) mb_tag(slot, p.epoch, (unsigned)(i + 1), (unsigned)(lw == 0x7fffffff ? 0 : lw + 1));
        for (int k = tid; k < G; k += SHR_THREADS) {
            const int bq = mb_poll(p.mbox, i & 1, G, k, p.mbw, p.epoch, (unsigned)(i + 1), status, p.spin_log2);
            if (bq < 0) sh_to = 1;
            sh_best[k] = bq <= 0 ? 0x7fffffff : bq - 1;
        }
        __syncthreads();
        if (sh_to) break;   // (uniform in the workgroup)
        int w = 0x7fffffff, gw = 0;
        for (int k = 0; k < G; k++)
            if (sh_best[k] < w) {
                w = sh_best[k];
                gw = k;
            }
        if (w != 0x7fffffff && w != sh_cw[SC_GUESS + i]) break;   // (uniform)
        if (w != 0x7fffffff && gw != g) {
            const double* ws = p.mbox + ((size_t)(i & 1) * G + gw) * p.mbw;
            for (int k = 1 + tid; k < npk; k += SHR_THREADS) sh_pkg[k] = mb_load(ws + k);
        } else if (w != 0x7fffffff && fused) {
            for (int k = 1 + tid; k < npk; k += SHR_THREADS) sh_pkg[k] = lpk[k];
        }
        if (tid == 0) sh_cw[SC_WIN] = w;
        q.col = p.cols + 4 * (size_t)i * N;
        __syncthreads();
        for (int j = g * SHR_THREADS + tid; j < N; j += stride) shard_step<T>(q, SH_APPLY, i, j, pv);
        __syncthreads();
        if (tid == 0) shard_step<T>(q, SH_ROBOT, i, 0, pv);
        __syncthreads();
    }
    // every workgroup's outcome to workgroup 0: its stopping line and whether one of its exchanges
    // timed out, one self-tagged word each (parity-0 slot, last word: the list words' region, which
    // the association kernel of a partitioned context never uses). Workgroup 0 decides the stopping
    // line over all G of them, so a workgroup that timed out — its landmarks then missed the line it
    // broke at, possibly the last one, which workgroup 0 completed — or never arrived makes the run
    // report L + 1, and the scan is abandoned on every rank
    if (tid == 0)
        mb_store_tagged(p.mbox + (size_t)g * p.mbw + p.mbw - 1, p.epoch,
                        ((unsigned long long)i << 1) | (sh_to ? 1ull : 0ull));
    if (g == 0) {
        for (int k = tid; k < G; k += SHR_THREADS) {
            int st = sh_to ? (int)EKF_ST_TIMEOUT_BIT : 0;   // (timed out already: no second wait)
            const unsigned long long w =
                mb_wait_tagged(p.mbox + (size_t)k * p.mbw + p.mbw - 1, p.epoch, st, p.spin_log2);
            if (st || (w & 1ull) || (int)(w >> 1) != i) atomicOr(&sh_bad, 1);
        }
        __syncthreads();
        if (tid == 0) {
            sh_cw[SC_NEXT] = i;
            *p.next_out = (sh_to || sh_bad) ? (double)(p.L + 1) : (double)i;
        }
    }
    __syncthreads();
    // the status bits of every workgroup's landmarks (each copy started from the same word)
    if (tid == 0) atomicOr(p.ctl + SC_STATUS, sh_cw[SC_STATUS] | (sh_to ? (int)EKF_ST_TIMEOUT_BIT : 0));
    if (g == 0) {
        for (int k = tid; k < SC_WORDS; k += SHR_THREADS)
            if (k != SC_STATUS) p.ctl[k] = sh_cw[k];
        if (tid < 12) p.rob[tid] = sh_rob[tid];
    }
}

// The speculative path's lines in the association kernel's form (ekf_shard_run with
// at most SH_MAX_LINES lines; K = ⌈N / (G·SHR_THREADS)⌉ landmarks per thread): instead of one
// exchange among the workgroups per line, every workgroup replays the guessed winners' chain itself
// from the exchanged guessed columns (p.cols, which hold every block (j, w_t), the winners' mutual
// blocks among them) and checks each line's guess on its own landmarks; one verdict exchange at the
// end. Per workgroup: two landmark waves (one landmark per thread, its record, history rows and
// flags kept in registers and LDS) and a replay wave (lane u = line u's guessed winner). Line t:
// the replay lane t evaluates its winner's gate at the state after lines < t (shard_step's
// SH_GATE sequence) and, if it passes, builds the line's package (build_package and the winner's
// V rows of the earlier matches, as SH_PACKAGE); every lane takes the robot update
// (robot_update, as SH_ROBOT) and the later winners' lanes apply the line to their winners (gain
// rows, as SH_APPLY). Meanwhile each landmark thread, per line as its package is published:
// its gate at that state (SH_GATE), a violation if it passes before the guess or while the guess
// fails, and the line's update (SH_APPLY: gain rows, history row, operand rows). The verdict (the
// first violating line over all workgroups) decides: the records, flags, history rows, control
// words and robot block are written as they stand after the lines before it (recomputed from the
// run's start when a violation cut the lines short), and *next_out = that line; the caller runs
// the per-line phases from there, as after shard_run_kernel. With several landmarks per thread
// (N > G·SHR_THREADS) each thread checks its landmarks one after the other without stores, and
// after the verdict runs each again over the lines kept, with the stores. Every value comes from
// the same functions on the same inputs as the per-line phases: bit-identical.
constexpr int SPR_THREADS = SHR_THREADS + 64;   // two landmark waves + the replay wave
template <typename T>
__global__ __launch_bounds__(SPR_THREADS) void shard_spec_kernel(ShardParams p)
{
    using C = typename Stor<T>::C;
    constexpr double ETA = gate_eta<T>();
    constexpr int SPK = MB_VH + 4 * SH_MAX_LINES;   // a package: build_package's words + the V rows
    __shared__ int sh_cw[SC_WORDS];
    __shared__ double sh_pk[SH_MAX_LINES][SPK];          // line t's package
    __shared__ double sh_robl[SH_MAX_LINES + 1][12];     // the robot block and x_pre before line t
    __shared__ int sh_pass[SH_MAX_LINES];                // line t's guessed winner passed its gate
    __shared__ int sh_ready;                              // packages published (lines < sh_ready)
    __shared__ double sh_wh[SH_MAX_LINES][SH_MAX_LINES][8];   // replay lane u: winner u's history rows
    __shared__ double sh_lh[SH_MAX_LINES][4][SHR_THREADS];    // landmark thread tid: its U rows
    __shared__ int sh_red[SPR_THREADS / 64];
    __shared__ int sh_to, sh_bad, sh_first;
    const int tid = threadIdx.x, g = blockIdx.x, G = gridDim.x;
    const Dims d = p.d;
    const int N = d.N, L = p.L;
    const bool sym = p.r_mode != 1 && sizeof(C) == 4;
    for (int k = tid; k < SC_WORDS; k += SPR_THREADS) sh_cw[k] = p.ctl[k];
    if (tid < 12) sh_robl[0][tid] = p.rob[tid];
    if (tid == 0) {
        sh_ready = 0;
        sh_to = sh_bad = 0;
        sh_first = L;
    }
    __syncthreads();
    const int s = sh_cw[SC_S];
    int tstatus = 0;

    // the operand rows of match m of landmark j (SH_APPLY's stores)
    auto store_ops = [&](int j, int m, const double (&kk)[4], const double (&uu)[4], const float (&F)[3]) {
        C* Uop = reinterpret_cast<C*>(p.cur.Uop);
        C* Vop = reinterpret_cast<C*>(p.cur.Vop);
#pragma unroll
        for (int pp = 0; pp < 2; pp++) {
            const int lr = 2 * j + pp;
            if constexpr (sizeof(C) == 4) {
                double o0 = uu[2 * pp], o1 = uu[2 * pp + 1], v0 = kk[2 * pp], v1 = kk[2 * pp + 1];
                if (sym) {
                    v0 = kk[2 * pp] * (double)F[0] + kk[2 * pp + 1] * (double)F[1];
                    v1 = kk[2 * pp + 1] * (double)F[2];
                    o0 = (double)(float)v0;
                    o1 = (double)(float)v1;
                }
                Uop[op_index_f32(lr, 2 * m, d.kmax)] = to_domain<T>(-o0, 0);
                Uop[op_index_f32(lr, 2 * m + 1, d.kmax)] = to_domain<T>(-o1, 0);
                Vop[op_index_f32(lr, 2 * m, d.kmax)] = (C)v0;
                Vop[op_index_f32(lr, 2 * m + 1, d.kmax)] = (C)v1;
            } else {
                Uop[op_index_f64(lr, 2 * m, d.kmax)] = (C)(-uu[2 * pp]);
                Uop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (C)(-uu[2 * pp + 1]);
                Vop[op_index_f64(lr, 2 * m, d.kmax)] = (C)kk[2 * pp];
                Vop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (C)kk[2 * pp + 1];
            }
        }
    };
    // the gate of one landmark at the robot state rob (SH_GATE's evaluation)
    auto gate_of = [&](const double* rob, const double2& rr0, const double2& rr1, const double2& rr2,
                       const double2& yb, const double (&Dj)[4], const double* rc, int line, Cand& c, bool& pass,
                       bool& sing, bool& amb) {
        const ekf_line ln = p.lines[line];
        double Rm[4];
        line_R(ln, line, p.r_mode, Rm);
        double R33[9], xp[3];
#pragma unroll
        for (int a = 0; a < 9; a++) R33[a] = rob[a];
        xp[0] = rob[9]; xp[1] = rob[10]; xp[2] = rob[11];
        Block5 b5;
        fill_block5(b5, R33, rr0, rr1, rr2, Dj);
        double sn, cs;
        pass = sing = amb = false;
        if (!quick_reject(b5, yb.x, yb.y, rc[12], rc[15], rc[16], xp, ln.alpha, ln.r, Rm, p.gate, ETA) &&
            (sincos_near(yb.x, rc[12], rc[13], rc[14], sn, cs),
             !certified_reject(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA))) {
            eval_candidate(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA, c);
            sing = c.singular;
            amb = c.amb;
            pass = c.pass;
        }
    };

    if (tid >= SHR_THREADS) {
        // ---- the replay wave: lane u carries line u's guessed winner up to its line ----
        const int u = tid - SHR_THREADS;
        const int wu = u < L ? sh_cw[SC_GUESS + u] : 0x7fffffff;
        const bool act = wu != 0x7fffffff && wu < N;
        double rc[SH_REC];
        if (act)
            for (int k = 0; k < SH_REC; k++) rc[k] = p.rec[(size_t)wu * SH_REC + k];
        else
            for (int k = 0; k < SH_REC; k++) rc[k] = 0.0;
        double2 rr0 = make_double2(rc[0], rc[1]), rr1 = make_double2(rc[2], rc[3]), rr2 = make_double2(rc[4], rc[5]);
        double2 yb = make_double2(rc[6], rc[7]);
        double Dj[4] = {rc[8], rc[9], rc[10], rc[11]};
        bool matched = false;
        int m = 0;
        for (int t = 0; t < L; t++) {
            const int wt = sh_cw[SC_GUESS + t];
            bool pass = false;
            if (u == t && act && !matched && wu < s) {
                // the exact evaluation without the reject filters, which never reject a landmark
                // that passes (the association kernel's replay wave does the same); its status
                // bits come from the landmark's own thread
                Cand c;
                const ekf_line ln = p.lines[t];
                double Rm[4];
                line_R(ln, t, p.r_mode, Rm);
                double R33[9], xp[3];
#pragma unroll
                for (int a = 0; a < 9; a++) R33[a] = sh_robl[t][a];
                xp[0] = sh_robl[t][9]; xp[1] = sh_robl[t][10]; xp[2] = sh_robl[t][11];
                Block5 b5;
                fill_block5(b5, R33, rr0, rr1, rr2, Dj);
                double sn, cs;
                sincos_near(yb.x, rc[12], rc[13], rc[14], sn, cs);
                eval_candidate<false>(b5, yb.x, yb.y, sn, cs, xp, ln.alpha, ln.r, Rm, p.gate, ETA, c);
                pass = c.pass;
                if (pass) {
                    build_package(c, R33, rr0, rr1, rr2, sh_pk[t]);
                    for (int q = 0; q < m; q++)
#pragma unroll
                        for (int k = 0; k < 4; k++) sh_pk[t][MB_VH + 4 * q + k] = sh_wh[u][q][4 + k];
                }
                sh_pass[t] = pass ? 1 : 0;
            } else if (u == t) {
                sh_pass[t] = 0;
            }
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const bool pt = sh_pass[t] != 0;
            // the robot block and x_pre after line t (SH_ROBOT; every lane the same bits)
            {
                double R33[9], xp[3];
#pragma unroll
                for (int a = 0; a < 9; a++) R33[a] = sh_robl[t][a];
                xp[0] = sh_robl[t][9]; xp[1] = sh_robl[t][10]; xp[2] = sh_robl[t][11];
                if (pt) robot_update(R33, xp, sh_pk[t]);
                if (u == 0) {
#pragma unroll
                    for (int a = 0; a < 9; a++) sh_robl[t + 1][a] = R33[a];
                    sh_robl[t + 1][9] = xp[0]; sh_robl[t + 1][10] = xp[1]; sh_robl[t + 1][11] = xp[2];
                }
            }
            // the later winners take line t's update (SH_APPLY on their own landmark)
            if (pt && act && u > t) {
                const double4 cb = *reinterpret_cast<const double4*>(p.cols + 4 * ((size_t)t * N + wu));
                double blk[4] = {cb.x, cb.y, cb.z, cb.w};
                const double* pk = sh_pk[t];
                double kk[4], uu[4];
                gain_rows<0>(pk, m,
                             [&](int q) { return make_double4(sh_wh[u][q][0], sh_wh[u][q][1], sh_wh[u][q][2], sh_wh[u][q][3]); },
                             [&](int q) {
                                 const double* vh = pk + MB_VH + 4 * q;
                                 return make_double4(vh[0], vh[1], vh[2], vh[3]);
                             },
                             blk, rr0, rr1, rr2, yb, Dj, kk, uu);
#pragma unroll
                for (int k = 0; k < 4; k++) {
                    sh_wh[u][m][k] = uu[k];
                    sh_wh[u][m][4 + k] = kk[k];
                }
                if (wu == wt) matched = true;
            }
            if (pt) m++;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            __builtin_amdgcn_wave_barrier();
            if (u == 0) __hip_atomic_store(&sh_ready, t + 1, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
        }
    }

    // ---- the landmark waves: landmark j = g·SHR_THREADS + tid + k·G·SHR_THREADS, k < K ----
    const int K = (N + G * SHR_THREADS - 1) / (G * SHR_THREADS);   // landmarks per thread (uniform)
    const int j0 = g * SHR_THREADS + tid;
    int stacc = 0;   // the status bits of the lines run (SH_APPLY's)
    int viol = L;    // this thread's first violating line
    // one pass over lines [0, upto) for landmark j: gates (check: the violations), updates into
    // the registers; store: the history and operand rows as they come (the same rows are
    // rewritten by the per-line phases for any line not kept)
    auto run_lines = [&](int j, const double* rc, int upto, bool check, bool store, double2& rr0, double2& rr1,
                         double2& rr2, double2& yb, double (&Dj)[4], bool& matched, int& m) {
        const bool own = tid < SHR_THREADS && j < N;
        for (int i = 0; i < upto; i++) {
            if (tid < SHR_THREADS) {
                int polls = 0;
                while (__hip_atomic_load(&sh_ready, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP) <= i) {
                    __builtin_amdgcn_s_sleep(1);
                    if ((tstatus & EKF_ST_TIMEOUT_BIT) || ++polls > (1 << p.spin_log2)) {
                        tstatus |= EKF_ST_TIMEOUT_BIT;
                        break;
                    }
                }
            }
            if (!own) continue;
            const int w = sh_cw[SC_GUESS + i];
            const bool pt = sh_pass[i] != 0;
            const int jstar = pt ? w : 0x7fffffff;
            bool pass = false, sing = false, amb = false;
            if (j < s && !matched) {
                Cand c;
                gate_of(sh_robl[i], rr0, rr1, rr2, yb, Dj, rc, i, c, pass, sing, amb);
            }
            if (check && pass && (!pt || j < w)) {   // the guess is not the line's first passing landmark
                viol = min(viol, i);
                return;
            }
            int st = sing && j <= jstar ? (int)EKF_ST_SINGULAR : 0;
            if (amb && j <= jstar) st |= EKF_ST_PRECISION_BIT;
            if (p.r_mode == 1 && (i == 1 || i == 2)) st |= EKF_ST_NSYM;
            stacc |= st;
            if (!pt) continue;
            const double4 cb = *reinterpret_cast<const double4*>(p.cols + 4 * ((size_t)i * N + j));
            double blk[4] = {cb.x, cb.y, cb.z, cb.w};
            const double* pk = sh_pk[i];
            double kk[4], uu[4];
            gain_rows<0>(pk, m,
                         [&](int q) { return make_double4(sh_lh[q][0][tid], sh_lh[q][1][tid], sh_lh[q][2][tid], sh_lh[q][3][tid]); },
                         [&](int q) {
                             const double* vh = pk + MB_VH + 4 * q;
                             return make_double4(vh[0], vh[1], vh[2], vh[3]);
                         },
                         blk, rr0, rr1, rr2, yb, Dj, kk, uu);
#pragma unroll
            for (int k = 0; k < 4; k++) {
                sh_lh[m][k][tid] = uu[k];
            }
            if (store) {
                float F[3] = {0.f, 0.f, 0.f};
                if (sym) sym_factor(pk, F);
                double* h = p.hist + ((size_t)j * d.max_lines + m) * 8;   // (SH_APPLY's history row)
                h[0] = uu[0]; h[1] = uu[1]; h[2] = uu[2]; h[3] = uu[3];
                h[4] = kk[0]; h[5] = kk[1]; h[6] = kk[2]; h[7] = kk[3];
                store_ops(j, m, kk, uu, F);
            }
            if (j == w) matched = true;
            m++;
        }
    };
    // one landmark's pass from its record at the run's start (the run starts at line 0:
    // ekf_shard_run, no match yet), its record and flag written at the end (write)
    auto run_landmark = [&](int j, int upto, bool check, bool store, bool write) {
        const bool own = tid < SHR_THREADS && j < N;
        double rc[SH_REC];
        for (int k = 0; k < SH_REC; k++) rc[k] = own ? p.rec[(size_t)j * SH_REC + k] : 0.0;
        double2 rr0 = make_double2(rc[0], rc[1]), rr1 = make_double2(rc[2], rc[3]), rr2 = make_double2(rc[4], rc[5]);
        double2 yb = make_double2(rc[6], rc[7]);
        double Dj[4] = {rc[8], rc[9], rc[10], rc[11]};
        bool matched = own && (p.flags[j] & 1);
        int m = 0;
        run_lines(j, rc, upto, check, store, rr0, rr1, rr2, yb, Dj, matched, m);
        if (write && own) {
            double* r = p.rec + (size_t)j * SH_REC;
            const double v[12] = {rr0.x, rr0.y, rr1.x, rr1.y, rr2.x, rr2.y, yb.x, yb.y, Dj[0], Dj[1], Dj[2], Dj[3]};
            for (int k = 0; k < 12; k++) r[k] = v[k];
            p.flags[j] = matched ? 1 : 0;
        }
    };
    // one landmark per thread (K = 1): its state stays in registers across the verdict and is
    // recomputed only when a violation cut the run short
    double2 rr0 = make_double2(0, 0), rr1 = rr0, rr2 = rr0, yb = rr0;
    double Dj[4] = {0, 0, 0, 0};
    bool matched = false;
    int m = 0;
    double rc0[SH_REC];
    const bool own0 = tid < SHR_THREADS && j0 < N;
    if (K == 1) {
        for (int k = 0; k < SH_REC; k++) rc0[k] = own0 ? p.rec[(size_t)j0 * SH_REC + k] : 0.0;
        rr0 = make_double2(rc0[0], rc0[1]); rr1 = make_double2(rc0[2], rc0[3]); rr2 = make_double2(rc0[4], rc0[5]);
        yb = make_double2(rc0[6], rc0[7]);
        Dj[0] = rc0[8]; Dj[1] = rc0[9]; Dj[2] = rc0[10]; Dj[3] = rc0[11];
        matched = own0 && (p.flags[j0] & 1);
        run_lines(j0, rc0, L, true, true, rr0, rr1, rr2, yb, Dj, matched, m);
    } else {
        // several landmarks per thread: check each in turn (no stores; lines at or past an earlier
        // violation of this thread are never kept), the stores after the verdict
        for (int k = 0; k < K; k++) run_landmark(j0 + k * G * SHR_THREADS, viol, true, false, false);
    }
    // ---- the verdict: the first violating line over every workgroup (one exchange) ----
    {
        int v = viol;
#pragma unroll
        for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
        if ((tid & 63) == 0) sh_red[tid >> 6] = v;
        __syncthreads();
        int wv = L;
        for (int w = 0; w < SHR_THREADS / 64; w++) wv = min(wv, sh_red[w]);
        double* slot = p.mbox + (size_t)g * p.mbw;
        if (tid == 0) mb_tag(slot, p.epoch, TAG_SPEC_VERDICT, (unsigned)(wv + 1));
        for (int k = tid; k < G; k += SPR_THREADS) {
            const int bq = mb_poll(p.mbox, 0, G, k, p.mbw, p.epoch, TAG_SPEC_VERDICT, tstatus, p.spin_log2);
            if (bq <= 0) sh_to = 1;
            else atomicMin(&sh_first, bq - 1);
        }
        if (tstatus & EKF_ST_TIMEOUT_BIT) sh_to = 1;
        __syncthreads();
    }
    const int first = sh_to ? 0 : sh_first;
    if (K == 1) {
        // the state after the lines before `first` (recomputed when the run was cut short)
        if (first < L && !sh_to) {
            rr0 = make_double2(rc0[0], rc0[1]); rr1 = make_double2(rc0[2], rc0[3]); rr2 = make_double2(rc0[4], rc0[5]);
            yb = make_double2(rc0[6], rc0[7]);
            Dj[0] = rc0[8]; Dj[1] = rc0[9]; Dj[2] = rc0[10]; Dj[3] = rc0[11];
            matched = own0 && (p.flags[j0] & 1);
            m = 0;
            stacc = 0;
            run_lines(j0, rc0, first, false, true, rr0, rr1, rr2, yb, Dj, matched, m);
        }
        if (own0 && !sh_to) {
            double* r = p.rec + (size_t)j0 * SH_REC;
            const double v[12] = {rr0.x, rr0.y, rr1.x, rr1.y, rr2.x, rr2.y, yb.x, yb.y, Dj[0], Dj[1], Dj[2], Dj[3]};
            for (int k = 0; k < 12; k++) r[k] = v[k];
            p.flags[j0] = matched ? 1 : 0;
        }
    } else if (!sh_to) {
        stacc = 0;
        for (int k = 0; k < K; k++) run_landmark(j0 + k * G * SHR_THREADS, first, false, true, true);
    }
    const bool own = own0 || (K > 1 && tid < SHR_THREADS);
    int st = own ? stacc : 0;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) st |= __shfl_xor(st, off, 64);
    __syncthreads();
    if ((tid & 63) == 0) sh_red[tid >> 6] = st;
    __syncthreads();
    // every workgroup's outcome to workgroup 0 (as shard_run_kernel): a workgroup whose verdict
    // poll timed out makes the run report L + 1, and the scan is abandoned on every rank
    if (tid == 0) {
        int wst = 0;
        for (int w = 0; w < SPR_THREADS / 64; w++) wst |= sh_red[w];
        atomicOr(p.ctl + SC_STATUS, wst | (sh_to ? (int)EKF_ST_TIMEOUT_BIT : 0));
        mb_store_tagged(p.mbox + (size_t)g * p.mbw + p.mbw - 1, p.epoch,
                        ((unsigned long long)first << 1) | (sh_to ? 1ull : 0ull));
    }
    if (g == 0) {
        for (int k = tid; k < G; k += SPR_THREADS) {
            int stw = sh_to ? (int)EKF_ST_TIMEOUT_BIT : 0;
            const unsigned long long w = mb_wait_tagged(p.mbox + (size_t)k * p.mbw + p.mbw - 1, p.epoch, stw, p.spin_log2);
            if (stw || (w & 1ull) || (int)(w >> 1) != first) atomicOr(&sh_bad, 1);
        }
        __syncthreads();
        if (tid == 0) {
            // the control words after the lines kept (SH_ROBOT's bookkeeping, line by line)
            int mm = 0, nx = sh_cw[SC_NEXTRA];
            for (int i = 0; i < first; i++) {
                if (sh_pass[i]) {
                    sh_cw[SC_MATCH + i] = sh_cw[SC_GUESS + i];
                    mm++;
                } else {
                    sh_cw[SC_MATCH + i] = -1;
                    sh_cw[SC_EXTRA + nx] = i;
                    nx++;
                }
            }
            sh_cw[SC_M] += mm;
            sh_cw[SC_NEXTRA] = nx;
            sh_cw[SC_WIN] = 0x7fffffff;
            sh_cw[SC_NEXT] = first;
            *p.next_out = (sh_to || sh_bad) ? (double)(L + 1) : (double)first;
        }
        __syncthreads();
        for (int k = tid; k < SC_WORDS; k += SPR_THREADS)
            if (k != SC_STATUS) p.ctl[k] = sh_cw[k];
        if (tid < 12) p.rob[tid] = sh_robl[first][tid];
    }
}

#pragma clang fp contract(fast)

// ---------------------------------------------------------------------------------------
// 2. covariance downdate of the landmark block on MFMA, one pass for a group of steps
// ---------------------------------------------------------------------------------------
// For every stored 32×32 tile and every step of the group, in order: the capacity reset
// (Robot.cpp:893-904), or X ← X − U_t·V_tᵀ summed over the step's matches (rank 2m, the
// reference's m dense passes of Robot.cpp:560-572) followed by the rows of the landmarks that
// step appended (Robot.cpp:845-862). The tile stays in the MFMA accumulators for the whole
// group: one HBM read and one write per tile per group.
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

// value of landmark-block element (i, j) written by a step's augmentation
__device__ __forceinline__ double patched_value(const double* prw0, const double* pdg, int M,
                                                int s0, int i, int j)
{
    const int li = i >> 1, lj = j >> 1;
    const int hi = li > lj ? li : lj;
    const int qa = hi - s0;
    if (li == lj) return pdg[qa * 4 + (i & 1) * 2 + (j & 1)];
    const double* prw = prw0 + (size_t)qa * 2 * M;
    return (li > lj) ? prw[(size_t)(i & 1) * M + j] : prw[(size_t)(j & 1) * M + i];
}

// fp32-layout tiles in fp32 or fp16 storage: lane's 4 consecutive elements of accumulator group qq
typedef _Float16 f16x4 __attribute__((ext_vector_type(4)));

template <typename TS>
__device__ __forceinline__ f32x4 tile_ld(const TS* tile, int lane, int qq)
{
    if constexpr (sizeof(TS) == 4) {
        return __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(tile) + lane + qq * 64);
    } else {
        const f16x4 h = __builtin_nontemporal_load(reinterpret_cast<const f16x4*>(tile) + lane + qq * 64);
        return f32x4{(float)h[0], (float)h[1], (float)h[2], (float)h[3]};
    }
}

template <typename TS>
__device__ __forceinline__ void tile_st(TS* tile, int lane, int qq, const f32x16& a)
{
    if constexpr (sizeof(TS) == 4) {
        const f32x4 v = {a[4 * qq + 0], a[4 * qq + 1], a[4 * qq + 2], a[4 * qq + 3]};
        __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(tile) + lane + qq * 64);
    } else {
        const f16x4 v = {(_Float16)a[4 * qq + 0], (_Float16)a[4 * qq + 1], (_Float16)a[4 * qq + 2],
                         (_Float16)a[4 * qq + 3]};
        __builtin_nontemporal_store(v, reinterpret_cast<f16x4*>(tile) + lane + qq * 64);
    }
}


// fp16 storage: the value a step leaves in the block is its fp16 rounding (see Stor)
template <typename TS>
__device__ __forceinline__ void round_acc(f32x16& a)
{
    if constexpr (sizeof(TS) == 2) {
#pragma unroll
        for (int k = 0; k < 16; k++) a[k] = round_step<_Float16>(a[k]);
    }
}

// f32 flush on super-tiles: a workgroup owns DD_SB × DD_SB tiles (wave w: tile row
// sbi·DD_SB + w, tile columns sbj·DD_SB + 0..3), keeps their 4 accumulators in registers for
// the whole group of steps and stages each step's operands for the DD_SB row blocks and DD_SB
// column blocks through LDS in chunks of 8 MFMA k-steps (double-buffered, one barrier per
// chunk, next chunk prefetched into registers while the current one runs). Operand traffic
// per tile and k-step falls from 512 B to 128 B; the MFMA chain per element is unchanged
// (k-ordered within a step, steps in order), so results are bit-identical to the per-tile form.
namespace {
constexpr int SBK = 8;   // MFMA k-steps per staged chunk (2 float4 per lane per block)

struct SbStep {
    int reset, ks, nadd, s0;
};

__device__ __forceinline__ SbStep sb_step(const DowndateParams& p, int q, int e)
{
    const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
    SbStep s;
    s.reset = r[RES_RESET];
    s.ks = s.reset ? 0 : r[RES_KSTEPS];
    s.nadd = r[RES_NADD];
    s.s0 = r[RES_SAVED_IN];
    return s;
}
}  // namespace

template <typename TS>
__global__ __launch_bounds__(DD_THREADS) void flush_f32_sb_kernel(DowndateParams p)
{
    const Dims d = p.d;
    const int nsb = (d.nb + DD_SB - 1) / DD_SB;
    const int64_t nst = (int64_t)nsb * (nsb + 1) / 2;
    const int64_t total = (int64_t)p.E * nst;
    // XCD-aware order: the hardware deals workgroup b to XCD b mod 8; give every XCD a
    // contiguous range of (instance, super-tile) so that its L2 holds one instance's operands
    const int64_t per = (total + 7) / 8;
    const int64_t g = (int64_t)(blockIdx.x & 7) * per + (blockIdx.x >> 3);
    if (g >= total) return;
    const int e = (int)(g / nst);
    const int2 sb = p.stile_rc[g - (int64_t)e * nst];
    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int bi = sb.x * DD_SB + w;
    const int kh = d.kmax / 2;
    const size_t opstride = (size_t)d.nb * 64 * kh;

    // does any step change this super-tile? (uniform)
    bool work = false;
    for (int q = 0; q < p.nsteps; q++) {
        const SbStep s = sb_step(p, q, e);
        work |= s.reset || s.ks > 0 ||
                (s.nadd > 0 && (sb.y + 1) * DD_SB * 16 > s.s0 && sb.y * DD_SB * 16 < s.s0 + s.nadd);
    }
    bool valid[DD_SB];
    size_t toff[DD_SB];
    int vmask = 0;
#pragma unroll
    for (int c = 0; c < DD_SB; c++) {
        const int bj = sb.y * DD_SB + c;
        valid[c] = bi < d.nb && bj < d.nb && bi <= bj;
        vmask |= valid[c] << c;
        toff[c] = valid[c] ? ((size_t)e * d.ntiles + tile_index(bi, bj, d.nb)) * TILE_ELEMS : 0;
    }
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    if (!work) {
        if (p.Pin != p.Pout) {
#pragma unroll
            for (int c = 0; c < DD_SB; c++)
                if (valid[c]) {
                    f32x16 t;
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) {
                        const f32x4 v = tile_ld(Pin + toff[c], lane, qq);
                        t[4 * qq + 0] = v[0]; t[4 * qq + 1] = v[1]; t[4 * qq + 2] = v[2]; t[4 * qq + 3] = v[3];
                    }
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) tile_st(Pout + toff[c], lane, qq, t);
                }
        }
        return;
    }
    f32x16 acc[DD_SB];
#pragma unroll
    for (int c = 0; c < DD_SB; c++) {
        if (valid[c]) {
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                const f32x4 v = tile_ld(Pin + toff[c], lane, qq);
                acc[c][4 * qq + 0] = v[0];
                acc[c][4 * qq + 1] = v[1];
                acc[c][4 * qq + 2] = v[2];
                acc[c][4 * qq + 3] = v[3];
            }
        } else {
#pragma unroll
            for (int k = 0; k < 16; k++) acc[c][k] = 0.f;
        }
    }

    // [buf][A/B][block][s4][lane] float4: 2 × 2 × 4 × 2 × 64 × 16 B = 32 KB
    __shared__ f32x4 lds[2][2][DD_SB][2][64];
    // staging: thread t moves float4 i = t + 256 j (j < 4): lane, s4, block, A/B
    const float us = us_of<TS>(p, e);
    auto fetch = [&](int q, int k0, f32x4 reg[4]) {
        const float* U = u_rows_flush(p, p.steps[q], e, opstride);
        const float* V = reinterpret_cast<const float*>(p.steps[q].Vop) + e * opstride;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = threadIdx.x + 256 * j;
            const int ln = i & 63, s4 = (i >> 6) & 1, blk = (i >> 7) & 3, ab = i >> 9;
            const int rb = (ab ? sb.y : sb.x) * DD_SB + blk;
            if (rb < d.nb) {
                const float* src = (ab ? V : U) + ((size_t)rb * 64 + ln) * kh + k0 + 4 * s4;
                reg[j] = *reinterpret_cast<const f32x4*>(src) * (ab ? 1.0f : us);
            }
        }
    };
    auto stage = [&](int buf, const f32x4 reg[4]) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int i = threadIdx.x + 256 * j;
            const int ln = i & 63, s4 = (i >> 6) & 1, blk = (i >> 7) & 3, ab = i >> 9;
            lds[buf][ab][blk][s4][ln] = reg[j];
        }
    };
    // reset or augmented rows of step q, after its downdate
    auto post = [&](int q) {
        const SbStep s = sb_step(p, q, e);
        if (s.reset) {
#pragma unroll
            for (int c = 0; c < DD_SB; c++)
#pragma unroll
                for (int k = 0; k < 16; k++) acc[c][k] = 0.f;
            return;
        }
        if (s.nadd <= 0) return;
        const double* prw0 = p.steps[q].patch + (size_t)e * d.max_lines * 2 * d.M;
        const double* pdg = p.steps[q].patch_diag + (size_t)e * d.max_lines * 4;
        // one tile at a time through acc[0], rotating the four accumulators (rare path: keeps
        // a single copy of the per-element code and its registers)
#pragma nounroll
        for (int c = 0; c < DD_SB; c++) {
            const int bj = sb.y * DD_SB + c;
            if (((vmask >> c) & 1) && bj * 16 + 15 >= s.s0 && bj * 16 < s.s0 + s.nadd) {
                const int col = bj * 32 + (lane & 31);
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int row = bi * 32 + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
                    const int hi = max(row >> 1, col >> 1);
                    if (hi >= s.s0 && hi < s.s0 + s.nadd)
                        acc[0][k] = round_step<TS>(to_domain<TS>(patched_value(prw0, pdg, d.M, s.s0, row, col), storage_exp<TS>(p.pexp, e)));
                }
            }
            const f32x16 t0 = acc[0];
            acc[0] = acc[1];
            acc[1] = acc[2];
            acc[2] = acc[3];
            acc[3] = t0;
        }
    };
    // first chunk at or after step q (k0 = 0): steps without a downdate are passed through post
    auto first_mfma = [&](int q) {
        while (q < p.nsteps && sb_step(p, q, e).ks == 0) q++;
        return q;
    };

    int q = first_mfma(0);
    for (int t = 0; t < q; t++) post(t);
    int k0 = 0, buf = 0;
    f32x4 reg[4];
    if (q < p.nsteps) fetch(q, 0, reg);
    while (q < p.nsteps) {
        const int ks = sb_step(p, q, e).ks;
        const int kc = min(SBK, ks - k0);
        stage(buf, reg);
        __syncthreads();
        // next chunk
        int qn = q, kn = k0 + SBK;
        if (kn >= ks) {
            qn = first_mfma(q + 1);
            kn = 0;
        }
        if (qn < p.nsteps) fetch(qn, kn, reg);
        const f32x4 a0 = lds[buf][0][w][0][lane];
        const f32x4 a1 = lds[buf][0][w][1][lane];
        f32x4 b0[DD_SB], b1[DD_SB];
#pragma unroll
        for (int c = 0; c < DD_SB; c++) {
            b0[c] = lds[buf][1][c][0][lane];
            b1[c] = lds[buf][1][c][1][lane];
        }
        {
#pragma unroll
            for (int s = 0; s < SBK; s++)
                if (s < kc) {
#pragma unroll
                    for (int c = 0; c < DD_SB; c++)
                        acc[c] = __builtin_amdgcn_mfma_f32_32x32x2f32(s < 4 ? a0[s & 3] : a1[s & 3],
                                                                      s < 4 ? b0[c][s & 3] : b1[c][s & 3],
                                                                      acc[c], 0, 0, 0);
                }
        }
        if (qn != q) {
#pragma unroll
            for (int c = 0; c < DD_SB; c++) round_acc<TS>(acc[c]);
            for (int t = q; t < qn && t < p.nsteps; t++) post(t);
        }
        q = qn;
        k0 = kn;
        buf ^= 1;
    }
#pragma unroll
    for (int c = 0; c < DD_SB; c++)
        if (valid[c]) {
#pragma unroll
            for (int qq = 0; qq < 4; qq++) tile_st(Pout + toff[c], lane, qq, acc[c]);
        }
}

// Groups of at most PST_MAXC steps with kmax <= 16 (one operand chunk per step) run the
// persistent form below; otherwise flush_f32_sb_kernel runs.
constexpr int PST_MAXC = 4;

// scalar (constant address space) load of a wave-uniform word that no kernel of this launch
// writes: keeps the control words on lgkmcnt, out of the vmcnt queue the prefetch occupies
template <typename T>
__device__ __forceinline__ T sload(const T* ptr)
{
    return *(const __attribute__((address_space(4))) T*)(ptr);
}

// f32/f16 flush, persistent 2-workgroups-per-CU form: super-tiles of 4 × 2 tiles (wave w: tile
// row sbi·4 + w, tile columns sbj·2 + 0..1), two accumulators per wave, single-buffered LDS
// operands (48 KB: 4 A blocks + 2 B blocks per chunk), two barriers per super-tile. Two
// independent workgroups per CU (≤ 256 registers per wave) let one workgroup's MFMA chains run
// while the other stages, waits or streams. Per super-tile the control is four scalar words
// (instance, super-tile, packed step flags); when every step of the group is a full 8-k-step
// downdate with nothing else to apply (the steady state) the MFMA block runs without predicates.
constexpr int P2_C = 2;   // tile columns per super-tile

struct P2Info {
    int e, sbi, sbj;
    int flags;   // per step q, byte q: bits 0-3 ks, bit 4 reset, bit 5 augmented rows present
};

template <typename TS>
__global__ __launch_bounds__(DD_THREADS, 2) void flush_f32_persist2_kernel(DowndateParams p)
{
    const Dims d = p.d;
    const int nst = p.nstiles2;
    const int total = p.E * nst;
    const int per = (total + 7) / 8;
    const int xcd = blockIdx.x & 7;
    const int wpx = gridDim.x >> 3;
    const int g_end = min(total, (xcd + 1) * per);
    int g = xcd * per + (blockIdx.x >> 3);
    if (g >= g_end) return;

    const int lane = threadIdx.x & 63;
    const int w = threadIdx.x >> 6;
    const int kh = d.kmax / 2;
    const size_t opstride = (size_t)d.nb * 64 * kh;
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    const int nsteps = p.nsteps;
    // this thread's staging slots j < 3 of a chunk: float4 i = tid + 256 j of
    // [A: 4 blocks × 2 × 64 | B: 2 blocks × 2 × 64]; offsets inside a block row are invariant
    const int ln = threadIdx.x & 63, s4 = (threadIdx.x >> 6) & 1, bl = threadIdx.x >> 7;
    const int in_blk = ln * kh + 4 * s4;

    auto load_flags = [&](P2Info& t) {
        int f = 0;
#pragma unroll
        for (int q = 0; q < PST_MAXC; q++) {
            if (q < nsteps) {
                const int* r = p.steps[q].res + (size_t)t.e * RES_STRIDE;
                const int reset = sload(r + RES_RESET);
                const int ks = reset ? 0 : sload(r + RES_KSTEPS);
                const int nadd = sload(r + RES_NADD);
                f |= ((ks & 15) | (reset ? 16 : 0) | (nadd > 0 ? 32 : 0)) << (8 * q);
            }
        }
        t.flags = f;
    };
    auto locate = [&](int li, P2Info& t) {
        const int* rc = reinterpret_cast<const int*>(p.stile2_rc + li);
        t.sbi = sload(rc);
        t.sbj = sload(rc + 1);
    };
    auto tile_off = [&](const P2Info& t, int c, bool& valid) {
        const int bi = t.sbi * DD_SB + w, bj = t.sbj * P2_C + c;
        valid = bi < d.nb && bj < d.nb && bi <= bj;
        return valid ? ((size_t)t.e * d.ntiles + tile_index(bi, bj, d.nb)) * TILE_ELEMS : (size_t)0;
    };
    auto fetch = [&](const P2Info& t, f32x4 opreg[PST_MAXC][3], f32x4 pref[P2_C][4]) {
        const int rA0 = min(t.sbi * DD_SB + bl, d.nb - 1), rA1 = min(t.sbi * DD_SB + 2 + bl, d.nb - 1);
        const int rB = min(t.sbj * P2_C + bl, d.nb - 1);   // rows past the block: unused
#pragma unroll
        for (int c = 0; c < PST_MAXC; c++) {
            const int qc = ((t.flags >> (8 * c)) & 15) ? c : 0;   // absent steps re-read step 0
            const float* U = u_rows_flush(p, p.steps[qc], t.e, opstride);
            const float* V = reinterpret_cast<const float*>(p.steps[qc].Vop) + t.e * opstride;
            const float us = us_of<TS>(p, t.e);
            opreg[c][0] = *reinterpret_cast<const f32x4*>(U + (size_t)rA0 * 64 * kh + in_blk) * us;
            opreg[c][1] = *reinterpret_cast<const f32x4*>(U + (size_t)rA1 * 64 * kh + in_blk) * us;
            opreg[c][2] = *reinterpret_cast<const f32x4*>(V + (size_t)rB * 64 * kh + in_blk);
        }
#pragma unroll
        for (int c = 0; c < P2_C; c++) {
            bool v;
            const TS* tl = Pin + tile_off(t, c, v);
#pragma unroll
            for (int qq = 0; qq < 4; qq++) pref[c][qq] = tile_ld(tl, lane, qq);
        }
    };
    __shared__ f32x4 ldsA[PST_MAXC][DD_SB][2][64];   // 32 KB
    __shared__ f32x4 ldsB[PST_MAXC][P2_C][2][64];    // 16 KB
    P2Info cur;
    cur.e = __builtin_amdgcn_readfirstlane(g / nst);
    int li = __builtin_amdgcn_readfirstlane(g - cur.e * nst);
    locate(li, cur);
    load_flags(cur);
    f32x4 opreg[PST_MAXC][3];
    f32x4 pref[P2_C][4];
    fetch(cur, opreg, pref);
    f32x16 acc[P2_C];
    // steady state: every step of the group a full chunk, no reset, no augmented rows
    int steady = 0;
#pragma unroll
    for (int q = 0; q < PST_MAXC; q++) steady |= (q < nsteps ? SBK : 0) << (8 * q);

    while (true) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // LDS free
#pragma unroll
        for (int c = 0; c < PST_MAXC; c++) {
            if ((cur.flags >> (8 * c)) & 15) {
                ldsA[c][bl][s4][ln] = opreg[c][0];
                ldsA[c][2 + bl][s4][ln] = opreg[c][1];
                ldsB[c][bl][s4][ln] = opreg[c][2];
            }
        }
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");   // LDS written
#pragma unroll
        for (int c = 0; c < P2_C; c++)
#pragma unroll
            for (int qq = 0; qq < 4; qq++) {
                acc[c][4 * qq + 0] = pref[c][qq][0];
                acc[c][4 * qq + 1] = pref[c][qq][1];
                acc[c][4 * qq + 2] = pref[c][qq][2];
                acc[c][4 * qq + 3] = pref[c][qq][3];
            }
        // next super-tile in flight (the last iteration re-reads its own)
        const int gn = g + wpx;
        const bool more = gn < g_end;
        P2Info nxt;
        nxt.e = cur.e;
        int lin = li;
        if (more) {
            lin += wpx;
            while (lin >= nst) {
                lin -= nst;
                nxt.e++;
            }
        }
        locate(lin, nxt);
        load_flags(nxt);
        fetch(nxt, opreg, pref);

        const int e = cur.e;
        const int bi = cur.sbi * DD_SB + w;
        if (cur.flags == steady) {
            __builtin_amdgcn_s_setprio(1);   // this MFMA cluster ahead of the partner's staging
#pragma unroll
            for (int q = 0; q < PST_MAXC; q++) {
                if (q < nsteps) {
                    const f32x4 a0 = ldsA[q][w][0][lane];
                    const f32x4 a1 = ldsA[q][w][1][lane];
                    const f32x4 b00 = ldsB[q][0][0][lane], b01 = ldsB[q][0][1][lane];
                    const f32x4 b10 = ldsB[q][1][0][lane], b11 = ldsB[q][1][1][lane];
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b00[s], acc[0], 0, 0, 0);
                        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a0[s], b10[s], acc[1], 0, 0, 0);
                    }
#pragma unroll
                    for (int s = 0; s < 4; s++) {
                        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b01[s], acc[0], 0, 0, 0);
                        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a1[s], b11[s], acc[1], 0, 0, 0);
                    }
                    round_acc<TS>(acc[0]);
                    round_acc<TS>(acc[1]);
                }
            }
            __builtin_amdgcn_s_setprio(0);
        } else {
            int vmask = 0;
#pragma unroll
            for (int c = 0; c < P2_C; c++) {
                bool v;
                (void)tile_off(cur, c, v);
                vmask |= (int)v << c;
            }
            auto post = [&](int q) {
                const int fq = (cur.flags >> (8 * q)) & 255;
                if (fq & 16) {
#pragma unroll
                    for (int c = 0; c < P2_C; c++)
#pragma unroll
                        for (int k = 0; k < 16; k++) acc[c][k] = 0.f;
                    return;
                }
                if (!(fq & 32)) return;
                const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
                const int nadd = sload(r + RES_NADD), s0 = sload(r + RES_SAVED_IN);
                if ((cur.sbj + 1) * P2_C * 16 <= s0 || cur.sbj * P2_C * 16 >= s0 + nadd) return;
                const double* prw0 = p.steps[q].patch + (size_t)e * d.max_lines * 2 * d.M;
                const double* pdg = p.steps[q].patch_diag + (size_t)e * d.max_lines * 4;
                const int ex = storage_exp<TS>(p.pexp, e);
#pragma nounroll
                for (int c = 0; c < P2_C; c++) {
                    const int bj = cur.sbj * P2_C + c;
                    if (((vmask >> c) & 1) && bj * 16 + 15 >= s0 && bj * 16 < s0 + nadd) {
                        const int col = bj * 32 + (lane & 31);
#pragma unroll
                        for (int k = 0; k < 16; k++) {
                            const int row = bi * 32 + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
                            const int hi = max(row >> 1, col >> 1);
                            if (hi >= s0 && hi < s0 + nadd)
                                acc[0][k] = round_step<TS>(to_domain<TS>(patched_value(prw0, pdg, d.M, s0, row, col), ex));
                        }
                    }
                    const f32x16 t0 = acc[0];
                    acc[0] = acc[1];
                    acc[1] = t0;
                }
            };
#pragma unroll
            for (int q = 0; q < PST_MAXC; q++) {
                if (q >= nsteps) break;
                const int kc = (cur.flags >> (8 * q)) & 15;
                if (kc > 0) {
                    const f32x4 a0 = ldsA[q][w][0][lane];
                    const f32x4 a1 = ldsA[q][w][1][lane];
                    f32x4 b0[P2_C], b1[P2_C];
#pragma unroll
                    for (int cc = 0; cc < P2_C; cc++) {
                        b0[cc] = ldsB[q][cc][0][lane];
                        b1[cc] = ldsB[q][cc][1][lane];
                    }
#pragma unroll
                    for (int s = 0; s < SBK; s++)
                        if (s < kc) {
#pragma unroll
                            for (int cc = 0; cc < P2_C; cc++)
                                acc[cc] = __builtin_amdgcn_mfma_f32_32x32x2f32(s < 4 ? a0[s & 3] : a1[s & 3],
                                                                               s < 4 ? b0[cc][s & 3] : b1[cc][s & 3],
                                                                               acc[cc], 0, 0, 0);
                        }
#pragma unroll
                    for (int cc = 0; cc < P2_C; cc++) round_acc<TS>(acc[cc]);
                }
                post(q);
            }
        }
#pragma unroll
        for (int c = 0; c < P2_C; c++) {
            bool v;
            const size_t off = tile_off(cur, c, v);
            if (v) {
#pragma unroll
                for (int qq = 0; qq < 4; qq++) tile_st(Pout + off, lane, qq, acc[c]);
            }
        }
        if (!more) break;
        g = gn;
        li = lin;
        cur = nxt;
    }
}

// One WT_R × WT_C wave-tile (instance e, table entry w) through a group of NS steps in order, operands
// loaded in place: per step its reset, or the rank-2m downdate (v_mfma_f32_32x32x2_f32, the exact
// k-ordered chain, fp16 rounding per step; once per group, at the store, under p.bf) and then its augmented rows (one tile at a time through
// acc[0], rotating the accumulators). Tiles outside the triangle are stored to the sink tile. The
// general path of the wave flushes (groups with a reset or new rows in some instance of the wave).
template <typename TS, int NS>
__device__ __forceinline__ void wt_general(const DowndateParams& p, int e, const WtEntry& w, int lane)
{
    const Dims d = p.d;
    const int kh = d.kmax / 2;
    const size_t opstride = (size_t)d.nb * 64 * kh;
    const size_t inst_elems = (size_t)d.ntiles * TILE_ELEMS;
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    TS* sink = reinterpret_cast<TS*>(p.sink);
    const int lofs = lane * kh;
    auto op_row = [&](int side, int k) { return (w.rows[side] >> (16 * k)) & 0xffff; };
    f32x16 acc[WT_N];
#pragma unroll
    for (int i = 0; i < WT_N; i++) {
        const TS* tl = Pin + (size_t)e * inst_elems + (size_t)w.tile[i] * TILE_ELEMS;
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const f32x4 v = tile_ld(tl, lane, qq);
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][4 * qq + j] = v[j];
        }
    }
    const int wr = w.rc & 0xffff, wc = w.rc >> 16;
    for (int q = 0; q < NS; q++) {
        const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
        const int reset = sload(r + RES_RESET);
        const int kc = reset ? 0 : sload(r + RES_KSTEPS);
        if (kc > 0) {
            const float* U = u_rows_flush(p, p.steps[q], e, opstride) + lofs;
            const float* V = reinterpret_cast<const float*>(p.steps[q].Vop) + e * opstride + lofs;
            const float us = us_of<TS>(p, e);
            f32x4 a[WT_R][2], b[WT_C][2];
#pragma unroll
            for (int rr = 0; rr < WT_R; rr++) {
                const float* src = U + (size_t)op_row(0, rr) * 64 * kh;
                a[rr][0] = *reinterpret_cast<const f32x4*>(src) * us;
                a[rr][1] = *reinterpret_cast<const f32x4*>(src + 4) * us;
            }
#pragma unroll
            for (int c = 0; c < WT_C; c++) {
                const float* src = V + (size_t)op_row(1, c) * 64 * kh;
                b[c][0] = *reinterpret_cast<const f32x4*>(src);
                b[c][1] = *reinterpret_cast<const f32x4*>(src + 4);
            }
#pragma unroll
            for (int s = 0; s < SBK; s++)
                if (s < kc) {
#pragma unroll
                    for (int rr = 0; rr < WT_R; rr++)
#pragma unroll
                        for (int c = 0; c < WT_C; c++)
                            acc[rr * WT_C + c] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                a[rr][s >> 2][s & 3], b[c][s >> 2][s & 3], acc[rr * WT_C + c], 0, 0, 0);
                }
            if (!p.bf) {   // split-bf16 flushes round fp16 storage once per group (at the store)
#pragma unroll
                for (int i = 0; i < WT_N; i++) round_acc<TS>(acc[i]);
            }
        }
        if (reset) {
#pragma unroll
            for (int i = 0; i < WT_N; i++)
#pragma unroll
                for (int k = 0; k < 16; k++) acc[i][k] = 0.f;
            continue;
        }
        const int nadd = sload(r + RES_NADD), s0 = sload(r + RES_SAVED_IN);
        if (nadd <= 0 || (wc + 1) * WT_C * 16 <= s0 || wc * WT_C * 16 >= s0 + nadd) continue;
        const double* prw0 = p.steps[q].patch + (size_t)e * d.max_lines * 2 * d.M;
        const double* pdg = p.steps[q].patch_diag + (size_t)e * d.max_lines * 4;
        const int ex = storage_exp<TS>(p.pexp, e);
#pragma nounroll
        for (int i = 0; i < WT_N; i++) {
            const int bi = wr * WT_R + i / WT_C, bj = wc * WT_C + i % WT_C;
            if (((w.valid >> i) & 1) && bj * 16 + 15 >= s0 && bj * 16 < s0 + nadd) {
                const int col = bj * 32 + (lane & 31);
#pragma unroll
                for (int k = 0; k < 16; k++) {
                    const int row = bi * 32 + (k & 3) + 8 * (k >> 2) + 4 * (lane >> 5);
                    const int hi = max(row >> 1, col >> 1);
                    if (hi >= s0 && hi < s0 + nadd) {
                        const float v = to_domain<TS>(patched_value(prw0, pdg, d.M, s0, row, col), ex);
                        acc[0][k] = p.bf ? v : round_step<TS>(v);
                    }
                }
            }
            const f32x16 t0 = acc[0];
#pragma unroll
            for (int j = 0; j < WT_N - 1; j++) acc[j] = acc[j + 1];
            acc[WT_N - 1] = t0;
        }
    }
#pragma unroll
    for (int i = 0; i < WT_N; i++) {
        TS* tl = ((w.valid >> i) & 1) ? Pout + (size_t)e * inst_elems + (size_t)w.tile[i] * TILE_ELEMS : sink;
#pragma unroll
        for (int qq = 0; qq < 4; qq++) tile_st(tl, lane, qq, acc[i]);
    }
}

// f32/f16 flush, barrier-free per-wave form for groups of an even number of steps NS (2..8,
// kmax <= 16). One wave per SIMD, each working alone (no LDS, no barriers) through a sequence of
// wave-tiles of WT_R × WT_C tiles (four 32×32 accumulators). Software pipeline, one wave-tile
// deep: while wave-tile k runs its NS·32 MFMAs, the tiles of wave-tile k+1 (issued first) and its
// operand rows (step q's issued right after step q's MFMAs free their registers) stream into
// registers, so every wait of a wave-tile covers only loads issued during the one before it. The
// host table wt (WtEntry) gives each wave-tile's tile indices, operand row blocks and validity;
// the entry of wave-tile k+2 is read (scalar loads) during wave-tile k. The wave-tiles of an
// instance are walked in panels and each XCD takes a contiguous range of (instance, wave-tile),
// so the wave-tiles an XCD has in flight share their operand rows in its L2. This pipelined loop
// serves the groups in which no step of the wave's instances resets the map or adds landmarks
// (partial downdates are predicated); otherwise the wave runs a plain per-wave-tile loop. Per
// element the chain is the one every other form runs (k-ordered MFMA steps, fp16 rounding per
// step, then the step's rows or the reset): bit-identical results.
//
// BF (EKF_ARITH_BF16X6, fp32 storage, symmetric operands): the plain groups run each step as six
// v_mfma_f32_32x32x16_bf16 per accumulator on V's exact three-part bf16 split (the scan's
// planes, Slot::Bop). With U = −V the accumulators hold −X (negated on load and store, exact), so
// both operands are V planes: of the wave-tile's row blocks (A) and column blocks (B). Operands
// stream through a ring of RD step-sets, RD − 1 steps ahead, across wave-tile boundaries.
// split-plane flushes: one wave per SIMD (two at <= 256 registers and a ring of 2 measured equal;
// scripts/xp/f16_wave_switches.patch restores that and the other A/B switches of this form)
constexpr int F16_RDMAX = 8;   // split-fp16 flush: the deepest operand ring (step-sets)
// the largest divisor of ns not above rmax (at least 2)
constexpr int ring_depth(int ns, int rmax)
{
    int r = 2;
    for (int k = 2; k <= rmax; k++)
        if (ns % k == 0) r = k;
    return r;
}
template <typename TS, int NS, bool BF = false, bool F16 = false>
__global__ __launch_bounds__(DD_THREADS, 1) void flush_f32_wave_kernel(DowndateParams p)
{
    static_assert(NS >= 2 && NS % 2 == 0 && NS <= PMAX, "even step count");
    static_assert(BF || NS <= 8, "fp32 wave flush: at most 8 steps (operands of every step in registers)");
    constexpr bool HALF = sizeof(TS) == 2;
    constexpr bool AM = HALF;   // fp16 storage: pair-major step order (below)
    const Dims d = p.d;
    const int nwt = p.nwt;
    const int total = p.E * nwt;
    const int per = (total + 7) / 8;
    const int xcd = blockIdx.x & 7;
    const int K = (int)(gridDim.x >> 3) * (DD_THREADS / 64);     // waves per XCD
    const int g_end = min(total, (xcd + 1) * per);
    const int g0 = __builtin_amdgcn_readfirstlane(
        xcd * per + (int)(blockIdx.x >> 3) * (DD_THREADS / 64) + (int)(threadIdx.x >> 6));
    if (g0 >= g_end) return;

    const int lane = threadIdx.x & 63;
    const int kh = d.kmax / 2;   // 8
    const size_t opstride = (size_t)d.nb * 64 * kh;
    const size_t inst_elems = (size_t)d.ntiles * TILE_ELEMS;
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    TS* sink = reinterpret_cast<TS*>(p.sink);
    const int lofs = lane * kh;

    // the pipelined loop needs every step of every instance this wave visits to be a plain
    // downdate (no reset, no new rows); the split-plane form also takes steps that add rows (it
    // writes them into the wave-tiles they touch, between the steps' MFMAs)
    bool fast = true, fast_rows = true;
    {
        const int e_lo = g0 / nwt, e_hi = (g_end - 1) / nwt;
        for (int e = e_lo; e <= e_hi; e++)
#pragma unroll
            for (int q = 0; q < NS; q++) {
                const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
                const bool rb = sload(r + RES_ROLLBACK), rs = sload(r + RES_RESET);
                fast_rows = fast_rows && !rb;
                fast = fast && !rb && !rs && sload(r + RES_NADD) == 0;
            }
    }

    // a wave-tile: instance, table entry (scalar registers)
    struct Item {
        int e, li, g;   // instance, table entry, flat index (g0 + k·K)
        WtEntry w;
    };
    typedef int i32x8 __attribute__((ext_vector_type(8)));
    static_assert(sizeof(WtEntry) == sizeof(i32x8), "one scalar dwordx8 per entry");
    auto load_entry = [&](int li, WtEntry& w) __attribute__((always_inline)) {
        const i32x8 v = sload(reinterpret_cast<const i32x8*>(p.wt + li));
#pragma unroll
        for (int i = 0; i < WT_N; i++) w.tile[i] = v[i];
        w.valid = v[WT_N];
        w.rows[0] = v[WT_N + 1];
        w.rows[1] = v[WT_N + 2];
        w.rc = v[WT_N + 3];
    };
    // the wave's k-th wave-tile follows from the (k−1)-th by adding K to the flat index
    auto first_item = [&](Item& t) __attribute__((always_inline)) {
        t.e = g0 / nwt;
        const int li = g0 - t.e * nwt;
        load_entry(li, t.w);
        t.li = li;
        t.g = g0;
    };
    auto next_item = [&](const Item& c, Item& t) __attribute__((always_inline)) {
        int li = c.li + K, e = c.e;
        while (li >= nwt) {
            li -= nwt;
            e++;
        }
        t.e = e;
        load_entry(e < p.E ? li : 0, t.w);
        t.li = li;
        t.g = c.g + K;
    };
    auto tile_ptr = [&](const Item& t, int i) __attribute__((always_inline)) {
        return (size_t)t.e * inst_elems + (size_t)t.w.tile[i] * TILE_ELEMS;
    };
    // every slot is stored, the invalid ones (outside the packed triangle) to the sink tile: no
    // branch around a store (a conditional store splits the wait-count tracking, and the join
    // then waits for every outstanding load, the next wave-tile's prefetch included)
    auto store_tiles = [&](const Item& t, const f32x16 (&acc)[WT_N], bool skip = false) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT_N; i++) {
            TS* tl = ((t.w.valid >> i) & 1) && !skip ? Pout + tile_ptr(t, i) : sink;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) tile_st(tl, lane, qq, acc[i]);
        }
    };
    auto op_row = [&](const Item& t, int side, int k) __attribute__((always_inline)) {
        return (t.w.rows[side] >> (16 * k)) & 0xffff;
    };
    // step q's operand rows (side 0: U, 1: V) from the contiguous slot buffers: scalar arithmetic
    // on a few kernel arguments, not 2·NS pointers (which the compiler reloaded from the kernel
    // arguments inside the loop, each load waited on before the next MFMA could issue)
    auto op_base = [&](int q, int side) __attribute__((always_inline)) {
        int sl = p.slot0 + q;
        if (sl >= p.nslots) sl -= p.nslots;
        return reinterpret_cast<const float*>(reinterpret_cast<const char*>(side || p.usym ? p.vbase : p.ubase) +
                                              (size_t)sl * (size_t)p.slot_bytes);
    };

    if constexpr (BF) {
        if (fast_rows) {
            // planes: BF16X6 hi, mid, lo bf16 (six products); F16X3 hi, lo fp16 of 2^σ·V (three)
            constexpr int NPL = F16 ? 2 : 3;
            typedef typename std::conditional<F16, f16x8r, bf16x8r>::type bf16x8;
            // operand ring depth (divides NS: a ring slot keeps its step index across wave-tiles).
            // F16: the deepest ring of at most F16_RDMAX step-sets, and the next wave-tile's tiles
            // issued RD − 1 steps before its start (late, below)
            constexpr int RD = F16 ? ring_depth(NS, F16_RDMAX) : (NS % 4 == 0 ? 4 : (NS % 3 == 0 ? 3 : 2));
            constexpr bool LATE = F16 && RD >= 3;
            // vmcnt retires in issue order, so every operand wait after the tile loads also waits for
            // them: issued at step TQ, the first such wait comes RD − 1 steps later, and so does
            // the next wave-tile's first use of them
            constexpr int TQ = NS - RD + 1;
            const size_t pstride = (size_t)d.nb * NPL * 64;   // 16-byte operands per instance
            // step q's planes: slot (slot0 + q) mod nslots
            auto pl_base = [&](int q) __attribute__((always_inline)) {
                int sl = p.slot0 + q;
                if (sl >= p.nslots) sl -= p.nslots;
                return reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(p.bbase) +
                                                       (size_t)sl * (size_t)p.bslot_bytes);
            };
            // raw tile words in flight (fp16 storage: converted when the wave-tile starts)
            using Raw = typename std::conditional<HALF, f16x4, f32x4>::type;
            Raw pref[WT_N][4];
            f32x16 acc[WT_N];
            bf16x8 R[RD][WT_R + WT_C][NPL];
            // step q of wave-tile t into ring set r: A row blocks, then B row blocks, three planes
            auto load_ops = [&](int r, const Item& t, int q) __attribute__((always_inline)) {
                const bf16x8* b = pl_base(q) + t.e * pstride + lane;
#pragma unroll
                for (int i = 0; i < WT_R + WT_C; i++) {
                    const bf16x8* rb = b + (size_t)(i < WT_R ? op_row(t, 0, i) : op_row(t, 1, i - WT_R)) * NPL * 64;
#pragma unroll
                    for (int pl = 0; pl < NPL; pl++) R[r][i][pl] = rb[pl * 64];
                }
            };
            auto load_tiles = [&](const Item& t) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < WT_N; i++) {
                    const Raw* tl = reinterpret_cast<const Raw*>(Pin + tile_ptr(t, i));
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) pref[i][qq] = __builtin_nontemporal_load(tl + lane + qq * 64);
                }
            };
            // the accumulators hold −P: fp32 storage −X; fp16 storage −2^−x·X (X = fp16(2^x·P), the
            // instance's exponent; power-of-two scalings, exact), so that both operands are the
            // unscaled V planes; the store scales back and rounds to fp16 once per group. F16X3: the
            // planes of step q carry 2^σ_q·V, so during step q the accumulators hold −2^(2σ_q)·P (σ
            // changes only at a step that adds rows: the accumulators are rescaled after it)
            // per instance of the wave-tiles (uniform, few registers): the landmarks the group's steps
            // add [u_lo, u_hi), σ of the first and last step, the steps after which σ changes
            auto rec_of = [&](int e, int q, int w) __attribute__((always_inline)) {
                return sload(p.steps[q].res + (size_t)e * RES_STRIDE + w);
            };
            // A step that resets the map (Robot.cpp:893-904) zeroes the block: only the landmarks
            // added after the instance's last reset of the group are nonzero at its end, so the
            // union is taken over those steps and every other wave-tile of the instance is stored
            // as zero (rz); σ changes before that reset do not matter.
            int st_e = -1, u_lo = 0, u_hi = 0, sg0 = 0, sgl = 0, zl = 0;
            unsigned smask = 0;
            bool rz = false;
            auto load_steps = [&](int e) __attribute__((always_inline)) {
                u_lo = 0x7fffffff;
                u_hi = 0;
                smask = 0;
                rz = false;
                zl = 0;   // landmarks past every step's RES_ZMAX: zero V rows, no new rows
                int prev = 0;
#pragma unroll
                for (int q = 0; q < NS; q++) {
                    zl = max(zl, rec_of(e, q, RES_ZMAX));
                    if (rec_of(e, q, RES_RESET)) {   // (its own new rows are wiped with the map)
                        u_lo = 0x7fffffff;
                        u_hi = 0;
                        smask = 0;
                        rz = true;
                        continue;
                    }
                    const int na = rec_of(e, q, RES_NADD), s0 = rec_of(e, q, RES_SAVED_IN);
                    if (na > 0) {
                        u_lo = min(u_lo, s0);
                        u_hi = max(u_hi, s0 + na);
                    }
                    const int sg = F16 ? rec_of(e, q, RES_PSIG) : 0;
                    if (q == 0) sg0 = sg;
                    else if (sg != prev) smask |= 1u << (q - 1);
                    if (sg == PLANE_SIGMA_EXACT) smask |= 1u << NS;   // (the whole group exact)
                    prev = sg;
                }
                sgl = prev;
                st_e = e;
            };
            auto in_exp = [&](const Item& t) __attribute__((always_inline)) {
                int ex = 2 * sg0;
                if constexpr (HALF) ex -= sload(p.pexp + t.e);
                return ex;
            };
            auto touched = [&](const Item& t) __attribute__((always_inline)) {
                if (t.e != st_e) load_steps(t.e);
                const int ra = (t.w.rc & 0xffff) * WT_R * 16, ca = (t.w.rc >> 16) * WT_C * 16;   // landmarks
                return (u_lo < ra + WT_R * 16 && u_hi > ra) || (u_lo < ca + WT_C * 16 && u_hi > ca);
            };
            auto skip_of = [&](const Item& t) __attribute__((always_inline)) {
                const bool tc = touched(t);
                return tc || (!rz && smask != 0);
            };
            auto zero_of = [&](const Item& t) __attribute__((always_inline)) {
                const bool tc = touched(t);
                return rz && !tc;
            };
            // a wave-tile whose columns all lie past zl is unchanged by the group (its V-side rows
            // are zero in every step, and no step writes new rows there): not loaded, not stored
            // (a reset zeroes the block: no skipping then)
            auto dead = [&](const Item& t) __attribute__((always_inline)) {
                if (!p.zskip || t.e >= p.E) return false;
                if (t.e != st_e) load_steps(t.e);
                return !rz && (t.w.rc >> 16) * WT_C * 16 >= zl;
            };
            auto next_live = [&](const Item& c, Item& t) __attribute__((always_inline)) {
                next_item(c, t);
                while (t.g < g_end && dead(t)) {
                    const Item u = t;
                    next_item(u, t);
                }
            };
            Item cur, nxt, nxt2;
            bool any_skip = false;
            first_item(cur);
            while (cur.g < g_end && dead(cur)) {
                const Item u = cur;
                next_item(u, cur);
            }
            if (cur.g >= g_end) return;   // (no live wave-tile: nothing to store, no second pass)
            next_live(cur, nxt);
            load_tiles(cur);
            // (the first tiles ahead of every operand load, as in the loop: the wait count at the loop
            // head then covers the tiles without draining the previous wave-tile's stores)
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < RD - 1; q++) load_ops(q, cur, q);
            while (true) {
                const bool more = nxt.g < g_end;
                next_live(nxt, nxt2);
                const Item ldi = more ? nxt : cur;   // the last wave-tile re-reads its own rows
                // a wave-tile holding a landmark some step of the group added, or of an instance whose
                // σ changes inside the group, is computed here but stored to the sink: the second pass
                // (below) runs it through the general loop
                const bool skip = skip_of(cur);
                const bool zero = zero_of(cur);   // (reset instance, untouched: stored as zero)
                any_skip |= skip;
                const int iex = in_exp(cur);
                const float isc = -ldexpf(1.0f, iex);
#pragma unroll
                for (int i = 0; i < WT_N; i++)
#pragma unroll
                    for (int qq = 0; qq < 4; qq++)
#pragma unroll
                        for (int j = 0; j < 4; j++) acc[i][4 * qq + j] = (float)pref[i][qq][j] * isc;
                if (!LATE && more) load_tiles(nxt);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int q = 0; q < NS; q++) {
                    if (LATE && q == TQ && more) load_tiles(nxt);
                    // ring set of step q + RD − 1 (this wave-tile's, else the next one's)
                    const int ql = q + RD - 1;
                    if (ql < NS) load_ops(ql % RD, cur, ql);
                    else load_ops(ql % RD, ldi, ql - NS);
                    const int r = q % RD;
                    if constexpr (F16) {
                        // (lo, hi), (hi, lo), (hi, hi): 12 MFMAs beside the 8 plane loads
#pragma unroll
                        for (int pp = 0; pp < 3; pp++) {
                            const int pa = pp == 0 ? 1 : 0, pb = pp == 1 ? 1 : 0;
#pragma unroll
                            for (int rr = 0; rr < WT_R; rr++)
#pragma unroll
                                for (int c = 0; c < WT_C; c++)
                                    acc[rr * WT_C + c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                                        R[r][rr][pa], R[r][WT_R + c][pb], acc[rr * WT_C + c], 0, 0, 0);
                        }
#pragma unroll
                        for (int i = 0; i < 8; i++) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);   // MFMA
                            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
                        }
                        __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
                    } else {
                        // part products smallest first: (mid, mid), (hi, lo), (lo, hi), (hi, mid),
                        // (mid, hi), (hi, hi)
#pragma unroll
                        for (int pp = 0; pp < 6; pp++) {
                            const int pa = (0x102010 >> (4 * (5 - pp))) & 0xf;
                            const int pb = (0x120100 >> (4 * (5 - pp))) & 0xf;
#pragma unroll
                            for (int rr = 0; rr < WT_R; rr++)
#pragma unroll
                                for (int c = 0; c < WT_C; c++)
                                    acc[rr * WT_C + c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                        R[r][rr][pa], R[r][WT_R + c][pb], acc[rr * WT_C + c], 0, 0, 0);
                        }
#pragma unroll
                        for (int i = 0; i < 12; i++) {
                            __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMA
                            __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
                        }
                    }
                    __builtin_amdgcn_sched_barrier(0);
                }
                // back from the last step's domain (−1, −2^x, −2^(x − 2σ): an exact power of two, no
                // division), as whole-vector products (packed multiplies); a zeroed wave-tile (zero is
                // uniform) takes no multiply at all
                const float osc = -ldexpf(1.0f, -iex - (F16 ? 2 * (sgl - sg0) : 0));
                if (zero) {
#pragma unroll
                    for (int i = 0; i < WT_N; i++) acc[i] = f32x16{};
                } else {
#pragma unroll
                    for (int i = 0; i < WT_N; i++) acc[i] = acc[i] * osc;
                }
                store_tiles(cur, acc, skip);
                if (!more) break;
                cur = nxt;
                nxt = nxt2;
            }
            // second pass: the skipped wave-tiles through the general loop (their input tiles are
            // as read: the first pass stored them to the sink). Exact arithmetic on the fp32 operand
            // rows there, the split arithmetic elsewhere: both within the fp32 bar (slam_ekf.h)
            if (any_skip) {
                Item t;
                first_item(t);
                for (int gg = g0; gg < g_end; gg += K) {
                    if (gg != g0) {
                        Item nn;
                        next_item(t, nn);
                        t = nn;
                    }
                    if (!dead(t) && skip_of(t)) wt_general<TS, NS>(p, t.e, t.w, lane);
                }
            }
            return;
        }
    } else if (fast) {
        // raw tile words in flight (fp16 storage: converted when the wave-tile starts)
        using Raw = typename std::conditional<HALF, f16x4, f32x4>::type;
        Raw pref[WT_N][4];
        f32x4 opA[NS][WT_R][2], opB[NS][WT_C][2];
        f32x16 acc[WT_N];
        // half h (k-steps 4h..4h+3) of step q's operand rows of wave-tile t, into slot q
        auto load_half = [&](int slot, const Item& t, int q, int h) __attribute__((always_inline)) {
            const float* U = op_base(q, 0) + t.e * opstride + lofs + 4 * h;
            const float* V = op_base(q, 1) + t.e * opstride + lofs + 4 * h;
            const float us = us_of<TS>(p, t.e);
#pragma unroll
            for (int r = 0; r < WT_R; r++)
                opA[slot][r][h] = *reinterpret_cast<const f32x4*>(U + (size_t)op_row(t, 0, r) * 64 * kh) * us;
#pragma unroll
            for (int c = 0; c < WT_C; c++)
                opB[slot][c][h] = *reinterpret_cast<const f32x4*>(V + (size_t)op_row(t, 1, c) * 64 * kh);
        };
        auto load_tiles = [&](const Item& t) __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < WT_N; i++) {
                const Raw* tl = reinterpret_cast<const Raw*>(Pin + tile_ptr(t, i));
#pragma unroll
                for (int qq = 0; qq < 4; qq++) pref[i][qq] = __builtin_nontemporal_load(tl + lane + qq * 64);
            }
        };
        // k-steps 4h..4h+3 of step q. Every k-step runs: past the step's matches the scan kernel
        // leaves (−0)·(+0) operand products, and x + (−0) == x for every x (zeros, NaN, inf too)
        auto mfma_half = [&](int q, int h) __attribute__((always_inline)) {
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int r = 0; r < WT_R; r++)
#pragma unroll
                    for (int c = 0; c < WT_C; c++)
                        acc[r * WT_C + c] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                            opA[q][r][h][s], opB[q][c][h][s], acc[r * WT_C + c], 0, 0, 0);
        };
        // one operand load after every group of four MFMAs (4 loads per half step)
        auto interleave = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int i = 0; i < 4; i++) {
                __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);   // MFMA
                __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
            }
        };
        Item cur, nxt, nxt2;
        first_item(cur);
        next_item(cur, nxt);
        load_tiles(cur);
#pragma unroll
        for (int q = 0; q < NS; q++) {
            load_half(q, cur, q, 0);
            load_half(q, cur, q, 1);
        }
        int g = g0;
        while (true) {
            const bool more = g + K < g_end;
            next_item(nxt, nxt2);   // read now, used by the next wave-tile
            // operand rows for the next wave-tile (the last one re-reads its own: no branch
            // splits the MFMA stream)
            const Item ldi = more ? nxt : cur;
#pragma unroll
            for (int i = 0; i < WT_N; i++)
#pragma unroll
                for (int qq = 0; qq < 4; qq++)
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[i][4 * qq + j] = (float)pref[i][qq][j];
            // the next wave-tile's tiles first: the waits of this wave-tile only cover loads issued
            // during the one before it, so these have the whole wave-tile to land
            if (more) load_tiles(nxt);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (AM) {
                // group-major steps (fp16 storage): the
                // per-step rounding of one group of accumulators runs on the VALU while the other
                // group's MFMAs run, so it leaves the MFMA stream. Per element the chain is
                // unchanged (k-ordered step q, then its rounding). Step q's operand registers are
                // refilled for the next wave-tile during step q+1's first group; the last step's
                // at the end. (Measured: one accumulator's 8 k-steps back to back, rounding the
                // previous accumulator beside them, ran 0.84 ms vs 0.79 for the step-major form.)
                // Pair-major form: group gi = accumulators (gi, 0) and (gi, 1) of the 2 × 2
                // wave-tile, their k-steps alternating (a dependent MFMA two issues later); the
                // previous group's 32 elements are rounded 2 per MFMA gap. The last step rounds
                // group 0 in the first half of group 1 and stores its tiles in the second half.
                auto mfma_grp = [&](int q, int gi, int pg, bool ld, int lq, bool last) __attribute__((always_inline)) {
#pragma unroll
                    for (int m = 0; m < 16; m++) {
                        const int s = m >> 1, c = m & 1, i = gi * WT_C + c;
                        acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(opA[q][gi][s >> 2][s & 3],
                                                                       opB[q][c][s >> 2][s & 3], acc[i], 0, 0, 0);
                        __builtin_amdgcn_sched_barrier(0);
                        if (pg >= 0 && !last) {
                            const int a = pg * WT_C + (m >> 3), k = 2 * (m & 7);
                            acc[a][k] = round_step<TS>(acc[a][k]);
                            acc[a][k + 1] = round_step<TS>(acc[a][k + 1]);
                        }
                        if (last) {
                            if (m < 8) {
                                const int a = pg * WT_C + (m >> 2), k = 4 * (m & 3);
#pragma unroll
                                for (int u = 0; u < 4; u++) acc[a][k + u] = round_step<TS>(acc[a][k + u]);
                            } else {
                                const int a = pg * WT_C + ((m - 8) >> 2), qq = (m - 8) & 3;
                                tile_st(((cur.w.valid >> a) & 1) ? Pout + tile_ptr(cur, a) : sink, lane, qq, acc[a]);
                            }
                        }
                        if (ld && (m & 1)) {
                            // load m/2 of slot lq: half, operand row (A rows, then B rows)
                            const int l = m >> 1, h = l >> 2, o = l & 3;
                            const bool isA = o < WT_R;
                            const float* base = op_base(lq, isA ? 0 : 1) + ldi.e * opstride + lofs + 4 * h;
                            const f32x4 v = *reinterpret_cast<const f32x4*>(
                                base + (size_t)op_row(ldi, isA ? 0 : 1, isA ? o : o - WT_R) * 64 * kh);
                            if (isA) opA[lq][o][h] = v * us_of<TS>(p, ldi.e);
                            else opB[lq][o - WT_R][h] = v;
                        }
                        __builtin_amdgcn_sched_barrier(0);
                    }
                };
                static_assert(WT_R == 2 && WT_C == 2, "pair-major form: two groups of two accumulators");
#pragma unroll
                for (int q = 0; q < NS; q++) {
                    mfma_grp(q, 0, q > 0 ? 1 : -1, q > 0, q > 0 ? q - 1 : 0, false);
                    mfma_grp(q, 1, 0, false, 0, q == NS - 1);
                }
#pragma unroll
                for (int a = 2; a < 4; a++)
#pragma unroll
                    for (int k = 0; k < 16; k++) acc[a][k] = round_step<TS>(acc[a][k]);
                load_half(NS - 1, ldi, NS - 1, 0);
                load_half(NS - 1, ldi, NS - 1, 1);
#pragma unroll
                for (int a = 2; a < 4; a++) {
                    TS* tl = ((cur.w.valid >> a) & 1) ? Pout + tile_ptr(cur, a) : sink;
#pragma unroll
                    for (int qq = 0; qq < 4; qq++) tile_st(tl, lane, qq, acc[a]);
                }
                if (!more) break;
                g += K;
                cur = nxt;
                nxt = nxt2;
                continue;
            }
#pragma unroll
            for (int q = 0; q < NS; q++) {
                // first half of step q, beside the second half of step q−1's rows for the next
                // wave-tile (their registers were last read by step q−1)
                mfma_half(q, 0);
                if (q > 0) {
                    load_half(q - 1, ldi, q - 1, 1);
                    interleave();
                }
                __builtin_amdgcn_sched_barrier(0);
                // second half, beside the first half of step q's rows for the next wave-tile
                mfma_half(q, 1);
#pragma unroll
                for (int i = 0; i < WT_N; i++) round_acc<TS>(acc[i]);
                load_half(q, ldi, q, 0);
                interleave();
                __builtin_amdgcn_sched_barrier(0);
            }
            load_half(NS - 1, ldi, NS - 1, 1);
            store_tiles(cur, acc);
            if (!more) break;
            g += K;
            cur = nxt;
            nxt = nxt2;
        }
        return;
    }

    // general loop: per wave-tile, every step in order with its operands loaded in place, then
    // the step's reset or rows (wt_general)
    Item t;
    first_item(t);
    for (int g = g0; g < g_end; g += K) {
        if (g != g0) {
            Item n;
            next_item(t, n);
            t = n;
        }
        wt_general<TS, NS>(p, t.e, t.w, lane);
    }
}

// Split-fp16 flush, quad form (EKF_ARITH_F16X3, EKF_OPT_FLUSH_FORM = 44; groups of >= 6 steps).
// The 2 × 2 wave form streams each wave's 8 KB of operand planes per step through L1/L2 into
// registers beside its 12 MFMAs, and that stream, not HBM, paces it. Here a
// workgroup's four MFMA waves take the four wave-tiles of a 2 × 2 group (p.wtq: four entries per
// group in panel order, entry 2a + b the wave-tile (2R + a, 2C + b); positions wholly below the
// diagonal or past the block are entries with no stored tile) and share the group's operand row
// blocks: its 4 A blocks (tile rows) and 4 B blocks (tile columns), both planes, 16 KB per step —
// half of what the four waves read alone. Loader waves (EKF_Q_LOADERS, no MFMA work) move them by
// LDS-DMA (global_load_lds_dwordx4, 1 KB per wave-instruction, no register staging) into a ring
// of D step slots, D − 1 steps ahead of the MFMA waves; one barrier per step: before it each loader
// waits (its own vmcnt, counted) for the step after the current one to land, and each MFMA wave
// for its own LDS reads of the current step; after it the MFMA waves read the next step's planes
// into the second of two register sets while the current step's 12 MFMAs run, and the loaders
// refill the slot just consumed. The MFMA waves' vector memory queue then holds only their own tile
// loads (issued EKF_Q_TQ steps into a group for the next one) and stores, so an operand wait never
// waits for a tile. Per accumulator the chain is the 2 × 2 form's (the same three products per
// step, in the same order, on the same planes): bit-identical. As there: −P in the accumulators
// (fp16 storage scaled out of its exponent), the second pass through wt_general for wave-tiles
// whose steps add rows or whose σ changes, reset instances stored as zero, and a group whose
// columns all lie past every step's RES_ZMAX skipped whole (dead).
#ifndef EKF_Q_DEPTH
#define EKF_Q_DEPTH 8      // quad flush: operand ring slots (16 KB each) = steps in flight
#endif
#ifndef EKF_Q_LOADERS
#define EKF_Q_LOADERS 2    // quad flush: LDS-DMA loader waves beside the four MFMA waves
#endif
#ifndef EKF_Q_TQ
#define EKF_Q_TQ 1         // quad flush: the step of a group at which the next group's tiles are issued
#endif
constexpr int Q_WAVES = 4 + EKF_Q_LOADERS;
constexpr int Q_SLOT = 16 * 1024;   // one step: 8 row blocks × 2 planes × 64 lanes × 16 B
template <typename TS, int NS>
__global__ __launch_bounds__(64 * Q_WAVES, 1) void flush_f16q_kernel(DowndateParams p)
{
    constexpr int D = EKF_Q_DEPTH < NS ? EKF_Q_DEPTH : NS;
    constexpr int PPL = 16 / EKF_Q_LOADERS;   // plane pieces per loader wave and step
    // (vmcnt holds at most 63 outstanding instructions)
    static_assert(16 % EKF_Q_LOADERS == 0 && D >= 3 && PPL * (D - 2) <= 63, "quad flush: ring");
    static_assert(NS >= 6 && NS % 2 == 0 && EKF_Q_TQ < NS, "quad flush: step count");
    constexpr bool HALF = sizeof(TS) == 2;
    constexpr int NPL = 2;
    typedef f16x8r f16x8;
    // the only LDS object: a second one beside a DMA target can make the compiler drain vmcnt
    // before LDS reads (cdna_hip_programming.md §5)
    __shared__ __attribute__((aligned(1024))) char ring[D * Q_SLOT];

    const Dims d = p.d;
    const int ngr = p.nwtq >> 2;   // groups per instance
    const int total = p.E * ngr;
    const int per = (total + 7) / 8;   // groups per XCD (a contiguous range)
    const int xcd = blockIdx.x & 7;
    const int K = (int)(gridDim.x >> 3);
    const int g_end = min(total, (xcd + 1) * per);
    const int gs = xcd * per + (int)(blockIdx.x >> 3);
    if (gs >= g_end) return;   // (the whole workgroup)
    const int wv = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    const size_t inst_elems = (size_t)d.ntiles * TILE_ELEMS;
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    TS* sink = reinterpret_cast<TS*>(p.sink);

    // the plain loop needs every step of the workgroup's instances to be a downdate without a
    // rollback (the 2 × 2 form's fast_rows), decided alike by every wave
    bool fast_rows = true;
    {
        const int e_lo = gs / ngr, e_hi = (g_end - 1) / ngr;
        for (int e = e_lo; e <= e_hi; e++)
#pragma unroll
            for (int q = 0; q < NS; q++)
                fast_rows = fast_rows && !sload(p.steps[q].res + (size_t)e * RES_STRIDE + RES_ROLLBACK);
    }
    struct Grp {
        int e, gi, g;   // instance, group of the instance, flat index (gs + k·K)
    };
    auto first_grp = [&](Grp& t) __attribute__((always_inline)) {
        t.e = gs / ngr;
        t.gi = gs - t.e * ngr;
        t.g = gs;
    };
    auto next_grp = [&](const Grp& c, Grp& t) __attribute__((always_inline)) {
        int gi = c.gi + K, e = c.e;
        while (gi >= ngr) {
            gi -= ngr;
            e++;
        }
        t.e = e;
        t.gi = gi;
        t.g = c.g + K;
    };
    typedef int i32x8 __attribute__((ext_vector_type(8)));
    static_assert(sizeof(WtEntry) == sizeof(i32x8), "one scalar dwordx8 per entry");
    auto load_entry = [&](int li, WtEntry& w) __attribute__((always_inline)) {
        const i32x8 v = sload(reinterpret_cast<const i32x8*>(p.wtq + li));
#pragma unroll
        for (int i = 0; i < WT_N; i++) w.tile[i] = v[i];
        w.valid = v[WT_N];
        w.rows[0] = v[WT_N + 1];
        w.rows[1] = v[WT_N + 2];
        w.rc = v[WT_N + 3];
    };
    if (!fast_rows) {   // every wave-tile through the general loop (no LDS, no barriers)
        if (wv >= 4) return;
        Grp t;
        first_grp(t);
        for (int g = gs; g < g_end; g += K) {
            if (g != gs) {
                Grp n;
                next_grp(t, n);
                t = n;
            }
            WtEntry w;
            load_entry(4 * t.gi + wv, w);
            wt_general<TS, NS>(p, t.e, w, lane);
        }
        return;
    }

    // per instance (the 2 × 2 form's bookkeeping): added landmarks [u_lo, u_hi), σ of the first and
    // last step, σ changes (smask), a reset (rz), the landmarks past every step's RES_ZMAX (zl)
    auto rec_of = [&](int e, int q, int w) __attribute__((always_inline)) {
        return sload(p.steps[q].res + (size_t)e * RES_STRIDE + w);
    };
    int st_e = -1, u_lo = 0, u_hi = 0, sg0 = 0, sgl = 0, zl = 0;
    unsigned smask = 0;
    bool rz = false;
    auto load_steps = [&](int e) __attribute__((always_inline)) {
        u_lo = 0x7fffffff;
        u_hi = 0;
        smask = 0;
        rz = false;
        zl = 0;
        int prev = 0;
#pragma unroll
        for (int q = 0; q < NS; q++) {
            zl = max(zl, rec_of(e, q, RES_ZMAX));
            if (rec_of(e, q, RES_RESET)) {
                u_lo = 0x7fffffff;
                u_hi = 0;
                smask = 0;
                rz = true;
                continue;
            }
            const int na = rec_of(e, q, RES_NADD), s0 = rec_of(e, q, RES_SAVED_IN);
            if (na > 0) {
                u_lo = min(u_lo, s0);
                u_hi = max(u_hi, s0 + na);
            }
            const int sg = rec_of(e, q, RES_PSIG);
            if (q == 0) sg0 = sg;
            else if (sg != prev) smask |= 1u << (q - 1);
            if (sg == PLANE_SIGMA_EXACT) smask |= 1u << NS;
            prev = sg;
        }
        sgl = prev;
        st_e = e;
    };
    // a group whose columns all lie past zl (its first wave-tile column, entry 0's): unchanged by
    // the group's steps, skipped by every wave alike
    auto dead = [&](const Grp& t) __attribute__((always_inline)) {
        if (!p.zskip || t.e >= p.E) return false;
        if (t.e != st_e) load_steps(t.e);
        const int rc = sload(&p.wtq[4 * t.gi].rc);
        return !rz && (rc >> 16) * WT_C * 16 >= zl;
    };
    auto next_live = [&](const Grp& c, Grp& t) __attribute__((always_inline)) {
        next_grp(c, t);
        while (t.g < g_end && dead(t)) {
            const Grp u = t;
            next_grp(u, t);
        }
    };
    auto barrier = [&]() __attribute__((always_inline)) {
        asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
    };
    Grp cur, nxt, nxt2;
    first_grp(cur);
    while (cur.g < g_end && dead(cur)) {
        const Grp u = cur;
        next_grp(u, cur);
    }
    if (cur.g >= g_end) return;   // (uniform: no live group)
    next_live(cur, nxt);

    if (wv >= 4) {
        // loader wave: plane pieces LW·PPL .. LW·PPL + PPL − 1 of every step; piece 2·blk + pl is
        // plane pl of row block blk: blocks 0-3 the group's tile rows (entry 0's A rows, then entry
        // 3's), 4-7 its tile columns (entry 0's B rows, then entry 3's)
        const size_t pstride = (size_t)d.nb * NPL * 64;
        auto pl_base = [&](int q) __attribute__((always_inline)) {
            int sl = p.slot0 + q;
            if (sl >= p.nslots) sl -= p.nslots;
            return reinterpret_cast<const f16x8*>(reinterpret_cast<const char*>(p.bbase) +
                                                  (size_t)sl * (size_t)p.bslot_bytes);
        };
        auto run = [&](auto lwc) __attribute__((always_inline)) {
            constexpr int LW = decltype(lwc)::value;
            struct Rows {
                int w[4];   // entry 0 rows[0], entry 3 rows[0], entry 0 rows[1], entry 3 rows[1]
            };
            auto rows_of = [&](const Grp& t, Rows& r) __attribute__((always_inline)) {
                const int li = 4 * t.gi;
                r.w[0] = sload(&p.wtq[li].rows[0]);
                r.w[1] = sload(&p.wtq[li + 3].rows[0]);
                r.w[2] = sload(&p.wtq[li].rows[1]);
                r.w[3] = sload(&p.wtq[li + 3].rows[1]);
            };
            // step q of group t into ring slot sl
            auto issue = [&](int sl, const Grp& t, const Rows& r, int q) __attribute__((always_inline)) {
                const f16x8* b = pl_base(q) + (size_t)t.e * pstride + lane;
#pragma unroll
                for (int i = 0; i < PPL; i++) {
                    const int pc = LW * PPL + i, blk = pc >> 1, pl = pc & 1;
                    const int row = (r.w[blk >> 1] >> (16 * (blk & 1))) & 0xffff;
                    __builtin_amdgcn_global_load_lds(
                        (const void*)(b + ((size_t)row * NPL + pl) * 64),
                        (__attribute__((address_space(3))) void*)(ring + sl * Q_SLOT + pc * 1024), 16, 0, 0);
                }
            };
            Rows rc, rn;
            rows_of(cur, rc);
#pragma unroll
            for (int s = 0; s < D; s++) issue(s, cur, rc, s);
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL * (D - 1)) : "memory");
            barrier();
            int sb = 0;   // ring slot of the group's step 0
            while (true) {
                const bool more = nxt.g < g_end;
                next_live(nxt, nxt2);
                const Grp ldi = more ? nxt : cur;   // (the last group re-reads its own rows)
                rows_of(ldi, rn);
#pragma unroll
                for (int q = 0; q < NS; q++) {
                    // step s + 1 landed (the pieces of the D − 2 steps after it may be in flight)
                    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(PPL * (D - 2)) : "memory");
                    barrier();
                    // step s + D into the slot of step s, which every MFMA wave has read
                    const int sl = (sb + q) % D;
                    if (q + D < NS) issue(sl, cur, rc, q + D);
                    else issue(sl, ldi, rn, q + D - NS);
                }
                if (!more) break;
                sb = (sb + NS) % D;
                cur = nxt;
                nxt = nxt2;
                rc = rn;
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        };
        if (wv == 4) run(std::integral_constant<int, 0>{});
#if EKF_Q_LOADERS >= 2
        else if (wv == 5) run(std::integral_constant<int, 1>{});
#endif
#if EKF_Q_LOADERS >= 4
        else if (wv == 6) run(std::integral_constant<int, 2>{});
        else if (wv == 7) run(std::integral_constant<int, 3>{});
#endif
        return;
    }

    // MFMA wave (a, b) = (wv >> 1, wv & 1): wave-tile entry 4·gi + wv; its A blocks 2a, 2a + 1
    // and B blocks 2b, 2b + 1 of the group
    const int qa = wv >> 1, qb = wv & 1;
    auto tile_ptr = [&](int e, const WtEntry& w, int i) __attribute__((always_inline)) {
        return (size_t)e * inst_elems + (size_t)w.tile[i] * TILE_ELEMS;
    };
    using Raw = typename std::conditional<HALF, f16x4, f32x4>::type;
    Raw pref[WT_N][4];
    f32x16 acc[WT_N];
    f16x8 op[2][4][NPL];   // [register set][A 2a, A 2a + 1, B 2b, B 2b + 1][hi, lo]
    auto load_tiles = [&](int e, const WtEntry& w) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT_N; i++) {
            const Raw* tl = reinterpret_cast<const Raw*>(Pin + tile_ptr(e, w, i));
#pragma unroll
            for (int qq = 0; qq < 4; qq++) pref[i][qq] = __builtin_nontemporal_load(tl + lane + qq * 64);
        }
    };
    // every slot is stored, the invalid ones to the sink tile (no branch around a store)
    auto store_tiles = [&](int e, const WtEntry& w, bool skip) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT_N; i++) {
            TS* tl = ((w.valid >> i) & 1) && !skip ? Pout + tile_ptr(e, w, i) : sink;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) tile_st(tl, lane, qq, acc[i]);
        }
    };
    const char* rbase = ring + lane * 16;
    const int aoff = (2 * (2 * qa)) * 1024, boff = (2 * (4 + 2 * qb)) * 1024;
    auto read_step = [&](int set, int sl) __attribute__((always_inline)) {
        const char* s = rbase + sl * Q_SLOT;
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int pl = 0; pl < NPL; pl++)
                op[set][i][pl] = *reinterpret_cast<const f16x8*>(s + (i < 2 ? aoff : boff) + (2 * (i & 1) + pl) * 1024);
    };
    auto touched = [&](int e, const WtEntry& w) __attribute__((always_inline)) {
        if (e != st_e) load_steps(e);
        const int ra = (w.rc & 0xffff) * WT_R * 16, ca = (w.rc >> 16) * WT_C * 16;
        return (u_lo < ra + WT_R * 16 && u_hi > ra) || (u_lo < ca + WT_C * 16 && u_hi > ca);
    };
    auto skip_of = [&](int e, const WtEntry& w) __attribute__((always_inline)) {
        return touched(e, w) || (!rz && smask != 0);
    };
    // the group's accumulators from its prefetched tiles, −2^iex·P (iex: 2σ of its first step, less
    // the fp16 storage exponent)
    auto in_exp = [&](int e) __attribute__((always_inline)) {
        if (e != st_e) load_steps(e);
        int ex = 2 * sg0;
        if constexpr (HALF) ex -= sload(p.pexp + e);
        return ex;
    };
    auto init_acc = [&](int e) __attribute__((always_inline)) {
        const float isc = -ldexpf(1.0f, in_exp(e));
#pragma unroll
        for (int i = 0; i < WT_N; i++)
#pragma unroll
            for (int qq = 0; qq < 4; qq++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][4 * qq + j] = (float)pref[i][qq][j] * isc;
    };
    WtEntry wc, wn;
    load_entry(4 * cur.gi + wv, wc);
    load_tiles(cur.e, wc);
    init_acc(cur.e);
    bool any_skip = false;
    barrier();
    read_step(0, 0);
    int sb = 0;
    while (true) {
        const bool more = nxt.g < g_end;
        next_live(nxt, nxt2);
        if (more) load_entry(4 * nxt.gi + wv, wn);
        const bool skip = skip_of(cur.e, wc);
        const bool zero = rz && !touched(cur.e, wc);
        any_skip |= skip;
        const int iex = in_exp(cur.e);
        const int sgl_c = sgl, sg0_c = sg0;
#pragma unroll
        for (int q = 0; q < NS; q++) {
            if (q == EKF_Q_TQ && more) load_tiles(nxt.e, wn);
            barrier();
            // the next step's planes (this group's, else the next group's first) into the other set
            read_step((q + 1) & 1, (sb + q + 1) % D);
            // (the reads ahead of the MFMAs: left to itself the scheduler sinks them below, and the
            // next step then waits for them)
            __builtin_amdgcn_sched_barrier(0);
            const int st = q & 1;
            // (lo, hi), (hi, lo), (hi, hi) per accumulator, as the 2 × 2 form
#pragma unroll
            for (int pp = 0; pp < 3; pp++) {
                const int pa = pp == 0 ? 1 : 0, pb = pp == 1 ? 1 : 0;
#pragma unroll
                for (int rr = 0; rr < WT_R; rr++)
#pragma unroll
                    for (int c = 0; c < WT_C; c++)
                        acc[rr * WT_C + c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                            op[st][rr][pa], op[st][2 + c][pb], acc[rr * WT_C + c], 0, 0, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        const float osc = -ldexpf(1.0f, -iex - 2 * (sgl_c - sg0_c));
        if (zero) {
#pragma unroll
            for (int i = 0; i < WT_N; i++) acc[i] = f32x16{};
        } else {
#pragma unroll
            for (int i = 0; i < WT_N; i++) acc[i] = acc[i] * osc;
        }
        store_tiles(cur.e, wc, skip);
        if (!more) break;
        sb = (sb + NS) % D;
        cur = nxt;
        nxt = nxt2;
        wc = wn;
        // (here, behind the stores on every path to it: the wait for the tiles then counts the
        // stores instead of draining them, as a merge with the first group's path would)
        init_acc(cur.e);
    }
    // second pass: the skipped wave-tiles through the general loop (their input tiles as read: the
    // first pass stored them to the sink)
    if (any_skip) {
        Grp t;
        first_grp(t);
        for (int g = gs; g < g_end; g += K) {
            if (g != gs) {
                Grp n;
                next_grp(t, n);
                t = n;
            }
            if (dead(t)) continue;
            WtEntry w;
            load_entry(4 * t.gi + wv, w);
            if (skip_of(t.e, w)) wt_general<TS, NS>(p, t.e, w, lane);
        }
    }
}

// Split-bf16 flush on wave-tiles of 2 × 4 tiles (EKF_ARITH_BF16X6; the default form for its groups).
// The 2 × 2 form of flush_f32_wave_kernel<TS, NS, true> streams 12 KB of operand planes per step
// through a CU's vector memory path per wave (3 KB per tile and step: 62 B per clock for the four
// waves at the MFMA rate) beside its tile stream, and every operand wait of a wave also waits for
// its older tile loads (one in-order vmcnt). Measured at N = 4096, E = 8, T = 12 (timing builds):
// MFMA alone 0.36 ms, + operand planes 0.46, + tiles 0.41, both 0.63. A 2 × 4 wave-tile needs 18 KB
// per step for twice the MFMAs (2.25 KB per tile and step) and amortises each wave-tile's
// boundary and tile-stream waits over twice the MFMA time. Registers: 8 accumulators (128), the
// next wave-tile's tiles (128 fp32 / 64 fp16), a ring of 2 operand step-sets (144). Otherwise the
// 2 × 2 form's scheme: one 4-wave workgroup per CU, barrier-free waves, XCD-ranged K-strided walk
// of a panel-ordered table (p.wt24: 8 wave-tile columns per panel), tile prefetch one wave-tile
// ahead, operand ring one step ahead across wave-tile boundaries, −P in the accumulators (fp16:
// scaled out of the storage exponent), invalid slots stored to the sink. Groups in which some
// instance of the wave resets or adds rows run wt_general on the two 2 × 2 halves.
// F16 (EKF_ARITH_F16X3, EKF_OPT_FLUSH_FORM = 24): two fp16 planes of 2^σ·V, three products; the
// 2 × 2 form then streams 8 KB of planes per wave and step for 12 MFMAs, which at the four waves'
// MFMA rate is more than a CU's 64 B per clock: 2 × 4 streams 12 KB for 24. Groups whose σ
// changes run the general halves too.
constexpr int W4_R = 2, W4_C = 4, W4_N = W4_R * W4_C;
template <typename TS, int NS, bool F16 = false>
__global__ __launch_bounds__(DD_THREADS, 1) void flush_bf24_kernel(DowndateParams p)
{
    static_assert(NS >= 2 && NS % 2 == 0 && NS <= PMAX, "even step count");
    constexpr bool HALF = sizeof(TS) == 2;
    constexpr int NPL = F16 ? 2 : 3;
    constexpr int RD = (F16 && NS % 4 == 0) ? 4 : 2;   // operand ring depth (divides NS)
    typedef typename std::conditional<F16, f16x8r, bf16x8r>::type bf16x8;
    using Raw = typename std::conditional<HALF, f16x4, f32x4>::type;
    const Dims d = p.d;
    const int nwt = p.nwt24;
    const int total = p.E * nwt;
    const int per = (total + 7) / 8;
    const int xcd = blockIdx.x & 7;
    const int K = (int)(gridDim.x >> 3) * (DD_THREADS / 64);     // waves per XCD
    const int g_end = min(total, (xcd + 1) * per);
    const int g0 = __builtin_amdgcn_readfirstlane(
        xcd * per + (int)(blockIdx.x >> 3) * (DD_THREADS / 64) + (int)(threadIdx.x >> 6));
    if (g0 >= g_end) return;
    const int lane = threadIdx.x & 63;
    const int nb = d.nb;
    const size_t inst_elems = (size_t)d.ntiles * TILE_ELEMS;
    const TS* Pin = reinterpret_cast<const TS*>(p.Pin);
    TS* Pout = reinterpret_cast<TS*>(p.Pout);
    TS* sink = reinterpret_cast<TS*>(p.sink);

    bool fast = true;
    {
        const int e_lo = g0 / nwt, e_hi = (g_end - 1) / nwt;
        for (int e = e_lo; e <= e_hi; e++)
#pragma unroll
            for (int q = 0; q < NS; q++) {
                const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
                fast = fast && !sload(r + RES_RESET) && sload(r + RES_NADD) == 0 && !sload(r + RES_ROLLBACK);
                if (F16) fast = fast && sload(r + RES_PSIG) == sload(p.steps[0].res + (size_t)e * RES_STRIDE + RES_PSIG) &&
                                sload(r + RES_PSIG) != PLANE_SIGMA_EXACT;
            }
    }
    struct Item {
        int e, li, wr, wc;
    };
    auto load_item = [&](int e, int li, Item& t) __attribute__((always_inline)) {
        t.e = e;
        t.li = li;
        const int v = sload(p.wt24 + (e < p.E ? li : 0));
        t.wr = v & 0xffff;
        t.wc = v >> 16;
    };
    auto next_item = [&](const Item& c, Item& t) __attribute__((always_inline)) {
        int li = c.li + K, e = c.e;
        while (li >= nwt) {
            li -= nwt;
            e++;
        }
        load_item(e, li, t);
    };
    // slot (r, c): tile (2wr + r, 4wc + c) if stored, else a stored tile of the wave-tile
    auto slot_tile = [&](const Item& t, int i, bool& valid) __attribute__((always_inline)) {
        const int bi = W4_R * t.wr + i / W4_C, bj = W4_C * t.wc + i % W4_C;
        valid = bi < nb && bj < nb && bi <= bj;
        return valid ? tile_index(bi, bj, nb) : tile_index(W4_R * t.wr, min(W4_C * t.wc + W4_C - 1, nb - 1), nb);
    };
    auto op_rowA = [&](const Item& t, int r) __attribute__((always_inline)) { return min(W4_R * t.wr + r, nb - 1); };
    auto op_rowB = [&](const Item& t, int c) __attribute__((always_inline)) { return min(W4_C * t.wc + c, nb - 1); };

    if (!fast) {
        Item t;
        load_item(g0 / nwt, g0 - (g0 / nwt) * nwt, t);
        for (int g = g0; g < g_end; g += K) {
            if (g != g0) {
                Item n;
                next_item(t, n);
                t = n;
            }
#pragma unroll 1
            for (int h = 0; h < 2; h++) {
                WtEntry w;
                w.valid = 0;
#pragma unroll
                for (int i = 0; i < WT_N; i++) {
                    bool v;
                    w.tile[i] = (int)slot_tile(t, (i / WT_C) * W4_C + 2 * h + i % WT_C, v);
                    w.valid |= (v ? 1 : 0) << i;
                }
                w.rows[0] = op_rowA(t, 0) | (op_rowA(t, 1) << 16);
                w.rows[1] = op_rowB(t, 2 * h) | (op_rowB(t, 2 * h + 1) << 16);
                w.rc = t.wr | ((2 * t.wc + h) << 16);
                wt_general<TS, NS>(p, t.e, w, lane);
            }
        }
        return;
    }

    const size_t pstride = (size_t)nb * NPL * 64;   // 16-byte operands per instance
    auto pl_base = [&](int q) __attribute__((always_inline)) {
        int sl = p.slot0 + q;
        if (sl >= p.nslots) sl -= p.nslots;
        return reinterpret_cast<const bf16x8*>(reinterpret_cast<const char*>(p.bbase) + (size_t)sl * (size_t)p.bslot_bytes);
    };
    Raw pref[W4_N][4];
    f32x16 acc[W4_N];
    bf16x8 R[RD][W4_R + W4_C][NPL];
    auto load_ops = [&](int r, const Item& t, int q) __attribute__((always_inline)) {
        const bf16x8* b = pl_base(q) + t.e * pstride + lane;
#pragma unroll
        for (int i = 0; i < W4_R + W4_C; i++) {
            const bf16x8* rb = b + (size_t)(i < W4_R ? op_rowA(t, i) : op_rowB(t, i - W4_R)) * NPL * 64;
#pragma unroll
            for (int pl = 0; pl < NPL; pl++) R[r][i][pl] = rb[pl * 64];
        }
    };
    auto load_tiles = [&](const Item& t) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < W4_N; i++) {
            bool v;
            const Raw* tl = reinterpret_cast<const Raw*>(Pin + (size_t)t.e * inst_elems + (size_t)slot_tile(t, i, v) * TILE_ELEMS);
#pragma unroll
            for (int qq = 0; qq < 4; qq++) pref[i][qq] = __builtin_nontemporal_load(tl + lane + qq * 64);
        }
    };
    // −P in the accumulators, scaled: fp16 storage out of its exponent x, F16 by 2^(2σ) (the
    // group's one σ): −2^(2σ − x)
    auto in_scale = [&](const Item& t) __attribute__((always_inline)) {
        int ex = F16 ? 2 * sload(p.steps[0].res + (size_t)t.e * RES_STRIDE + RES_PSIG) : 0;
        if constexpr (HALF) ex -= sload(p.pexp + t.e);
        return -ldexpf(1.0f, ex);
    };
    Item cur, nxt, nxt2;
    load_item(g0 / nwt, g0 - (g0 / nwt) * nwt, cur);
    next_item(cur, nxt);
    load_tiles(cur);
#pragma unroll
    for (int q = 0; q < RD - 1; q++) load_ops(q, cur, q);
    int g = g0;
    while (true) {
        const bool more = g + K < g_end;
        next_item(nxt, nxt2);
        const Item ldi = more ? nxt : cur;   // the last wave-tile re-reads its own rows
        const float isc = in_scale(cur);
#pragma unroll
        for (int i = 0; i < W4_N; i++)
#pragma unroll
            for (int qq = 0; qq < 4; qq++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][4 * qq + j] = (float)pref[i][qq][j] * isc;
        if (more) load_tiles(nxt);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int q = 0; q < NS; q++) {
            const int ql = q + RD - 1;
            if (ql < NS) load_ops(ql % RD, cur, ql);
            else load_ops(ql % RD, ldi, ql - NS);
            const int r = q % RD;
            if constexpr (F16) {
                // (lo, hi), (hi, lo), (hi, hi): 24 MFMAs beside the 12 plane loads
#pragma unroll
                for (int pp = 0; pp < 3; pp++) {
                    const int pa = pp == 0 ? 1 : 0, pb = pp == 1 ? 1 : 0;
#pragma unroll
                    for (int rr = 0; rr < W4_R; rr++)
#pragma unroll
                        for (int c = 0; c < W4_C; c++)
                            acc[rr * W4_C + c] = __builtin_amdgcn_mfma_f32_32x32x16_f16(
                                R[r][rr][pa], R[r][W4_R + c][pb], acc[rr * W4_C + c], 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 12; i++) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);   // VMEM read
                }
            } else {
                // part products smallest first: (mid, mid), (hi, lo), (lo, hi), (hi, mid), (mid, hi), (hi, hi)
#pragma unroll
                for (int pp = 0; pp < 6; pp++) {
                    const int pa = (0x102010 >> (4 * (5 - pp))) & 0xf;
                    const int pb = (0x120100 >> (4 * (5 - pp))) & 0xf;
#pragma unroll
                    for (int rr = 0; rr < W4_R; rr++)
#pragma unroll
                        for (int c = 0; c < W4_C; c++)
                            acc[rr * W4_C + c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                                R[r][rr][pa], R[r][W4_R + c][pb], acc[rr * W4_C + c], 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 6; i++) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);   // MFMA
                    __builtin_amdgcn_sched_group_barrier(0x020, 3, 0);   // VMEM read
                }
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        const float osc = 1.0f / isc;   // (a power of two: exact)
#pragma unroll
        for (int i = 0; i < W4_N; i++) {
            bool v;
            const size_t ti = slot_tile(cur, i, v);
            TS* tl = v ? Pout + (size_t)cur.e * inst_elems + ti * TILE_ELEMS : sink;
#pragma unroll
            for (int k = 0; k < 16; k++) acc[i][k] = acc[i][k] * osc;
#pragma unroll
            for (int qq = 0; qq < 4; qq++) tile_st(tl, lane, qq, acc[i]);
        }
        if (!more) break;
        g += K;
        cur = nxt;
        nxt = nxt2;
    }
}

// f64 flush, barrier-free per-wave form for groups of NS <= F64_WAVE_MAXS steps (kmax == 16):
// the f32 wave kernel's scheme at fp64. One wave per SIMD walks wave-tiles of 1 × 2 tiles (eight
// 16×16 v_mfma_f64_16x16x4_f64 accumulators, 64 registers); while wave-tile k runs its NS × 32
// MFMAs, the tiles of wave-tile k+1 (issued first) and, step by step, its operand rows stream
// into registers. fp64 is HBM-bound at T = 4 (8 B per element: 0.54 ms of traffic vs 0.44 ms of
// MFMA per launch at E = 8, N = 4096), so the wave keeps a whole wave-tile of loads in flight.
// Every k-step runs (the scan pads the operands past the matches with −0·(+0)); per element the
// chain is that of downdate_f64_kernel and of the on-read replay: bit-identical results. Groups
// with a reset or augmented rows for the wave's instances take a plain per-wave-tile loop.
template <int NS>
__global__ __launch_bounds__(DD_THREADS, 1) void flush_f64_wave_kernel(DowndateParams p)
{
    static_assert(NS >= 1 && NS <= F64_WAVE_MAXS, "steps per launch");
    const Dims d = p.d;
    const int nwt = p.nwt64;
    const int total = p.E * nwt;
    const int per = (total + 7) / 8;
    const int xcd = blockIdx.x & 7;
    const int K = (int)(gridDim.x >> 3) * (DD_THREADS / 64);     // waves per XCD
    const int g_end = min(total, (xcd + 1) * per);
    const int g0 = __builtin_amdgcn_readfirstlane(
        xcd * per + (int)(blockIdx.x >> 3) * (DD_THREADS / 64) + (int)(threadIdx.x >> 6));
    if (g0 >= g_end) return;
    const int lane = threadIdx.x & 63;
    const int kh = d.kmax / 2;   // doubles per lane per row block (2 halves × kmax/4)
    const int kq = d.kmax / 4;
    const size_t opstride = (size_t)d.nb * 64 * kh;
    const size_t inst_elems = (size_t)d.ntiles * TILE_ELEMS;
    const double* Pin = reinterpret_cast<const double*>(p.Pin);
    double* Pout = reinterpret_cast<double*>(p.Pout);

    bool fast = d.kmax == 16;
    {
        const int e_lo = g0 / nwt, e_hi = (g_end - 1) / nwt;
        for (int e = e_lo; e <= e_hi; e++)
#pragma unroll
            for (int q = 0; q < NS; q++) {
                const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
                fast = fast && !sload(r + RES_RESET) && sload(r + RES_NADD) == 0 && !sload(r + RES_ROLLBACK);
            }
    }
    struct Item {
        int e, li;
        int tile[WT64_C];
        int valid, rowA, rowsB;
    };
    typedef int i32x8 __attribute__((ext_vector_type(8)));
    auto load_entry = [&](int li, Item& t) __attribute__((always_inline)) {
        const i32x8 v = sload(reinterpret_cast<const i32x8*>(p.wt64 + li));
        t.tile[0] = v[0];
        t.tile[1] = v[1];
        t.valid = v[WT_N];
        t.rowA = v[WT_N + 1];
        t.rowsB = v[WT_N + 2];
    };
    auto first_item = [&](Item& t) __attribute__((always_inline)) {
        t.e = g0 / nwt;
        t.li = g0 - t.e * nwt;
        load_entry(t.li, t);
    };
    auto next_item = [&](const Item& c, Item& t) __attribute__((always_inline)) {
        int li = c.li + K, e = c.e;
        while (li >= nwt) {
            li -= nwt;
            e++;
        }
        t.e = e;
        t.li = li;
        load_entry(e < p.E ? li : 0, t);
    };
    auto tile_base = [&](const Item& t, int i) __attribute__((always_inline)) {
        return (size_t)t.e * inst_elems + (size_t)t.tile[i] * TILE_ELEMS;
    };
    // lane's registers 0-1 of 16×16 block b of a tile at f64x2 b·128 + lane, 2-3 at b·128 + 64 + lane
    auto load_tiles = [&](const Item& t, f64x2 (&pref)[WT64_C][8]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT64_C; i++) {
            const f64x2* src = reinterpret_cast<const f64x2*>(Pin + tile_base(t, i)) + lane;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                pref[i][2 * b] = __builtin_nontemporal_load(src + b * 128);
                pref[i][2 * b + 1] = __builtin_nontemporal_load(src + b * 128 + 64);
            }
        }
    };
    // invalid slots to the sink tile (no branch around a store: see flush_f32_wave_kernel)
    auto store_tiles = [&](const Item& t, const f64x4 (&acc)[WT64_C][4]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT64_C; i++) {
            f64x2* dst = reinterpret_cast<f64x2*>(((t.valid >> i) & 1) ? Pout + tile_base(t, i)
                                                                      : reinterpret_cast<double*>(p.sink)) + lane;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                const f64x2 v0 = {acc[i][b][0], acc[i][b][1]};
                const f64x2 v1 = {acc[i][b][2], acc[i][b][3]};
                __builtin_nontemporal_store(v0, dst + b * 128);
                __builtin_nontemporal_store(v1, dst + b * 128 + 64);
            }
        }
    };
    // operand rows of step q for wave-tile t: A (its row block), B (its two column blocks), each
    // 8 doubles per lane ([half h][k-step s] at h·kq + s)
    auto load_ops = [&](const Item& t, int q, f64x2 (&a)[4], f64x2 (&b)[WT64_C][4]) __attribute__((always_inline)) {
        const double* U = reinterpret_cast<const double*>(p.steps[q].Uop) + t.e * opstride + lane * kh;
        const double* V = reinterpret_cast<const double*>(p.steps[q].Vop) + t.e * opstride + lane * kh;
        const f64x2* ua = reinterpret_cast<const f64x2*>(U + (size_t)t.rowA * 64 * kh);
#pragma unroll
        for (int k = 0; k < 4; k++) a[k] = ua[k];
#pragma unroll
        for (int c = 0; c < WT64_C; c++) {
            const int rb = (t.rowsB >> (16 * c)) & 0xffff;
            const f64x2* vb = reinterpret_cast<const f64x2*>(V + (size_t)rb * 64 * kh);
#pragma unroll
            for (int k = 0; k < 4; k++) b[c][k] = vb[k];
        }
    };
    // the 4 k-steps of one step: acc[c][h·2 + hc] += A[h] · B[c][hc]
    auto mfma_step = [&](const f64x2 (&a)[4], const f64x2 (&b)[WT64_C][4], f64x4 (&acc)[WT64_C][4]) __attribute__((always_inline)) {
#pragma unroll
        for (int s4 = 0; s4 < 4; s4++) {
            const double a0 = a[s4 >> 1][s4 & 1], a1 = a[2 + (s4 >> 1)][s4 & 1];
#pragma unroll
            for (int c = 0; c < WT64_C; c++) {
                const double b0 = b[c][s4 >> 1][s4 & 1], b1 = b[c][2 + (s4 >> 1)][s4 & 1];
                acc[c][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[c][0], 0, 0, 0);
                acc[c][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[c][1], 0, 0, 0);
                acc[c][2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[c][2], 0, 0, 0);
                acc[c][3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[c][3], 0, 0, 0);
            }
        }
    };
    auto to_acc = [&](const f64x2 (&pref)[WT64_C][8], f64x4 (&acc)[WT64_C][4]) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < WT64_C; i++)
#pragma unroll
            for (int b = 0; b < 4; b++)
                acc[i][b] = f64x4{pref[i][2 * b][0], pref[i][2 * b][1], pref[i][2 * b + 1][0], pref[i][2 * b + 1][1]};
    };

    if (fast) {
        // operand ring of RD steps: step q + RD's rows load into step q's registers after its
        // MFMAs (the next wave-tile's once q + RD >= NS; RD = NS up to four steps)
        constexpr int RD = NS < F64_RING ? NS : F64_RING;
        f64x2 pref[WT64_C][8];
        f64x2 opa[RD][4], opb[RD][WT64_C][4];
        f64x4 acc[WT64_C][4];
        Item cur, nxt, nxt2;
        first_item(cur);
        next_item(cur, nxt);
        load_tiles(cur, pref);
#pragma unroll
        for (int q = 0; q < RD; q++) load_ops(cur, q, opa[q], opb[q]);
        int g = g0;
        while (true) {
            const bool more = g + K < g_end;
            next_item(nxt, nxt2);
            const Item ldi = more ? nxt : cur;   // the last wave-tile re-reads its own (no branch)
            to_acc(pref, acc);
            if (more) load_tiles(nxt, pref);
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int q = 0; q < NS; q++) {
                mfma_step(opa[q % RD], opb[q % RD], acc);
                __builtin_amdgcn_sched_barrier(0);
                if (q + RD < NS) load_ops(cur, q + RD, opa[q % RD], opb[q % RD]);
                else load_ops(ldi, q + RD - NS, opa[q % RD], opb[q % RD]);   // the next wave-tile's
            }
            store_tiles(cur, acc);
            if (!more) break;
            g += K;
            cur = nxt;
            nxt = nxt2;
        }
        return;
    }

    // general loop: per wave-tile, every step in order (reset, or the k-steps of its matches, then
    // its augmented rows), operands loaded in place
    Item t;
    first_item(t);
    for (int g = g0; g < g_end; g += K) {
        if (g != g0) {
            Item n;
            next_item(t, n);
            t = n;
        }
        f64x2 pref[WT64_C][8];
        f64x4 acc[WT64_C][4];
        load_tiles(t, pref);
        to_acc(pref, acc);
        const int wc0 = (t.rowsB & 0xffff);
        for (int q = 0; q < NS; q++) {
            const int* r = p.steps[q].res + (size_t)t.e * RES_STRIDE;
            if (sload(r + RES_RESET)) {
#pragma unroll
                for (int i = 0; i < WT64_C; i++)
#pragma unroll
                    for (int b = 0; b < 4; b++) acc[i][b] = f64x4{0.0, 0.0, 0.0, 0.0};
                continue;
            }
            const int ks = sload(r + RES_KSTEPS);
            if (ks > 0) {
                const double* U = reinterpret_cast<const double*>(p.steps[q].Uop) + t.e * opstride + lane * kh;
                const double* V = reinterpret_cast<const double*>(p.steps[q].Vop) + t.e * opstride + lane * kh;
                const double* A = U + (size_t)t.rowA * 64 * kh;
                for (int s4 = 0; s4 < ks; s4++) {
                    const double a0 = A[s4], a1 = A[kq + s4];
#pragma unroll
                    for (int c = 0; c < WT64_C; c++) {
                        const double* B = V + (size_t)((t.rowsB >> (16 * c)) & 0xffff) * 64 * kh;
                        const double b0 = B[s4], b1 = B[kq + s4];
                        acc[c][0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[c][0], 0, 0, 0);
                        acc[c][1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[c][1], 0, 0, 0);
                        acc[c][2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[c][2], 0, 0, 0);
                        acc[c][3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[c][3], 0, 0, 0);
                    }
                }
            }
            const int nadd = sload(r + RES_NADD), s0 = sload(r + RES_SAVED_IN);
            if (nadd <= 0 || (wc0 + WT64_C) * 16 <= s0 || wc0 * 16 >= s0 + nadd) continue;
            const double* prw0 = p.steps[q].patch + (size_t)t.e * d.max_lines * 2 * d.M;
            const double* pdg = p.steps[q].patch_diag + (size_t)t.e * d.max_lines * 4;
#pragma unroll
            for (int c = 0; c < WT64_C; c++) {
                const int bj = wc0 + c;
                if (!((t.valid >> c) & 1) || bj * 16 + 15 < s0 || bj * 16 >= s0 + nadd) continue;
#pragma unroll
                for (int blk = 0; blk < 4; blk++)
#pragma unroll
                    for (int reg = 0; reg < 4; reg++) {
                        const int row = t.rowA * 32 + (lane >> 4) + 4 * reg + 16 * (blk >> 1);
                        const int col = bj * 32 + (lane & 15) + 16 * (blk & 1);
                        const int hi = max(row >> 1, col >> 1);
                        if (hi >= s0 && hi < s0 + nadd) acc[c][blk][reg] = patched_value(prw0, pdg, d.M, s0, row, col);
                    }
            }
        }
        store_tiles(t, acc);
    }
}

#if !defined(EKF_TU) || EKF_TU == 2   // (a plain kernel: defined in the flush unit only)
__global__ __launch_bounds__(DD_THREADS) void downdate_f64_kernel(DowndateParams p)
{
    const Dims d = p.d;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (DD_THREADS / 64);
    const int64_t total = (int64_t)p.E * d.ntiles;
    const int kh = d.kmax / 2;   // doubles per lane per row block (2 halves × kmax/4)
    const int kq = d.kmax / 4;
    const size_t opstride = (size_t)d.nb * 64 * kh;
    for (int64_t g = (int64_t)blockIdx.x * (DD_THREADS / 64) + (threadIdx.x >> 6); g < total;
         g += nwaves) {
        const int e = (int)(g / d.ntiles);
        const int64_t t = g - (int64_t)e * d.ntiles;
        const size_t toff = ((size_t)e * d.ntiles + t) * TILE_ELEMS;
        // lane's registers 0-1 of block qq at qq·128 + lane, registers 2-3 at qq·128 + 64 + lane
        const f64x2* src = reinterpret_cast<const f64x2*>(reinterpret_cast<const double*>(p.Pin) + toff) + lane;
        f64x2* dst = reinterpret_cast<f64x2*>(reinterpret_cast<double*>(p.Pout) + toff) + lane;
        const int2 rc = p.tile_rc[t];
        bool work = false;
        for (int q = 0; q < p.nsteps; q++) {
            const int* r = p.steps[q].res + (size_t)e * RES_STRIDE;
            const int nadd = r[RES_NADD], s0 = r[RES_SAVED_IN];
            work |= r[RES_RESET] || r[RES_KSTEPS] > 0 ||
                    (nadd > 0 && rc.y * 16 + 15 >= s0 && rc.y * 16 < s0 + nadd);
        }
        if (!work) {
            if (p.Pin != p.Pout) {
#pragma unroll
                for (int qq = 0; qq < 4; qq++) {
                    __builtin_nontemporal_store(__builtin_nontemporal_load(src + qq * 128), dst + qq * 128);
                    __builtin_nontemporal_store(__builtin_nontemporal_load(src + qq * 128 + 64), dst + qq * 128 + 64);
                }
            }
            continue;
        }
        f64x4 acc[4];
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const f64x2 v0 = __builtin_nontemporal_load(src + qq * 128);
            const f64x2 v1 = __builtin_nontemporal_load(src + qq * 128 + 64);
            acc[qq][0] = v0[0];
            acc[qq][1] = v0[1];
            acc[qq][2] = v1[0];
            acc[qq][3] = v1[1];
        }
        for (int q = 0; q < p.nsteps; q++) {
            const Slot& sq = p.steps[q];
            const int* r = sq.res + (size_t)e * RES_STRIDE;
            if (r[RES_RESET]) {
#pragma unroll
                for (int qq = 0; qq < 4; qq++) acc[qq] = f64x4{0.0, 0.0, 0.0, 0.0};
                continue;
            }
            const int ks = r[RES_KSTEPS];
            if (ks > 0) {
                const double* A = reinterpret_cast<const double*>(sq.Uop) + e * opstride +
                                  ((size_t)rc.x * 64 + lane) * kh;
                const double* B = reinterpret_cast<const double*>(sq.Vop) + e * opstride +
                                  ((size_t)rc.y * 64 + lane) * kh;
                for (int s = 0; s < ks; s++) {
                    const double a0 = A[s], a1 = A[kq + s];
                    const double b0 = B[s], b1 = B[kq + s];
                    acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
                    acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
                    acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
                    acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
                }
            }
            const int nadd = r[RES_NADD], s0 = r[RES_SAVED_IN];
            if (nadd > 0 && rc.y * 16 + 15 >= s0 && rc.y * 16 < s0 + nadd) {
                const double* prw0 = sq.patch + (size_t)e * d.max_lines * 2 * d.M;
                const double* pdg = sq.patch_diag + (size_t)e * d.max_lines * 4;
#pragma unroll
                for (int blk = 0; blk < 4; blk++)
#pragma unroll
                    for (int reg = 0; reg < 4; reg++) {
                        const int row = rc.x * 32 + (lane >> 4) + 4 * reg + 16 * (blk >> 1);
                        const int col = rc.y * 32 + (lane & 15) + 16 * (blk & 1);
                        const int hi = max(row >> 1, col >> 1);
                        if (hi >= s0 && hi < s0 + nadd)
                            acc[blk][reg] = patched_value(prw0, pdg, d.M, s0, row, col);
                    }
            }
        }
#pragma unroll
        for (int qq = 0; qq < 4; qq++) {
            const f64x2 v0 = {acc[qq][0], acc[qq][1]};
            const f64x2 v1 = {acc[qq][2], acc[qq][3]};
            __builtin_nontemporal_store(v0, dst + qq * 128);
            __builtin_nontemporal_store(v1, dst + qq * 128 + 64);
        }
    }
}

// ---------------------------------------------------------------------------------------
// state transfer / initialisation
// ---------------------------------------------------------------------------------------
#endif

template <typename T>
__device__ __forceinline__ void tile_rc_of(int rem, int& r, int& c)
{
    if (sizeof(typename Stor<T>::L) == 4) {
        const int q = rem & 3, lane = (rem >> 2) & 63, grp = rem >> 8;
        c = lane & 31;
        r = q + 4 * (lane >> 5) + 8 * grp;
    } else {
        const int reg = (rem & 1) + 2 * ((rem >> 7) & 1), lane = (rem >> 1) & 63, blk = rem >> 8;
        c = (lane & 15) + 16 * (blk & 1);
        r = (lane >> 4) + 4 * reg + 16 * (blk >> 1);
    }
}

// pack / unpack / lowrank cover the tiles [t0, t1) (a partitioned instance stores a slice; Pll points
// at the slice's first tile, t0)
template <typename T>
__global__ void pack_kernel(Dims d, const double* __restrict__ Pfull, T* __restrict__ Pll,
                            double* __restrict__ Rs, const int2* __restrict__ tile_rc, int ex,
                            int64_t t0, int64_t t1)
{
    const int64_t total = (t1 - t0) * TILE_ELEMS;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = t0 + g / TILE_ELEMS;
        int r, c;
        tile_rc_of<T>((int)(g % TILE_ELEMS), r, c);
        const int2 rc = tile_rc[t];
        const int i = rc.x * TILE + r, j = rc.y * TILE + c;
        double v = 0.0;
        if (i < d.M && j < d.M) v = Pfull[(size_t)(3 + i) * d.n + (3 + j)];
        Pll[g] = to_store<T>(to_domain<T>(v, ex));
    }
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < 3 * (int64_t)d.n;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(g / d.n), b = (int)(g % d.n);
        Rs[g] = Pfull[(size_t)a * d.n + b];
    }
}

template <typename T>
__global__ void unpack_kernel(Dims d, double* __restrict__ Pfull, const T* __restrict__ Pll,
                              const double* __restrict__ Rs, int ex, int64_t t0, int64_t t1)
{
    const int64_t total = (int64_t)d.n * d.n;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(g / d.n), b = (int)(g % d.n);
        double v;
        if (a < 3) v = Rs[(size_t)a * d.n + b];
        else if (b < 3) v = Rs[(size_t)b * d.n + a];
        else {
            // the tiles of another rank read as 0
            const int ba = (a - 3) >> 5, bb = (b - 3) >> 5;
            const int64_t t = tile_index(ba < bb ? ba : bb, ba < bb ? bb : ba, d.nb);
            v = (t >= t0 && t < t1)
                    ? from_domain<T>(from_store<T>(Pll[ll_offset<typename Stor<T>::L>(a - 3, b - 3, d.nb) - t0 * TILE_ELEMS]), ex)
                    : 0.0;
        }
        Pfull[g] = v;
    }
}

template <typename T>
__global__ void lowrank_kernel(Dims d, const double* __restrict__ diag,
                               const double* __restrict__ U, int rank, T* __restrict__ Pll,
                               double* __restrict__ Rs, const int2* __restrict__ tile_rc, int ex,
                               int64_t t0, int64_t t1)
{
    const int64_t total = (t1 - t0) * TILE_ELEMS;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = t0 + g / TILE_ELEMS;
        int r, c;
        tile_rc_of<T>((int)(g % TILE_ELEMS), r, c);
        const int2 rc = tile_rc[t];
        const int i = rc.x * TILE + r, j = rc.y * TILE + c;
        double v = 0.0;
        if (i < d.M && j < d.M) {
            const double* ui = U + (size_t)(3 + i) * rank;
            const double* uj = U + (size_t)(3 + j) * rank;
            for (int k = 0; k < rank; k++) v += ui[k] * uj[k];
            if (i == j) v += diag[3 + i];
        }
        Pll[g] = to_store<T>(to_domain<T>(v, ex));
    }
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < 3 * (int64_t)d.n;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(g / d.n), b = (int)(g % d.n);
        const double* ua = U + (size_t)a * rank;
        const double* ub = U + (size_t)b * rank;
        double v = 0.0;
        for (int k = 0; k < rank; k++) v += ua[k] * ub[k];
        if (a == b) v += diag[a];
        Rs[g] = v;
    }
}

// ---------------------------------------------------------------------------------------
// launchers
// ---------------------------------------------------------------------------------------
// The association kernel on 128 / 64 landmarks per workgroup (ScanParams::nt): its HOT
// instantiations (symmetric fp32 operands, kmax = 16; HOT = 2 split-fp16, 1 the others), one
// compilation unit per width (EKF_TU 7, 8)
hipError_t launch_scan_nt128(const ScanParams& p, bool half, bool f16x3, hipStream_t st);
hipError_t launch_scan_nt64(const ScanParams& p, bool half, bool f16x3, hipStream_t st);

#if !defined(EKF_TU) || EKF_TU == 7
hipError_t launch_scan_nt128(const ScanParams& p, bool half, bool f16x3, hipStream_t st)
{
    const dim3 grid(p.G * p.E), block(128 + 64);
    if (f16x3) {
        if (half) hipLaunchKernelGGL((scan_kernel<_Float16, false, 2, 128>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 2, 128>), grid, block, 0, st, p);
    } else {
        if (half) hipLaunchKernelGGL((scan_kernel<_Float16, false, 1, 128>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 1, 128>), grid, block, 0, st, p);
    }
    return hipGetLastError();
}
#endif

#if !defined(EKF_TU) || EKF_TU == 8
hipError_t launch_scan_nt64(const ScanParams& p, bool half, bool f16x3, hipStream_t st)
{
    const dim3 grid(p.G * p.E), block(64 + 64);
    if (f16x3) {
        if (half) hipLaunchKernelGGL((scan_kernel<_Float16, false, 2, 64>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 2, 64>), grid, block, 0, st, p);
    } else {
        if (half) hipLaunchKernelGGL((scan_kernel<_Float16, false, 1, 64>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 1, 64>), grid, block, 0, st, p);
    }
    return hipGetLastError();
}
#endif

#if !defined(EKF_TU) || EKF_TU == 1
int scan_blocks_per_cu(int precision)
{
    int nb = 0;
    hipError_t err =
        (precision == EKF_PREC_F64) ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, scan_kernel<double, false, 0>, SCAN_BLOCK, 0)
        : (precision == EKF_PREC_F16) ? hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, scan_kernel<_Float16, false, 0>, SCAN_BLOCK, 0)
        : hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, scan_kernel<float, false, 0>, SCAN_BLOCK, 0);
    return err == hipSuccess ? nb : 0;
}

size_t scan_lds_bytes(int precision)
{
    hipFuncAttributes a;
    hipError_t err =
        (precision == EKF_PREC_F64) ? hipFuncGetAttributes(&a, reinterpret_cast<const void*>(scan_kernel<double, false, 0>))
        : (precision == EKF_PREC_F16) ? hipFuncGetAttributes(&a, reinterpret_cast<const void*>(scan_kernel<_Float16, false, 0>))
        : hipFuncGetAttributes(&a, reinterpret_cast<const void*>(scan_kernel<float, false, 0>));
    return err == hipSuccess ? a.sharedSizeBytes : 0;
}

#endif

#if !defined(EKF_TU) || EKF_TU == 3
hipError_t launch_shard_run(const ShardParams& p, int precision, hipStream_t st)
{
    const unsigned G = (unsigned)shard_run_workgroups(p.d.N);
    // at most SH_MAX_LINES lines: one verdict exchange for the run (shard_spec_kernel); otherwise
    // one exchange per line (shard_run_kernel)
    if (EKF_SHARD_SPEC && p.L <= SH_MAX_LINES && p.d.max_lines <= SH_MAX_LINES) {
        if (precision == EKF_PREC_F64) hipLaunchKernelGGL(shard_spec_kernel<double>, dim3(G), dim3(SPR_THREADS), 0, st, p);
        else if (precision == EKF_PREC_F32) hipLaunchKernelGGL(shard_spec_kernel<float>, dim3(G), dim3(SPR_THREADS), 0, st, p);
        else return hipErrorInvalidValue;
        return hipGetLastError();
    }
    if (precision == EKF_PREC_F64) hipLaunchKernelGGL(shard_run_kernel<double>, dim3(G), dim3(SHR_THREADS), 0, st, p);
    else if (precision == EKF_PREC_F32) hipLaunchKernelGGL(shard_run_kernel<float>, dim3(G), dim3(SHR_THREADS), 0, st, p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

hipError_t launch_shard(const ShardParams& p, int precision, hipStream_t st)
{
    // every landmark, one per thread, spread over ⌈N/64⌉ CUs
    // (the guesses and the guessed columns: one grid row per line)
    const bool per_line = p.phase == SH_SPEC_COLS || p.phase == SH_GUESS;
    const dim3 grid((unsigned)((p.d.N + SH_THREADS - 1) / SH_THREADS), per_line ? (unsigned)max(p.L, 1) : 1u);
    if (precision == EKF_PREC_F64) hipLaunchKernelGGL(shard_kernel<double>, grid, dim3(SH_THREADS), 0, st, p);
    else if (precision == EKF_PREC_F32) hipLaunchKernelGGL(shard_kernel<float>, grid, dim3(SH_THREADS), 0, st, p);
    else return hipErrorInvalidValue;
    return hipGetLastError();
}

#endif

#if !defined(EKF_TU) || EKF_TU == 1
hipError_t launch_scan(const ScanParams& p, int precision, hipStream_t st)
{
    if (p.nt != SCAN_THREADS) {   // (the context picks a narrow width for the HOT instantiations only)
        if (p.dbg || precision == EKF_PREC_F64 || p.r_mode == 1 || p.d.kmax != 16) return hipErrorInvalidValue;
        const bool half = precision == EKF_PREC_F16, f16x3 = p.bf == 2;
        if (p.nt == 128) return launch_scan_nt128(p, half, f16x3, st);
        if (p.nt == 64) return launch_scan_nt64(p, half, f16x3, st);
        return hipErrorInvalidValue;
    }
    const dim3 grid(p.G * p.E), block(SCAN_BLOCK);
    if (p.dbg) {   // phase timers (EKF_OPT_SCAN_STAMPS): the instrumented instantiation
        if (precision == EKF_PREC_F64) hipLaunchKernelGGL((scan_kernel<double, true, 0>), grid, block, 0, st, p);
        else if (precision == EKF_PREC_F16) hipLaunchKernelGGL((scan_kernel<_Float16, true, 0>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, true, 0>), grid, block, 0, st, p);
    } else if (precision != EKF_PREC_F64 && p.r_mode != 1 && p.d.kmax == 16 && p.bf == 2) {
        if (precision == EKF_PREC_F16) hipLaunchKernelGGL((scan_kernel<_Float16, false, 2>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 2>), grid, block, 0, st, p);
    } else if (precision != EKF_PREC_F64 && p.r_mode != 1 && p.d.kmax == 16) {
        if (precision == EKF_PREC_F16) hipLaunchKernelGGL((scan_kernel<_Float16, false, 1>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 1>), grid, block, 0, st, p);
    } else {
        if (precision == EKF_PREC_F64) hipLaunchKernelGGL((scan_kernel<double, false, 0>), grid, block, 0, st, p);
        else if (precision == EKF_PREC_F16) hipLaunchKernelGGL((scan_kernel<_Float16, false, 0>), grid, block, 0, st, p);
        else hipLaunchKernelGGL((scan_kernel<float, false, 0>), grid, block, 0, st, p);
    }
    return hipGetLastError();
}

#endif

// The split-arithmetic flush launchers, one compilation unit each (EKF_TU 4-6: their template
// instantiations are most of the library's device code)
hipError_t launch_flush_bf24(const DowndateParams& p, bool half, bool f16, hipStream_t st, hipEvent_t ev_a,
                             hipEvent_t ev_b);
hipError_t launch_flush_f16x3(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b);
hipError_t launch_flush_bf16x6(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b);
hipError_t launch_flush_f16q(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b);

#if !defined(EKF_TU) || EKF_TU == 9
hipError_t launch_flush_f16q(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b)
{
    const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one workgroup per CU
#define EKF_F16Q_CASE(NSV)                                                                              \
    case NSV:                                                                                           \
        if (half) hipExtLaunchKernelGGL((flush_f16q_kernel<_Float16, NSV>), dim3(wgrid), dim3(64 * Q_WAVES), 0, st, \
                                        ev_a, ev_b, 0, p);                                              \
        else hipExtLaunchKernelGGL((flush_f16q_kernel<float, NSV>), dim3(wgrid), dim3(64 * Q_WAVES), 0, st, ev_a, \
                                   ev_b, 0, p);                                                         \
        break;
    switch (p.nsteps) {
        EKF_F16Q_CASE(6)
        EKF_F16Q_CASE(8)
        EKF_F16Q_CASE(10)
        EKF_F16Q_CASE(12)
        EKF_F16Q_CASE(14)
        EKF_F16Q_CASE(16)
        EKF_F16Q_CASE(18)
        EKF_F16Q_CASE(20)
        EKF_F16Q_CASE(22)
        EKF_F16Q_CASE(24)
        default: return hipErrorInvalidValue;
    }
#undef EKF_F16Q_CASE
    return hipGetLastError();
}
#endif

#if !defined(EKF_TU) || EKF_TU == 4
hipError_t launch_flush_f16x3(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b)
{
    const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one 4-wave workgroup per CU
#define EKF_F16_CASE(NSV)                                                                               \
case NSV:                                                                                           \
    if (half) hipExtLaunchKernelGGL((flush_f32_wave_kernel<_Float16, NSV, true, true>), dim3(wgrid),  \
                                    dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);                      \
    else hipExtLaunchKernelGGL((flush_f32_wave_kernel<float, NSV, true, true>), dim3(wgrid),          \
                               dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);                           \
    break;
    switch (p.nsteps) {
        EKF_F16_CASE(2)
        EKF_F16_CASE(4)
        EKF_F16_CASE(6)
        EKF_F16_CASE(8)
        EKF_F16_CASE(10)
        EKF_F16_CASE(12)
        EKF_F16_CASE(14)
        EKF_F16_CASE(16)
        EKF_F16_CASE(18)
        EKF_F16_CASE(20)
        EKF_F16_CASE(22)
        EKF_F16_CASE(24)
    }
#undef EKF_F16_CASE
    return hipGetLastError();
}
#endif

#if !defined(EKF_TU) || EKF_TU == 5
hipError_t launch_flush_bf24(const DowndateParams& p, bool half, bool f16, hipStream_t st, hipEvent_t ev_a,
                             hipEvent_t ev_b)
{
    if (!f16) {
        // EKF_ARITH_BF16X6, EKF_FLUSH_VARIANT=24: the 2 × 4 split-bf16 wave flush (measured 7 %
        // slower than the 2 × 2 form below at T = 12; kept as an option, bit-identical)
        const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one 4-wave workgroup per CU
#define EKF_BF24_CASE(NSV)                                                                              \
    case NSV:                                                                                           \
        if (half) hipExtLaunchKernelGGL((flush_bf24_kernel<_Float16, NSV>), dim3(wgrid), dim3(DD_THREADS), 0, st, \
                                        ev_a, ev_b, 0, p);                                              \
        else hipExtLaunchKernelGGL((flush_bf24_kernel<float, NSV>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, \
                                   ev_b, 0, p);                                                         \
        break;
        switch (p.nsteps) {
            EKF_BF24_CASE(2)
            EKF_BF24_CASE(4)
            EKF_BF24_CASE(6)
            EKF_BF24_CASE(8)
            EKF_BF24_CASE(10)
            EKF_BF24_CASE(12)
            EKF_BF24_CASE(14)
            EKF_BF24_CASE(16)
        }
#undef EKF_BF24_CASE
        return hipGetLastError();
        }
        // EKF_ARITH_F16X3, EKF_OPT_FLUSH_FORM = 24: the 2 × 4 split-fp16 flush
        const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));
#define EKF_F24_CASE(NSV)                                                                               \
    case NSV:                                                                                           \
        if (half) hipExtLaunchKernelGGL((flush_bf24_kernel<_Float16, NSV, true>), dim3(wgrid), dim3(DD_THREADS), 0, st, \
                                        ev_a, ev_b, 0, p);                                               \
        else hipExtLaunchKernelGGL((flush_bf24_kernel<float, NSV, true>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, \
                                   ev_b, 0, p);                                                          \
        break;
        switch (p.nsteps) {
            EKF_F24_CASE(2)
            EKF_F24_CASE(4)
            EKF_F24_CASE(6)
            EKF_F24_CASE(8)
            EKF_F24_CASE(10)
            EKF_F24_CASE(12)
            EKF_F24_CASE(14)
            EKF_F24_CASE(16)
            EKF_F24_CASE(18)
            EKF_F24_CASE(20)
            EKF_F24_CASE(22)
            EKF_F24_CASE(24)
        }
#undef EKF_F24_CASE
        return hipGetLastError();
    }
#endif

#if !defined(EKF_TU) || EKF_TU == 6
hipError_t launch_flush_bf16x6(const DowndateParams& p, bool half, hipStream_t st, hipEvent_t ev_a, hipEvent_t ev_b)
{
    const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one 4-wave workgroup per CU
#define EKF_BF_CASE(NSV)                                                                                \
case NSV:                                                                                           \
    if (half) hipExtLaunchKernelGGL((flush_f32_wave_kernel<_Float16, NSV, true>), dim3(wgrid), dim3(DD_THREADS), 0, \
                                    st, ev_a, ev_b, 0, p);                                          \
    else hipExtLaunchKernelGGL((flush_f32_wave_kernel<float, NSV, true>), dim3(wgrid), dim3(DD_THREADS), 0, st, \
                               ev_a, ev_b, 0, p);                                                   \
    break;
    switch (p.nsteps) {
        EKF_BF_CASE(2)
        EKF_BF_CASE(4)
        EKF_BF_CASE(6)
        EKF_BF_CASE(8)
        EKF_BF_CASE(10)
        EKF_BF_CASE(12)
        EKF_BF_CASE(14)
        EKF_BF_CASE(16)
    }
#undef EKF_BF_CASE
    return hipGetLastError();
}
#endif

#if !defined(EKF_TU) || EKF_TU == 2
hipError_t launch_downdate(const DowndateParams& p, int precision, int grid, hipStream_t st, hipEvent_t ev_a,
                           hipEvent_t ev_b)
{
    if (precision == EKF_PREC_F64) {
        if (p.nsteps <= F64_WAVE_MAXS && p.d.kmax == 16 && p.nwt64 > 0 && p.wt64 != nullptr && p.variant != 2) {
            const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one 4-wave workgroup per CU
            switch (p.nsteps) {
            case 1: hipExtLaunchKernelGGL((flush_f64_wave_kernel<1>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 2: hipExtLaunchKernelGGL((flush_f64_wave_kernel<2>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 3: hipExtLaunchKernelGGL((flush_f64_wave_kernel<3>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 4: hipExtLaunchKernelGGL((flush_f64_wave_kernel<4>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 5: hipExtLaunchKernelGGL((flush_f64_wave_kernel<5>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 6: hipExtLaunchKernelGGL((flush_f64_wave_kernel<6>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            case 7: hipExtLaunchKernelGGL((flush_f64_wave_kernel<7>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            default: hipExtLaunchKernelGGL((flush_f64_wave_kernel<8>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); break;
            }
            return hipGetLastError();
        }
        hipExtLaunchKernelGGL(downdate_f64_kernel, dim3(grid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);
        return hipGetLastError();
    }
    const bool half = precision == EKF_PREC_F16;
    // default: the wave flush for groups of 6 or 8 steps; EKF_FLUSH_VARIANT 8 forces it (also
    // for 2 or 4 steps)
    const bool wave_shape = p.nsteps >= 2 && p.nsteps <= 8 && p.nsteps % 2 == 0 && p.d.kmax <= 16 &&
                            p.nwt > 0 && p.wt != nullptr;
    const bool wave_ok = wave_shape && (p.nsteps >= 6 || p.variant == 8);
    const bool bf_shape = p.nsteps >= 2 && p.nsteps <= (p.bf == 2 ? F16X3_MAXS : 16) && p.nsteps % 2 == 0 && p.d.kmax <= 16 &&
                          p.nwt > 0 && p.wt != nullptr;
    if (p.bf == 1 && bf_shape && p.variant == 24 && p.nwt24 > 0 && p.wt24 != nullptr)
        return launch_flush_bf24(p, half, false, st, ev_a, ev_b);
    if (p.bf == 2 && bf_shape && p.variant == 24 && p.nwt24 > 0 && p.wt24 != nullptr)
        return launch_flush_bf24(p, half, true, st, ev_a, ev_b);
    if (p.bf == 2 && bf_shape && p.variant == 44 && p.nsteps >= 6 && p.nwtq > 0 && p.wtq != nullptr)
        return launch_flush_f16q(p, half, st, ev_a, ev_b);   // the quad form (groups of 6-24 steps)
    if (p.bf == 2 && bf_shape)   // EKF_ARITH_F16X3: split-fp16 wave flush, groups of 2-24 steps (even)
        return launch_flush_f16x3(p, half, st, ev_a, ev_b);
    if (p.bf == 1 && bf_shape)   // EKF_ARITH_BF16X6: split-bf16 wave flush, groups of 2-16 steps (even)
        return launch_flush_bf16x6(p, half, st, ev_a, ev_b);
    if (wave_ok) {
        const unsigned wgrid = (unsigned)(8 * ((p.ncu + 7) / 8));   // one 4-wave workgroup per CU
#define EKF_WAVE_CASE(NSV)                                                                              \
    case NSV:                                                                                           \
        if (half) hipExtLaunchKernelGGL((flush_f32_wave_kernel<_Float16, NSV>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p); \
        else hipExtLaunchKernelGGL((flush_f32_wave_kernel<float, NSV>), dim3(wgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);         \
        break;
        switch (p.nsteps) {
            EKF_WAVE_CASE(2)
            EKF_WAVE_CASE(4)
            EKF_WAVE_CASE(6)
            EKF_WAVE_CASE(8)
        }
#undef EKF_WAVE_CASE
        return hipGetLastError();
    }
    if (p.nsteps <= PST_MAXC && p.d.kmax <= 16 && p.variant != 2) {
        const int pgrid = 16 * ((p.ncu + 7) / 8);   // two workgroups per CU (48 KB LDS each)
        if (half)
            hipExtLaunchKernelGGL(flush_f32_persist2_kernel<_Float16>, dim3((unsigned)pgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);
        else
            hipExtLaunchKernelGGL(flush_f32_persist2_kernel<float>, dim3((unsigned)pgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);
    } else {
        const int64_t nsb = (p.d.nb + DD_SB - 1) / DD_SB;
        const int64_t total = (int64_t)p.E * (nsb * (nsb + 1) / 2);
        const unsigned sgrid = (unsigned)(8 * ((total + 7) / 8));
        if (half)
            hipExtLaunchKernelGGL(flush_f32_sb_kernel<_Float16>, dim3(sgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);
        else
            hipExtLaunchKernelGGL(flush_f32_sb_kernel<float>, dim3(sgrid), dim3(DD_THREADS), 0, st, ev_a, ev_b, 0, p);
    }
    return hipGetLastError();
}

#endif

#if !defined(EKF_TU) || EKF_TU == 3
static int grid_for(int64_t work, int block)
{
    int64_t g = (work + block - 1) / block;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_pack(const Dims& d, int precision, const double* Pfull, void* Pll, double* Rs,
                       const int2* tile_rc, int ex, hipStream_t st, int64_t t0, int64_t t1)
{
    if (t1 < 0) t1 = d.ntiles;
    const int grid = grid_for((t1 - t0) * TILE_ELEMS, 256);
    if (precision == EKF_PREC_F64)
        hipLaunchKernelGGL(pack_kernel<double>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (double*)Pll, Rs, tile_rc, ex, t0, t1);
    else if (precision == EKF_PREC_F16)
        hipLaunchKernelGGL(pack_kernel<_Float16>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (_Float16*)Pll, Rs, tile_rc, ex, t0, t1);
    else
        hipLaunchKernelGGL(pack_kernel<float>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (float*)Pll, Rs, tile_rc, ex, t0, t1);
    return hipGetLastError();
}

hipError_t launch_unpack(const Dims& d, int precision, double* Pfull, const void* Pll,
                         const double* Rs, int ex, hipStream_t st, int64_t t0, int64_t t1)
{
    if (t1 < 0) t1 = d.ntiles;
    const int grid = grid_for((int64_t)d.n * d.n, 256);
    if (precision == EKF_PREC_F64)
        hipLaunchKernelGGL(unpack_kernel<double>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (const double*)Pll, Rs, ex, t0, t1);
    else if (precision == EKF_PREC_F16)
        hipLaunchKernelGGL(unpack_kernel<_Float16>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (const _Float16*)Pll, Rs, ex, t0, t1);
    else
        hipLaunchKernelGGL(unpack_kernel<float>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (const float*)Pll, Rs, ex, t0, t1);
    return hipGetLastError();
}

hipError_t launch_lowrank(const Dims& d, int precision, const double* diag, const double* U,
                          int rank, void* Pll, double* Rs, const int2* tile_rc, int ex, hipStream_t st,
                          int64_t t0, int64_t t1)
{
    if (t1 < 0) t1 = d.ntiles;
    const int grid = grid_for((t1 - t0) * TILE_ELEMS, 256);
    if (precision == EKF_PREC_F64)
        hipLaunchKernelGGL(lowrank_kernel<double>, dim3(grid), dim3(256), 0, st, d, diag, U,
                           rank, (double*)Pll, Rs, tile_rc, ex, t0, t1);
    else if (precision == EKF_PREC_F16)
        hipLaunchKernelGGL(lowrank_kernel<_Float16>, dim3(grid), dim3(256), 0, st, d, diag, U,
                           rank, (_Float16*)Pll, Rs, tile_rc, ex, t0, t1);
    else
        hipLaunchKernelGGL(lowrank_kernel<float>, dim3(grid), dim3(256), 0, st, d, diag, U,
                           rank, (float*)Pll, Rs, tile_rc, ex, t0, t1);
    return hipGetLastError();
}

#endif

}  // namespace ekf
