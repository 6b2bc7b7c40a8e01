// ekf_kernels.hip — gfx950 kernels of the EKF-SLAM update (slam_ros Robot::localize).
//
// Per scan, three launches on one stream, all E ensemble instances at once:
//   1. scan_kernel     (1 workgroup of 1024 threads per instance)
//        predict of the robot strip (Robot.cpp:130-286, only rows 0..2 of Fx differ from I),
//        then for every observed line in order: Mahalanobis gating of all unmatched saved
//        landmarks in parallel with a min-index reduction (== the reference's first-passing
//        candidate, Robot.cpp:313-504), and for a match the gain chain in deferred low-rank
//        form (Robot.cpp:515-602): W_t = P_{t-1}·H_tᵀ from the robot strip + two landmark
//        columns of P_ll corrected by the earlier matches of this scan, K_t = W_t·S_t⁻¹,
//        U_t = K_t·S_t, y += K_t·v_t. The robot strip and the landmark 2×2 diagonal blocks are
//        downdated eagerly (O(n) per match); the landmark block P_ll is not touched.
//   2. downdate_kernel (grid-stride over E × packed 32×32 tiles, one tile per wave)
//        P_ll ← P_ll − Σ_t U_t·V_tᵀ (rank 2m) on MFMA, reading and writing every stored tile
//        once — the reference's m dense n×n passes (Robot.cpp:560-572) fused into one.
//        Also performs the capacity reset of P_ll (Robot.cpp:893-904).
//   3. augment_kernel  (1 workgroup per instance): new landmarks (Robot.cpp:776-866).
#include <hip/hip_runtime.h>

#include "ekf_kernels.h"

namespace ekf {

#define EKF_PI 3.14159265358979323846

__device__ __forceinline__ double normalize_radian(double rad)
{
    // Robot.cpp:62-71
    if (rad > EKF_PI) {
        rad = rad - (2.0 * EKF_PI + floor(rad / (2.0 * EKF_PI)) * 2.0 * EKF_PI);
    } else if (rad < -EKF_PI) {
        rad = rad + (2.0 * EKF_PI + floor(fabs(rad) / (2.0 * EKF_PI)) * 2.0 * EKF_PI);
    }
    return rad;
}

// gsl_linalg_LU_decomp + LU_invert on 2x2 (Robot.cpp:449-457); returns false when singular
// (GSL_EDOM), leaving Si untouched.
__device__ __forceinline__ bool lu_invert2(const double S[4], double Si[4])
{
    double a0 = S[0], a1 = S[1], a2 = S[2], a3 = S[3];
    int p0 = 0, p1 = 1;
    if (fabs(a2) > fabs(a0)) {
        double t0 = a0, t1 = a1;
        a0 = a2; a1 = a3;
        a2 = t0; a3 = t1;
        p0 = 1; p1 = 0;
    }
    if (a0 != 0.0) {
        const double l = a2 / a0;
        a2 = l;
        a3 -= l * a1;
    }
    if (a0 == 0.0 || a3 == 0.0) return false;
#pragma unroll
    for (int c = 0; c < 2; c++) {
        double b0 = (p0 == c) ? 1.0 : 0.0;
        double b1 = (p1 == c) ? 1.0 : 0.0;
        b1 = b1 - a2 * b0;
        const double x1 = b1 / a3;
        const double x0 = (b0 - a1 * x1) / a0;
        Si[c] = x0;
        Si[2 + c] = x1;
    }
    return true;
}

template <typename T>
__device__ __forceinline__ double ll_get(const T* P, int i, int j, int nb)
{
    return (double)P[ll_offset<T>(i, j, nb)];
}

template <typename T>
__device__ __forceinline__ void ll_store_sym(T* P, int i, int j, int nb, double v)
{
    P[ll_offset<T>(i, j, nb)] = (T)v;
    if ((i >> 5) == (j >> 5) && i != j) P[ll_offset<T>(j, i, nb)] = (T)v;
}

struct Cand {
    double S[4];
    double Si[4];
    double v[2];
    double h10, h11, h1l;
    bool pass;
    bool singular;
};

// One association candidate (line z vs saved landmark j), Robot.cpp:367-489, on the 5×5
// block {0,1,2, 3+2j, 4+2j} of the current P (robot strip + diagonal cache).
__device__ __forceinline__ void eval_candidate(int j, const double* Rs, int n, const double* D,
                                               int Nc, const double* y, const double xp[3],
                                               double za, double zr, const double Rm[4],
                                               double gate, Cand& c)
{
    const int l0 = 3 + 2 * j, l1 = l0 + 1;
    const double ma = y[l0], mr = y[l1];
    double sn, cs;
    sincos(ma, &sn, &cs);
    c.h10 = -cs;
    c.h11 = -sn;
    c.h1l = xp[0] * sn - xp[1] * cs;
    // P rows: P[a][b] for a,b<3 from the strip; P[a][L] = Rs[a][L]; P[L][a] = Rs[a][L];
    // P[L][L'] from the diagonal cache.
    const double p00 = Rs[0], p01 = Rs[1], p02 = Rs[2];
    const double p10 = Rs[n + 0], p11 = Rs[n + 1], p12 = Rs[n + 2];
    const double p20 = Rs[2 * n + 0], p21 = Rs[2 * n + 1], p22 = Rs[2 * n + 2];
    const double p0a = Rs[l0], p1a = Rs[n + l0], p2a = Rs[2 * n + l0];
    const double p0b = Rs[l1], p1b = Rs[n + l1], p2b = Rs[2 * n + l1];
    const double daa = D[j], dab = D[Nc + j], dba = D[2 * Nc + j], dbb = D[3 * Nc + j];
    // hp0 = hr0·P5 with hr0 = (0,0,-1,1,0); hp1 = hr1·P5 with hr1 = (h10,h11,0,h1l,1)
    const double hp0_0 = -p20 + p0a, hp0_1 = -p21 + p1a, hp0_2 = -p22 + p2a;
    const double hp0_3 = -p2a + daa, hp0_4 = -p2b + dab;
    const double hp1_0 = c.h10 * p00 + c.h11 * p10 + c.h1l * p0a + p0b;
    const double hp1_1 = c.h10 * p01 + c.h11 * p11 + c.h1l * p1a + p1b;
    const double hp1_2 = c.h10 * p02 + c.h11 * p12 + c.h1l * p2a + p2b;
    const double hp1_3 = c.h10 * p0a + c.h11 * p1a + c.h1l * daa + dba;
    const double hp1_4 = c.h10 * p0b + c.h11 * p1b + c.h1l * dab + dbb;
    (void)hp0_4;
    c.S[0] = -hp0_2 + hp0_3 + Rm[0];
    c.S[1] = hp0_0 * c.h10 + hp0_1 * c.h11 + hp0_3 * c.h1l + hp0_4 + Rm[1];
    c.S[2] = -hp1_2 + hp1_3 + Rm[2];
    c.S[3] = hp1_0 * c.h10 + hp1_1 * c.h11 + hp1_3 * c.h1l + hp1_4 + Rm[3];
    // h (Robot.cpp:423-426), S⁻¹ (Robot.cpp:443-457), v and its 2π fold (Robot.cpp:465-475)
    double h0 = normalize_radian(ma - xp[2]);
    const double h1 = mr - (xp[0] * cs + xp[1] * sn);
    c.Si[0] = c.Si[1] = c.Si[2] = c.Si[3] = 0.0;
    c.singular = !lu_invert2(c.S, c.Si);
    double v0 = za - h0;
    const double v1 = zr - h1;
    if (fabs(v0 - 2.0 * EKF_PI) < fabs(v0)) v0 -= 2.0 * EKF_PI;
    else if (fabs(v0 + 2.0 * EKF_PI) < fabs(v0)) v0 += 2.0 * EKF_PI;
    c.v[0] = v0;
    c.v[1] = v1;
    // vᵀ·S⁻¹·v (Robot.cpp:479-486); gate (Robot.cpp:489): NaN passes, as in the reference
    const double vs0 = v0 * c.Si[0] + v1 * c.Si[2];
    const double vs1 = v0 * c.Si[1] + v1 * c.Si[3];
    const double d2 = vs0 * v0 + vs1 * v1;
    c.pass = !(sqrt(fabs(d2)) > gate);
}

__device__ __forceinline__ int wave_min(int v)
{
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) v = min(v, __shfl_xor(v, off, 64));
    return v;
}

// --------------------------------------------------------------------------------------
// 1. association + gain chain
// --------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(SCAN_THREADS) void scan_kernel(ScanParams p)
{
    const Dims d = p.d;
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = d.n, N = d.N;
    double* Rs = p.Rs + (size_t)e * 3 * n;
    double* y = p.y + (size_t)e * n;
    double* D = p.D + (size_t)e * 4 * N;
    double* Ust = p.Ust + (size_t)e * d.max_lines * 2 * n;
    double* Vst = p.Vst + (size_t)e * d.max_lines * 2 * n;
    const size_t opstride = (size_t)d.nb * 64 * (d.kmax / 2);
    T* Uop = reinterpret_cast<T*>(p.Uop) + (size_t)e * opstride;
    T* Vop = reinterpret_cast<T*>(p.Vop) + (size_t)e * opstride;
    const T* Pll = reinterpret_cast<const T*>(p.Pll) + (size_t)e * d.ntiles * TILE_ELEMS;
    int* res = p.res + (size_t)e * RES_STRIDE;

    __shared__ double sh_xp[3];
    __shared__ double sh_u[6];     // U_t rows 0..2 (k = 0, 1)
    __shared__ int sh_red[SCAN_THREADS / 64];
    extern __shared__ unsigned int sh_matched[];  // bitmask over N landmarks

    double xp[3];
    if (p.phase & PHASE_PREDICT) {
        // Robot.cpp:130-148 (SIMULATIONOFF == true: `rot` unused)
        const double x0 = p.pose[3 * e + 0], y0 = p.pose[3 * e + 1], t0 = p.pose[3 * e + 2];
        const double* enc = p.enc + 3 * e;
        const double u2 = t0 - enc[2];
        const double dx = x0 - enc[0], dy = y0 - enc[1];
        const double u0 = sqrt(dx * dx + dy * dy);
        xp[0] = x0 + u0 * cos(t0 + u2 / 2.0);
        xp[1] = y0 + u0 * sin(t0 + u2 / 2.0);
        xp[2] = t0 + u2;
        const double c = u2 / 2.0 + t0;
        double sc, cc;
        sincos(c, &sc, &cc);
        const double F3[9] = {1, 0, -u0 * sc, 0, 1, u0 * cc, 0, 0, 1};
        // robot–landmark block: rows 0..2 of Fx·P (Robot.cpp:242); columns b >= 3
        for (int b = 3 + tid; b < n; b += SCAN_THREADS) {
            const double r0 = Rs[b], r1 = Rs[n + b], r2 = Rs[2 * n + b];
            Rs[b] = F3[0] * r0 + F3[1] * r1 + F3[2] * r2;
            Rs[n + b] = F3[3] * r0 + F3[4] * r1 + F3[5] * r2;
            Rs[2 * n + b] = F3[6] * r0 + F3[7] * r1 + F3[8] * r2;
        }
        if (tid == 0) {
            // 3×3 block: F3·P33·F3ᵀ + Fu3·Q·Fu3ᵀ (Robot.cpp:178-258)
            const double Fu3[9] = {cc, 0, -u0 * sc / 2.0, sc, 1, u0 * cc / 2.0, 0, 0, 1};
            const double qs = (-1.0 / (1 + fabs(u0)) + 1);
            const double Q[9] = {p.enc_noise * qs, 0, 0, 0, 2 * p.enc_noise * qs, 0, 0, 0,
                                 p.enc_noise * qs};
            double P33[9], FP[9], FuQ[9];
            for (int a = 0; a < 9; a++) P33[a] = Rs[(a / 3) * n + (a % 3)];
            for (int a = 0; a < 3; a++)
                for (int b = 0; b < 3; b++) {
                    double s = 0.0, t = 0.0;
                    for (int k = 0; k < 3; k++) {
                        s += F3[a * 3 + k] * P33[k * 3 + b];
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
                    Rs[a * n + b] = s + t;
                }
            if (!(p.phase & PHASE_UPDATE)) {
                p.xpre[3 * e + 0] = xp[0];
                p.xpre[3 * e + 1] = xp[1];
                p.xpre[3 * e + 2] = xp[2];
            }
        }
        __syncthreads();
    } else {
        xp[0] = p.xpre[3 * e + 0];
        xp[1] = p.xpre[3 * e + 1];
        xp[2] = p.xpre[3 * e + 2];
    }
    if (!(p.phase & PHASE_UPDATE)) return;

    // ---------------- association / update (Robot.cpp:288-904) ----------------
    int L = p.nlines[e];
    L = L < 0 ? 0 : (L > d.max_lines ? d.max_lines : L);
    const int s = p.saved[e];
    const ekf_line* lines = p.lines + (size_t)e * d.max_lines;

    // diagonal cache of P_ll and matched bitmask
    for (int j = tid; j < s; j += SCAN_THREADS) {
        D[j] = ll_get(Pll, 2 * j, 2 * j, d.nb);
        D[N + j] = ll_get(Pll, 2 * j, 2 * j + 1, d.nb);
        D[2 * N + j] = ll_get(Pll, 2 * j + 1, 2 * j, d.nb);
        D[3 * N + j] = ll_get(Pll, 2 * j + 1, 2 * j + 1, d.nb);
    }
    const int nwords = (N + 31) / 32;
    for (int w = tid; w < nwords; w += SCAN_THREADS) sh_matched[w] = 0u;
    __syncthreads();

    int m = 0, nextra = 0, status = 0;
    for (int i = 0; i < L; ++i) {
        const ekf_line ln = lines[i];
        double Rm[4] = {0, 0, 0, 0};
        if (p.r_mode == 1) {
            if (i < 4) Rm[i] = ln.R[3];   // Robot.cpp:302-304 as written (zero-init stack)
        } else {
            Rm[0] = ln.R[0]; Rm[1] = ln.R[1]; Rm[2] = ln.R[2]; Rm[3] = ln.R[3];
        }
        // parallel gating, first passing unmatched j wins (Robot.cpp:313-498)
        int best = 0x7fffffff;
        bool sing = false;
        for (int j = tid; j < s; j += SCAN_THREADS) {
            if (sh_matched[j >> 5] & (1u << (j & 31))) continue;
            Cand c;
            eval_candidate(j, Rs, n, D, N, y, xp, ln.alpha, ln.r, Rm, p.gate, c);
            sing |= c.singular;
            if (c.pass) { best = j; break; }
        }
        if (sing) status |= EKF_ST_SINGULAR;
        best = wave_min(best);
        if ((tid & 63) == 0) sh_red[tid >> 6] = best;
        __syncthreads();
        int jstar = sh_red[0];
#pragma unroll
        for (int w = 1; w < SCAN_THREADS / 64; w++) jstar = min(jstar, sh_red[w]);
        if (jstar == 0x7fffffff) {
            // no match (or s == 0): the line goes to extraLines (Robot.cpp:308-310, 492-496)
            if (tid == 0) {
                res[RES_MATCH + i] = -1;
                res[RES_EXTRA + nextra] = i;
            }
            nextra++;
            __syncthreads();   // sh_red reuse
            continue;
        }
        // ---- match (Robot.cpp:500-641) in deferred low-rank form ----
        Cand c;
        eval_candidate(jstar, Rs, n, D, N, y, xp, ln.alpha, ln.r, Rm, p.gate, c);
        const int t = m;
        const int l0 = 3 + 2 * jstar, l1 = l0 + 1;
        if (p.r_mode == 1 && (i == 1 || i == 2)) status |= EKF_ST_NSYM;
        double* Ut0 = Ust + (size_t)(2 * t) * n;
        double* Ut1 = Ut0 + n;
        double* Vt0 = Vst + (size_t)(2 * t) * n;
        double* Vt1 = Vt0 + n;
        for (int b = tid; b < n; b += SCAN_THREADS) {
            double pb0, pb1, pb2, pba, pbb;
            if (b < 3) {
                pb0 = Rs[b * n + 0]; pb1 = Rs[b * n + 1]; pb2 = Rs[b * n + 2];
                pba = Rs[b * n + l0]; pbb = Rs[b * n + l1];
            } else {
                pb0 = Rs[b]; pb1 = Rs[n + b]; pb2 = Rs[2 * n + b];
                pba = ll_get(Pll, b - 3, l0 - 3, d.nb);
                pbb = ll_get(Pll, b - 3, l1 - 3, d.nb);
                for (int q = 0; q < t; q++) {   // earlier matches of this scan, in order
                    const double* Uq = Ust + (size_t)(2 * q) * n;
                    const double* Vq = Vst + (size_t)(2 * q) * n;
                    pba -= Uq[b] * Vq[l0] + Uq[n + b] * Vq[n + l0];
                    pbb -= Uq[b] * Vq[l1] + Uq[n + b] * Vq[n + l1];
                }
            }
            // W = P·Hᵀ (Robot.cpp:522), K = W·S⁻¹ (:526), U = K·S (:560)
            const double w0 = -pb2 + pba;
            const double w1 = c.h10 * pb0 + c.h11 * pb1 + c.h1l * pba + pbb;
            const double k0 = w0 * c.Si[0] + w1 * c.Si[2];
            const double k1 = w0 * c.Si[1] + w1 * c.Si[3];
            const double u0 = k0 * c.S[0] + k1 * c.S[2];
            const double u1 = k0 * c.S[1] + k1 * c.S[3];
            Ut0[b] = u0; Ut1[b] = u1;
            Vt0[b] = k0; Vt1[b] = k1;
            // y = x_pre ⊕ y_landmarks + K·v (Robot.cpp:579-592)
            const double yb = (b < 3) ? xp[b] : y[b];
            y[b] = yb + (k0 * c.v[0] + k1 * c.v[1]);
            if (b < 3) {
                sh_u[b] = u0;
                sh_u[3 + b] = u1;
            } else {
                const int lr = b - 3;
                if constexpr (sizeof(T) == 4) {
                    Uop[op_index_f32(lr, 2 * t, d.kmax)] = (T)(-u0);
                    Uop[op_index_f32(lr, 2 * t + 1, d.kmax)] = (T)(-u1);
                    Vop[op_index_f32(lr, 2 * t, d.kmax)] = (T)k0;
                    Vop[op_index_f32(lr, 2 * t + 1, d.kmax)] = (T)k1;
                } else {
                    Uop[op_index_f64(lr, 2 * t, d.kmax)] = (T)(-u0);
                    Uop[op_index_f64(lr, 2 * t + 1, d.kmax)] = (T)(-u1);
                    Vop[op_index_f64(lr, 2 * t, d.kmax)] = (T)k0;
                    Vop[op_index_f64(lr, 2 * t + 1, d.kmax)] = (T)k1;
                }
            }
        }
        __syncthreads();
        // eager downdate of the robot strip and the diagonal cache (Robot.cpp:568)
        for (int b = tid; b < n; b += SCAN_THREADS) {
            const double k0 = Vt0[b], k1 = Vt1[b];
            Rs[b] -= sh_u[0] * k0 + sh_u[3] * k1;
            Rs[n + b] -= sh_u[1] * k0 + sh_u[4] * k1;
            Rs[2 * n + b] -= sh_u[2] * k0 + sh_u[5] * k1;
        }
        for (int j = tid; j < s; j += SCAN_THREADS) {
            const int a = 3 + 2 * j, bb = a + 1;
            const double ua0 = Ut0[a], ua1 = Ut1[a], ub0 = Ut0[bb], ub1 = Ut1[bb];
            const double va0 = Vt0[a], va1 = Vt1[a], vb0 = Vt0[bb], vb1 = Vt1[bb];
            D[j] -= ua0 * va0 + ua1 * va1;
            D[N + j] -= ua0 * vb0 + ua1 * vb1;
            D[2 * N + j] -= ub0 * va0 + ub1 * va1;
            D[3 * N + j] -= ub0 * vb0 + ub1 * vb1;
        }
        if (tid == 0) {
            y[2] = normalize_radian(y[2]);     // Robot.cpp:596
            sh_xp[0] = y[0];
            sh_xp[1] = y[1];
            sh_xp[2] = y[2];
            sh_matched[jstar >> 5] |= (1u << (jstar & 31));
            res[RES_MATCH + i] = jstar;
        }
        __syncthreads();
        xp[0] = sh_xp[0];
        xp[1] = sh_xp[1];
        xp[2] = sh_xp[2];
        m++;
    }

    // ---------------- commit (Robot.cpp:702-716, 893-904) ----------------
    const int added = min(nextra, N - s);
    const int reset = (s + added > N - p.reset_margin) ? 1 : 0;
    if (tid == 0) {
        if (L == 0 || m == 0) {
            y[0] = xp[0];
            y[1] = xp[1];
            y[2] = xp[2];
            p.pose[3 * e + 0] = xp[0];
            p.pose[3 * e + 1] = xp[1];
            p.pose[3 * e + 2] = normalize_radian(xp[2]);
        } else {
            p.pose[3 * e + 0] = y[0];
            p.pose[3 * e + 1] = y[1];
            p.pose[3 * e + 2] = y[2];
        }
        if (nextra > added) status |= EKF_ST_CAP;
        res[RES_M] = m;
        res[RES_NEXTRA] = nextra;
        res[RES_SAVED_IN] = s;
        res[RES_SAVED] = reset ? 0 : s + added;
        res[RES_RESET] = reset;
        res[RES_STATUS] = status;
        res[RES_NLINES] = L;
        res[RES_KSTEPS] = (sizeof(T) == 4) ? m : (m + 1) / 2;
        if (reset) p.saved[e] = 0;
    }
    // f64 operands: zero the odd tail column pair of the last 4-wide k-step
    if (sizeof(T) == 8 && (m & 1)) {
        for (int lr = tid; lr < d.M; lr += SCAN_THREADS) {
            Uop[op_index_f64(lr, 2 * m, d.kmax)] = (T)0;
            Uop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (T)0;
            Vop[op_index_f64(lr, 2 * m, d.kmax)] = (T)0;
            Vop[op_index_f64(lr, 2 * m + 1, d.kmax)] = (T)0;
        }
    }
    if (reset) {
        for (int b = 3 + tid; b < n; b += SCAN_THREADS) {
            y[b] = 0.0;
            Rs[b] = 0.0;
            Rs[n + b] = 0.0;
            Rs[2 * n + b] = 0.0;
        }
    }
}

// --------------------------------------------------------------------------------------
// 2. packed rank-2m covariance downdate on MFMA
// --------------------------------------------------------------------------------------
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef double f64x4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(DD_THREADS) void downdate_f32_kernel(DowndateParams p)
{
    const Dims d = p.d;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (DD_THREADS / 64);
    const int64_t total = (int64_t)p.E * d.ntiles;
    const int kh = d.kmax / 2;   // operand floats per lane per row block
    for (int64_t g = (int64_t)blockIdx.x * (DD_THREADS / 64) + (threadIdx.x >> 6); g < total;
         g += nwaves) {
        const int e = (int)(g / d.ntiles);
        const int64_t t = g - (int64_t)e * d.ntiles;
        const int* res = p.res + (size_t)e * RES_STRIDE;
        const int ks = res[RES_KSTEPS];
        const int reset = res[RES_RESET];
        if (!reset && ks == 0) continue;
        float* tile = reinterpret_cast<float*>(p.Pll) + ((size_t)e * d.ntiles + t) * TILE_ELEMS;
        f32x4* tv = reinterpret_cast<f32x4*>(tile) + lane;
        if (reset) {
            const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int q = 0; q < 4; q++) __builtin_nontemporal_store(z, tv + q * 64);
            continue;
        }
        const int2 rc = p.tile_rc[t];
        f32x16 acc;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const f32x4 v = __builtin_nontemporal_load(tv + q * 64);
            acc[4 * q + 0] = v[0];
            acc[4 * q + 1] = v[1];
            acc[4 * q + 2] = v[2];
            acc[4 * q + 3] = v[3];
        }
        const size_t opbase = (size_t)e * d.nb * 64 * kh;
        const float* A = reinterpret_cast<const float*>(p.Uop) + opbase +
                         ((size_t)rc.x * 64 + lane) * kh;
        const float* B = reinterpret_cast<const float*>(p.Vop) + opbase +
                         ((size_t)rc.y * 64 + lane) * kh;
        for (int s0 = 0; s0 < ks; s0 += 8) {
            const f32x4 a0 = *reinterpret_cast<const f32x4*>(A + s0);
            const f32x4 a1 = *reinterpret_cast<const f32x4*>(A + s0 + 4);
            const f32x4 b0 = *reinterpret_cast<const f32x4*>(B + s0);
            const f32x4 b1 = *reinterpret_cast<const f32x4*>(B + s0 + 4);
            const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
            for (int s = 0; s < 8; s++)
                if (s0 + s < ks) acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s], bv[s], acc, 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const f32x4 v = {acc[4 * q + 0], acc[4 * q + 1], acc[4 * q + 2], acc[4 * q + 3]};
            __builtin_nontemporal_store(v, tv + q * 64);
        }
    }
}

__global__ __launch_bounds__(DD_THREADS) void downdate_f64_kernel(DowndateParams p)
{
    const Dims d = p.d;
    const int lane = threadIdx.x & 63;
    const int64_t nwaves = (int64_t)gridDim.x * (DD_THREADS / 64);
    const int64_t total = (int64_t)p.E * d.ntiles;
    const int kh = d.kmax / 2;   // doubles per lane per row block (2 halves × kmax/4)
    const int kq = d.kmax / 4;
    for (int64_t g = (int64_t)blockIdx.x * (DD_THREADS / 64) + (threadIdx.x >> 6); g < total;
         g += nwaves) {
        const int e = (int)(g / d.ntiles);
        const int64_t t = g - (int64_t)e * d.ntiles;
        const int* res = p.res + (size_t)e * RES_STRIDE;
        const int ks = res[RES_KSTEPS];
        const int reset = res[RES_RESET];
        if (!reset && ks == 0) continue;
        double* tile = reinterpret_cast<double*>(p.Pll) + ((size_t)e * d.ntiles + t) * TILE_ELEMS;
        f64x2* tv = reinterpret_cast<f64x2*>(tile) + 2 * lane;
        if (reset) {
            const f64x2 z = {0.0, 0.0};
#pragma unroll
            for (int q = 0; q < 4; q++) {
                __builtin_nontemporal_store(z, tv + q * 128);
                __builtin_nontemporal_store(z, tv + q * 128 + 1);
            }
            continue;
        }
        const int2 rc = p.tile_rc[t];
        f64x4 acc[4];
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const f64x2 v0 = __builtin_nontemporal_load(tv + q * 128);
            const f64x2 v1 = __builtin_nontemporal_load(tv + q * 128 + 1);
            acc[q][0] = v0[0];
            acc[q][1] = v0[1];
            acc[q][2] = v1[0];
            acc[q][3] = v1[1];
        }
        const size_t opbase = (size_t)e * d.nb * 64 * kh;
        const double* A = reinterpret_cast<const double*>(p.Uop) + opbase +
                          ((size_t)rc.x * 64 + lane) * kh;
        const double* B = reinterpret_cast<const double*>(p.Vop) + opbase +
                          ((size_t)rc.y * 64 + lane) * kh;
        for (int s = 0; s < ks; s++) {
            const double a0 = A[s], a1 = A[kq + s];
            const double b0 = B[s], b1 = B[kq + s];
            acc[0] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b0, acc[0], 0, 0, 0);
            acc[1] = __builtin_amdgcn_mfma_f64_16x16x4f64(a0, b1, acc[1], 0, 0, 0);
            acc[2] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b0, acc[2], 0, 0, 0);
            acc[3] = __builtin_amdgcn_mfma_f64_16x16x4f64(a1, b1, acc[3], 0, 0, 0);
        }
#pragma unroll
        for (int q = 0; q < 4; q++) {
            const f64x2 v0 = {acc[q][0], acc[q][1]};
            const f64x2 v1 = {acc[q][2], acc[q][3]};
            __builtin_nontemporal_store(v0, tv + q * 128);
            __builtin_nontemporal_store(v1, tv + q * 128 + 1);
        }
    }
}

// --------------------------------------------------------------------------------------
// 3. landmark augmentation (Robot.cpp:776-866)
// --------------------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(SCAN_THREADS) void augment_kernel(ScanParams p)
{
    const Dims d = p.d;
    const int e = blockIdx.x;
    const int tid = threadIdx.x;
    const int n = d.n, N = d.N;
    int* res = p.res + (size_t)e * RES_STRIDE;
    const int nextra = res[RES_NEXTRA];
    if (res[RES_RESET] || nextra == 0) return;
    double* Rs = p.Rs + (size_t)e * 3 * n;
    double* y = p.y + (size_t)e * n;
    T* Pll = reinterpret_cast<T*>(p.Pll) + (size_t)e * d.ntiles * TILE_ELEMS;
    const ekf_line* lines = p.lines + (size_t)e * d.max_lines;
    const double px = p.pose[3 * e + 0], py = p.pose[3 * e + 1], pt = p.pose[3 * e + 2];
    int s = res[RES_SAVED_IN];
    for (int q = 0; q < nextra; q++) {
        if (s >= N) break;   // capacity (flagged by scan_kernel)
        const ekf_line ln = lines[res[RES_EXTRA + q]];
        double alfa = ln.alpha;
        const double r = ln.r + (px * cos(alfa) + py * sin(alfa));
        alfa += pt;
        double sa, ca;
        sincos(alfa, &sa, &ca);
        const double y0 = y[0], y1 = y[1];
        const double gl10 = y1 * ca - y0 * sa;
        const int l0 = 3 + 2 * s;
        // P_ll = Gx·Prr·Gxᵀ + Gl·R·Glᵀ (Robot.cpp:813-847); Gx = [[0,0,1],[ca,sa,0]],
        // Gl = [[1,0],[gl10,1]]
        double Prr[9];
        for (int a = 0; a < 9; a++) Prr[a] = Rs[(a / 3) * n + (a % 3)];
        const double Gx[6] = {0, 0, 1, ca, sa, 0};
        double GP[6];
        for (int a = 0; a < 2; a++)
            for (int b = 0; b < 3; b++) {
                double acc = 0.0;
                for (int k = 0; k < 3; k++) acc += Gx[a * 3 + k] * Prr[k * 3 + b];
                GP[a * 3 + b] = acc;
            }
        const double Gl[4] = {1.0, 0, gl10, 1};
        double GlR[4];
        for (int a = 0; a < 2; a++)
            for (int b = 0; b < 2; b++)
                GlR[a * 2 + b] = Gl[a * 2 + 0] * ln.R[0 * 2 + b] + Gl[a * 2 + 1] * ln.R[1 * 2 + b];
        double Pnew[4];
        for (int a = 0; a < 2; a++)
            for (int b = 0; b < 2; b++) {
                double g = 0.0;
                for (int k = 0; k < 3; k++) g += GP[a * 3 + k] * Gx[b * 3 + k];
                const double h = GlR[a * 2 + 0] * Gl[b * 2 + 0] + GlR[a * 2 + 1] * Gl[b * 2 + 1];
                Pnew[a * 2 + b] = g + h;
            }
        // P[l0:l0+2, 0:l0] = Gx·P[0:3, 0:l0] and its transpose (Robot.cpp:852-862)
        for (int c = tid; c < l0; c += SCAN_THREADS) {
            const double v0 = Rs[2 * n + c];
            const double v1 = ca * Rs[c] + sa * Rs[n + c];
            if (c >= 3) {
                ll_store_sym(Pll, l0 - 3, c - 3, d.nb, v0);
                ll_store_sym(Pll, l0 - 2, c - 3, d.nb, v1);
            }
        }
        __syncthreads();
        if (tid < 3) {
            const int c = tid;
            const double v0 = Rs[2 * n + c];
            const double v1 = ca * Rs[c] + sa * Rs[n + c];
            Rs[c * n + l0] = v0;
            Rs[c * n + l0 + 1] = v1;
        }
        if (tid == 0) {
            const int i0 = l0 - 3;
            Pll[ll_offset<T>(i0, i0, d.nb)] = (T)Pnew[0];
            Pll[ll_offset<T>(i0, i0 + 1, d.nb)] = (T)Pnew[1];
            Pll[ll_offset<T>(i0 + 1, i0, d.nb)] = (T)Pnew[2];
            Pll[ll_offset<T>(i0 + 1, i0 + 1, d.nb)] = (T)Pnew[3];
            y[l0] = normalize_radian(alfa);
            y[l0 + 1] = r;
        }
        __syncthreads();
        s++;
    }
    if (tid == 0) {
        p.saved[e] = s;
        res[RES_SAVED] = s;
    }
}

// --------------------------------------------------------------------------------------
// state transfer / initialisation
// --------------------------------------------------------------------------------------
template <typename T>
__global__ void pack_kernel(Dims d, const double* __restrict__ Pfull, T* __restrict__ Pll,
                            double* __restrict__ Rs, const int2* __restrict__ tile_rc)
{
    const int64_t total = d.ntiles * TILE_ELEMS;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = g / TILE_ELEMS;
        const int rem = (int)(g - t * TILE_ELEMS);
        // invert the intra-tile layout by brute force over (r, c): map rem → (r, c)
        int r, c;
        if (sizeof(T) == 4) {
            const int q = rem & 3, lane = (rem >> 2) & 63, grp = rem >> 8;
            c = lane & 31;
            r = q + 4 * (lane >> 5) + 8 * grp;
        } else {
            const int reg = rem & 3, lane = (rem >> 2) & 63, blk = rem >> 8;
            c = (lane & 15) + 16 * (blk & 1);
            r = (lane >> 4) + 4 * reg + 16 * (blk >> 1);
        }
        const int2 rc = tile_rc[t];
        const int i = rc.x * TILE + r, j = rc.y * TILE + c;
        double v = 0.0;
        if (i < d.M && j < d.M) v = Pfull[(size_t)(3 + i) * d.n + (3 + j)];
        Pll[g] = (T)v;
    }
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < 3 * (int64_t)d.n;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(g / d.n), b = (int)(g % d.n);
        Rs[g] = Pfull[(size_t)a * d.n + b];
    }
}

template <typename T>
__global__ void unpack_kernel(Dims d, double* __restrict__ Pfull, const T* __restrict__ Pll,
                              const double* __restrict__ Rs)
{
    const int64_t total = (int64_t)d.n * d.n;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int a = (int)(g / d.n), b = (int)(g % d.n);
        double v;
        if (a < 3) v = Rs[(size_t)a * d.n + b];
        else if (b < 3) v = Rs[(size_t)b * d.n + a];
        else v = (double)Pll[ll_offset<T>(a - 3, b - 3, d.nb)];
        Pfull[g] = v;
    }
}

template <typename T>
__global__ void lowrank_kernel(Dims d, const double* __restrict__ diag,
                               const double* __restrict__ U, int rank, T* __restrict__ Pll,
                               double* __restrict__ Rs, const int2* __restrict__ tile_rc)
{
    const int64_t total = d.ntiles * TILE_ELEMS;
    for (int64_t g = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; g < total;
         g += (int64_t)gridDim.x * blockDim.x) {
        const int64_t t = g / TILE_ELEMS;
        const int rem = (int)(g - t * TILE_ELEMS);
        int r, c;
        if (sizeof(T) == 4) {
            const int q = rem & 3, lane = (rem >> 2) & 63, grp = rem >> 8;
            c = lane & 31;
            r = q + 4 * (lane >> 5) + 8 * grp;
        } else {
            const int reg = rem & 3, lane = (rem >> 2) & 63, blk = rem >> 8;
            c = (lane & 15) + 16 * (blk & 1);
            r = (lane >> 4) + 4 * reg + 16 * (blk >> 1);
        }
        const int2 rc = tile_rc[t];
        const int i = rc.x * TILE + r, j = rc.y * TILE + c;
        double v = 0.0;
        if (i < d.M && j < d.M) {
            const double* ui = U + (size_t)(3 + i) * rank;
            const double* uj = U + (size_t)(3 + j) * rank;
            for (int k = 0; k < rank; k++) v += ui[k] * uj[k];
            if (i == j) v += diag[3 + i];
        }
        Pll[g] = (T)v;
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

// --------------------------------------------------------------------------------------
// launchers
// --------------------------------------------------------------------------------------
hipError_t launch_scan(const ScanParams& p, int precision, hipStream_t st)
{
    const size_t lds = sizeof(unsigned int) * (size_t)((p.d.N + 31) / 32);
    if (precision == 0)
        hipLaunchKernelGGL(scan_kernel<double>, dim3(p.E), dim3(SCAN_THREADS), lds, st, p);
    else
        hipLaunchKernelGGL(scan_kernel<float>, dim3(p.E), dim3(SCAN_THREADS), lds, st, p);
    return hipGetLastError();
}

hipError_t launch_downdate(const DowndateParams& p, int precision, int grid, hipStream_t st)
{
    if (precision == 0)
        hipLaunchKernelGGL(downdate_f64_kernel, dim3(grid), dim3(DD_THREADS), 0, st, p);
    else
        hipLaunchKernelGGL(downdate_f32_kernel, dim3(grid), dim3(DD_THREADS), 0, st, p);
    return hipGetLastError();
}

hipError_t launch_augment(const ScanParams& p, int precision, hipStream_t st)
{
    if (precision == 0)
        hipLaunchKernelGGL(augment_kernel<double>, dim3(p.E), dim3(SCAN_THREADS), 0, st, p);
    else
        hipLaunchKernelGGL(augment_kernel<float>, dim3(p.E), dim3(SCAN_THREADS), 0, st, p);
    return hipGetLastError();
}

static int grid_for(int64_t work, int block)
{
    int64_t g = (work + block - 1) / block;
    if (g > 8192) g = 8192;
    if (g < 1) g = 1;
    return (int)g;
}

hipError_t launch_pack(const Dims& d, int precision, const double* Pfull, void* Pll, double* Rs,
                       const int2* tile_rc, hipStream_t st)
{
    const int grid = grid_for(d.ntiles * TILE_ELEMS, 256);
    if (precision == 0)
        hipLaunchKernelGGL(pack_kernel<double>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (double*)Pll, Rs, tile_rc);
    else
        hipLaunchKernelGGL(pack_kernel<float>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (float*)Pll, Rs, tile_rc);
    return hipGetLastError();
}

hipError_t launch_unpack(const Dims& d, int precision, double* Pfull, const void* Pll,
                         const double* Rs, hipStream_t st)
{
    const int grid = grid_for((int64_t)d.n * d.n, 256);
    if (precision == 0)
        hipLaunchKernelGGL(unpack_kernel<double>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (const double*)Pll, Rs);
    else
        hipLaunchKernelGGL(unpack_kernel<float>, dim3(grid), dim3(256), 0, st, d, Pfull,
                           (const float*)Pll, Rs);
    return hipGetLastError();
}

hipError_t launch_lowrank(const Dims& d, int precision, const double* diag, const double* U,
                          int rank, void* Pll, double* Rs, const int2* tile_rc, hipStream_t st)
{
    const int grid = grid_for(d.ntiles * TILE_ELEMS, 256);
    if (precision == 0)
        hipLaunchKernelGGL(lowrank_kernel<double>, dim3(grid), dim3(256), 0, st, d, diag, U,
                           rank, (double*)Pll, Rs, tile_rc);
    else
        hipLaunchKernelGGL(lowrank_kernel<float>, dim3(grid), dim3(256), 0, st, d, diag, U,
                           rank, (float*)Pll, Rs, tile_rc);
    return hipGetLastError();
}

}  // namespace ekf
