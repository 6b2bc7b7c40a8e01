/*
 * ekf_oracle.c — CPU restatement of slam_ros Robot::localize (TEST INFRASTRUCTURE, see header).
 *
 * Every block cites the reference statement it follows (slam_ros/Robot.cpp line numbers).
 * GSL is not available in this image; its semantics are restated from its documented
 * behaviour (gslcblas dgemm loop order, LU with partial pivoting, LU_invert by column
 * solves, singular → GSL_EDOM leaving the output untouched). These are recalled, not
 * verified against a GSL build: any bit-level ordering claim is "parity unpinned".
 */
#include "ekf_oracle.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

/* B1 "fast" baseline on all host cores: built a second time with -fopenmp (libekf_oracle_omp.so,
 * BASELINE.md §2). Every element is still computed by one thread with the same operation order,
 * so the threaded build returns bit-identical results; only the O(n²) loops are split by rows. */
#ifdef _OPENMP
#include <omp.h>
#define ORACLE_PAR_ROWS _Pragma("omp parallel for schedule(static)")
#else
#define ORACLE_PAR_ROWS
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* Robot.h:15-17 */
#define MAHALANOBIS 0.4
#define ENCODERNOISE 0.024

struct oracle_robot {
    int N;          /* LINESIZE */
    int n;          /* SLAMSIZE = 3 + 2N */
    int mode;
    int r_mode;
    int saved;      /* savedLineCount */
    int status;
    double gate_margin; /* min |sqrt(|d²|) − MAHALANOBIS| over the candidates the last localize
                           evaluated (test instrumentation: SURVEY §8d's gate-margin rejection) */
    /* Test instrumentation: where a stored state of relative precision pred_eta could not resolve
     * this restatement's decisions (the conditions the GPU library reports as EKF_ST_PRECISION /
     * EKF_ST_RANGE, computed here from the restatement's own fp64 state): ORACLE_PRED_* bits of
     * the last localize. pred_eta = 0 disables it. */
    double pred_eta;
    double pred_cancel;  /* the cancellation ratio above which an update is predicted (16: 4 bits) */
    int pred;
    double pose[3]; /* xPos, yPos, thetaPos */
    double* P;      /* P_t0, n*n */
    double* y;      /* y, n */
    /* scratch */
    double* P_pre;
    double* tmpA;   /* n*n (faithful: Fx, FxP; fast: unused) */
    double* tmpB;   /* n*n */
    double* W;      /* n*2 */
    double* K;      /* n*2 */
    double* KS;     /* n*2 */
    double* Hs;     /* 2*n */
    double* HP;     /* 2*n */
    int* matched;   /* N */
};

/* ------------------------------------------------------------------------------------ */
/* primitives                                                                            */
/* ------------------------------------------------------------------------------------ */

double oracle_normalize_radian(double rad)
{
    /* Robot.cpp:62-71 */
    if (rad > M_PI) {
        rad = rad - (2.0 * M_PI + floor(rad / (2.0 * M_PI)) * 2.0 * M_PI);
    } else if (rad < -M_PI) {
        rad = rad + (2.0 * M_PI + floor(fabs(rad) / (2.0 * M_PI)) * 2.0 * M_PI);
    }
    return rad;
}

void oracle_dgemm(int transA, int transB, int M, int N, int K, double alpha, const double* A,
                  int lda, const double* B, int ldb, double beta, double* C, int ldc)
{
    /* gslcblas row-major: C := beta*C, then NN / NT / TN loops (NN and TN skip zero A). */
    int i, j, k;
    if (alpha == 0.0 && beta == 1.0) return;
    if (beta == 0.0) {
        for (i = 0; i < M; i++)
            for (j = 0; j < N; j++) C[(size_t)ldc * i + j] = 0.0;
    } else if (beta != 1.0) {
        for (i = 0; i < M; i++)
            for (j = 0; j < N; j++) C[(size_t)ldc * i + j] *= beta;
    }
    if (alpha == 0.0) return;
    if (!transA && !transB) {
        for (k = 0; k < K; k++)
            for (i = 0; i < M; i++) {
                const double temp = alpha * A[(size_t)lda * i + k];
                if (temp != 0.0) {
                    const double* b = B + (size_t)ldb * k;
                    double* c = C + (size_t)ldc * i;
                    for (j = 0; j < N; j++) c[j] += temp * b[j];
                }
            }
    } else if (!transA && transB) {
        for (i = 0; i < M; i++) {
            const double* a = A + (size_t)lda * i;
            for (j = 0; j < N; j++) {
                const double* b = B + (size_t)ldb * j;
                double temp = 0.0;
                for (k = 0; k < K; k++) temp += a[k] * b[k];
                C[(size_t)ldc * i + j] += alpha * temp;
            }
        }
    } else if (transA && !transB) {
        for (k = 0; k < K; k++)
            for (i = 0; i < M; i++) {
                const double temp = alpha * A[(size_t)lda * k + i];
                if (temp != 0.0) {
                    const double* b = B + (size_t)ldb * k;
                    double* c = C + (size_t)ldc * i;
                    for (j = 0; j < N; j++) c[j] += temp * b[j];
                }
            }
    } else {
        for (i = 0; i < M; i++)
            for (j = 0; j < N; j++) {
                double temp = 0.0;
                for (k = 0; k < K; k++) temp += A[(size_t)lda * k + i] * B[(size_t)ldb * j + k];
                C[(size_t)ldc * i + j] += alpha * temp;
            }
    }
}

int oracle_lu_invert2(const double S[4], double Sinv[4])
{
    /* gsl_linalg_LU_decomp (partial pivoting, strict '>' pivot search), Robot.cpp:450 */
    double a[4] = {S[0], S[1], S[2], S[3]};
    int perm[2] = {0, 1};
    if (fabs(a[2]) > fabs(a[0])) {
        double t0 = a[0], t1 = a[1];
        a[0] = a[2]; a[1] = a[3];
        a[2] = t0;   a[3] = t1;
        perm[0] = 1; perm[1] = 0;
    }
    if (a[0] != 0.0) {
        const double l = a[2] / a[0];
        a[2] = l;
        a[3] -= l * a[1];
    }
    /* gsl_linalg_LU_invert, Robot.cpp:454: singular U → GSL_EDOM, output untouched */
    if (a[0] == 0.0 || a[3] == 0.0) return 1;
    for (int c = 0; c < 2; c++) {
        /* b = P·e_c ; forward (unit L) ; backward (U) */
        double b0 = (perm[0] == c) ? 1.0 : 0.0;
        double b1 = (perm[1] == c) ? 1.0 : 0.0;
        b1 = b1 - a[2] * b0;
        const double x1 = b1 / a[3];
        const double x0 = (b0 - a[1] * x1) / a[0];
        Sinv[0 * 2 + c] = x0;
        Sinv[1 * 2 + c] = x1;
    }
    return 0;
}

/* ------------------------------------------------------------------------------------ */
/* object                                                                                */
/* ------------------------------------------------------------------------------------ */

oracle_robot* oracle_create(int capacity, double x, double y, double theta, int mode, int r_mode)
{
    if (capacity < 1) return NULL;
    oracle_robot* o = (oracle_robot*)calloc(1, sizeof(*o));
    if (!o) return NULL;
    o->N = capacity;
    o->n = 3 + 2 * capacity;
    o->mode = mode;
    o->r_mode = r_mode;
    const size_t n = (size_t)o->n;
    o->P = (double*)calloc(n * n, sizeof(double));
    o->y = (double*)calloc(n, sizeof(double));
    o->P_pre = (double*)calloc(n * n, sizeof(double));
    if (mode == ORACLE_FAITHFUL) {
        o->tmpA = (double*)calloc(n * n, sizeof(double));
        o->tmpB = (double*)calloc(n * n, sizeof(double));
    }
    o->W = (double*)calloc(n * 2, sizeof(double));
    o->K = (double*)calloc(n * 2, sizeof(double));
    o->KS = (double*)calloc(n * 2, sizeof(double));
    o->Hs = (double*)calloc(n * 2, sizeof(double));
    o->HP = (double*)calloc(n * 2, sizeof(double));
    o->matched = (int*)calloc((size_t)capacity, sizeof(int));
    if (!o->P || !o->y || !o->P_pre || !o->W || !o->K || !o->KS || !o->Hs || !o->HP ||
        !o->matched || (mode == ORACLE_FAITHFUL && (!o->tmpA || !o->tmpB))) {
        oracle_destroy(o);
        return NULL;
    }
    /* Robot.cpp:22-30 */
    o->pose[0] = x;
    o->pose[1] = y;
    o->pose[2] = theta;
    o->P[0 * n + 0] = 0.05;
    o->P[1 * n + 1] = 0.05;
    o->P[2 * n + 2] = 0.0;
    o->pred_eta = 0.0;
    o->pred_cancel = 16.0;
    o->pred = 0;
    return o;
}

void oracle_destroy(oracle_robot* o)
{
    if (!o) return;
    free(o->P); free(o->y); free(o->P_pre); free(o->tmpA); free(o->tmpB);
    free(o->W); free(o->K); free(o->KS); free(o->Hs); free(o->HP); free(o->matched);
    free(o);
}

int oracle_n(const oracle_robot* o) { return o->n; }
int oracle_capacity(const oracle_robot* o) { return o->N; }
int oracle_saved(const oracle_robot* o) { return o->saved; }
int oracle_status(const oracle_robot* o) { return o->status; }
double oracle_gate_margin(const oracle_robot* o) { return o->gate_margin; }
void oracle_set_pred(oracle_robot* o, double eta, double cancel)
{
    o->pred_eta = eta;
    o->pred_cancel = cancel;
}
int oracle_pred_flags(const oracle_robot* o) { return o->pred; }
int oracle_threads(void)
{
#ifdef _OPENMP
    int t = 1;
#pragma omp parallel
    {
#pragma omp single
        t = omp_get_num_threads();
    }
    return t;
#else
    return 1;
#endif
}
void oracle_pose(const oracle_robot* o, double pose[3]) { memcpy(pose, o->pose, 3 * sizeof(double)); }
double* oracle_P(oracle_robot* o) { return o->P; }
double* oracle_y(oracle_robot* o) { return o->y; }

void oracle_set_state(oracle_robot* o, const double* P, const double* y, int saved,
                      const double pose[3])
{
    const size_t n = (size_t)o->n;
    if (P) memcpy(o->P, P, n * n * sizeof(double));
    if (y) memcpy(o->y, y, n * sizeof(double));
    o->saved = saved;
    if (pose) memcpy(o->pose, pose, 3 * sizeof(double));
}

/* ------------------------------------------------------------------------------------ */
/* predict: P_pre = Fx·P·Fxᵀ + Fu·Q·Fuᵀ  (Robot.cpp:152-258)                             */
/* ------------------------------------------------------------------------------------ */

static void predict_faithful(oracle_robot* o, const double F3[9], const double Fu3[9],
                             const double Q[9])
{
    const int n = o->n;
    double* Fx = o->tmpA;
    double* FxP = o->tmpB;
    double* P_pre = o->P_pre;
    /* Fx (Robot.cpp:153-167) */
    memset(Fx, 0, sizeof(double) * (size_t)n * n);
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Fx[(size_t)i * n + j] = F3[i * 3 + j];
    for (int i = 3; i < n; i++) Fx[(size_t)i * n + i] = 1.0;
    /* Fu (n×3, Robot.cpp:178-188) */
    double* Fu = (double*)calloc((size_t)n * 3, sizeof(double));
    double* FuQ = (double*)calloc((size_t)n * 3, sizeof(double));
    for (int i = 0; i < 3; i++)
        for (int j = 0; j < 3; j++) Fu[i * 3 + j] = Fu3[i * 3 + j];
    /* Robot.cpp:242, 246 */
    oracle_dgemm(0, 0, n, n, n, 1.0, Fx, n, o->P, n, 0.0, FxP, n);
    oracle_dgemm(0, 1, n, n, n, 1.0, FxP, n, Fx, n, 0.0, P_pre, n);
    /* Robot.cpp:250, 254 — reuse Fx as Fu·Q·Fuᵀ (n×n) */
    oracle_dgemm(0, 0, n, 3, 3, 1.0, Fu, 3, Q, 3, 0.0, FuQ, 3);
    oracle_dgemm(0, 1, n, n, 3, 1.0, FuQ, 3, Fu, 3, 0.0, Fx, n);
    /* Robot.cpp:258 gsl_matrix_add */
    for (size_t e = 0; e < (size_t)n * n; e++) P_pre[e] += Fx[e];
    free(Fu);
    free(FuQ);
}

static void predict_fast(oracle_robot* o, const double F3[9], const double Fu3[9],
                         const double Q[9])
{
    /* Only rows/cols 0..2 of Fx differ from I: P_pre[i][j] = P[i][j] for i,j >= 3. */
    const int n = o->n;
    const double* P = o->P;
    double* Pp = o->P_pre;
    ORACLE_PAR_ROWS
    for (int r = 0; r < n; r++) memcpy(Pp + (size_t)r * n, P + (size_t)r * n, sizeof(double) * (size_t)n);
    /* rows 0..2: (Fx·P)[a][b] = Σ_k F3[a][k] P[k][b]; cols 0..2 by the transposed product. */
    ORACLE_PAR_ROWS
    for (int b = 3; b < n; b++) {
        for (int a = 0; a < 3; a++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += F3[a * 3 + k] * P[(size_t)k * n + b];
            Pp[(size_t)a * n + b] = s;
        }
        for (int a = 0; a < 3; a++) {
            double s = 0.0;
            for (int k = 0; k < 3; k++) s += P[(size_t)b * n + k] * F3[a * 3 + k];
            Pp[(size_t)b * n + a] = s;
        }
    }
    /* 3×3 block: F3·P33·F3ᵀ + Fu3·Q·Fu3ᵀ */
    double FP[9], FuQ[9];
    for (int a = 0; a < 3; a++)
        for (int b = 0; b < 3; b++) {
            double s = 0.0, t = 0.0;
            for (int k = 0; k < 3; k++) {
                s += F3[a * 3 + k] * P[(size_t)k * n + b];
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
            Pp[(size_t)a * n + b] = s + t;
        }
}

/* ------------------------------------------------------------------------------------ */
/* localize                                                                              */
/* ------------------------------------------------------------------------------------ */

int oracle_localize(oracle_robot* o, const oracle_line* lines, int L, const double enc[3],
                    int* match_out)
{
    const int n = o->n;
    const int N = o->N;
    const int fast = (o->mode == ORACLE_FAST);
    double* P = o->P;
    double* P_pre = o->P_pre;
    double* y = o->y;
    o->status = 0;
    o->gate_margin = INFINITY;
    o->pred = 0;
    const int s_in = o->saved;   /* the landmarks this scan can update (before any augmentation) */

    /* Robot.cpp:130-148 (SIMULATIONOFF branch; `rot` unused) */
    const double x_t0[3] = {o->pose[0], o->pose[1], o->pose[2]};
    double u[3] = {0, 0, 0};
    u[2] = x_t0[2] - enc[2];
    const double deltaX = x_t0[0] - enc[0];
    const double deltaY = x_t0[1] - enc[1];
    u[0] = sqrt(deltaX * deltaX + deltaY * deltaY);
    double x_pre[3] = {x_t0[0] + u[0] * cos(x_t0[2] + u[2] / 2.0),
                       x_t0[1] + u[0] * sin(x_t0[2] + u[2] / 2.0), x_t0[2] + u[2]};

    /* Fx rows 0..2 (Robot.cpp:155-163), Fu rows 0..2 (Robot.cpp:180-188), Q (Robot.cpp:215-218) */
    const double c = u[2] / 2.0 + x_t0[2];
    const double F3[9] = {1, 0, -u[0] * sin(c), 0, 1, u[0] * cos(c), 0, 0, 1};
    const double Fu3[9] = {cos(c), 0, -u[0] * sin(c) / 2.0, sin(c), 1, u[0] * cos(c) / 2.0, 0, 0, 1};
    const double qs = (-1.0 / (1 + fabs(u[0])) + 1);
    const double Q[9] = {ENCODERNOISE * qs, 0, 0, 0, 2 * ENCODERNOISE * qs, 0, 0, 0,
                         ENCODERNOISE * qs};
    if (fast) predict_fast(o, F3, Fu3, Q);
    else predict_faithful(o, F3, Fu3, Q);

    /* Robot.cpp:288-296 */
    int matchesNum = 0;
    int* extra = (int*)malloc(sizeof(int) * (size_t)(L > 0 ? L : 1));
    int nextra = 0;
    int nmatched = 0;
    double delta[2] = {0, 0};
    (void)delta;

    for (int i = 0; i < L; ++i) {                               /* Robot.cpp:298 */
        if (match_out) match_out[i] = -1;
        double R[4] = {0, 0, 0, 0};                              /* Robot.cpp:301-305 */
        if (o->r_mode == ORACLE_R_AS_WRITTEN) {
            if (i < 4) R[i] = lines[i].R[3];
        } else {
            memcpy(R, lines[i].R, sizeof(R));
        }
        const int s = o->saved;
        if (s == 0) extra[nextra++] = i;                         /* Robot.cpp:308-310 */

        for (int j = 0; j < s; ++j) {                            /* Robot.cpp:313 */
            int skip = 0;                                        /* Robot.cpp:315-330 */
            for (int q = 0; q < nmatched; q++)
                if (o->matched[q] == j) { skip = 1; break; }
            if (skip) {
                if (j == s - 1) { extra[nextra++] = i; break; }
                continue;
            }
            const int l0 = 3 + 2 * j, l1 = l0 + 1;
            const double ma = y[l0], mr = y[l1];
            /* Hx_small (Robot.cpp:367-380) */
            const double h10 = -cos(ma), h11 = -sin(ma);
            const double h1l = x_pre[0] * sin(ma) - x_pre[1] * cos(ma);
            double S[4] = {0, 0, 0, 0};
            if (!fast) {
                double* H = o->Hs;
                double* HP = o->HP;
                memset(H, 0, sizeof(double) * 2 * (size_t)n);
                H[0 * n + 2] = -1.0;
                H[1 * n + 0] = h10;
                H[1 * n + 1] = h11;
                H[0 * n + l0] = 1.0;
                H[0 * n + l1] = 0.0;
                H[1 * n + l0] = h1l;
                H[1 * n + l1] = 1.0;
                /* Robot.cpp:397, 401, 405 */
                oracle_dgemm(0, 0, 2, n, n, 1.0, H, n, P_pre, n, 0.0, HP, n);
                oracle_dgemm(0, 1, 2, 2, n, 1.0, HP, n, H, n, 0.0, S, 2);
            } else {
                const int idx[5] = {0, 1, 2, l0, l1};
                const double hr0[5] = {0, 0, -1.0, 1.0, 0};
                const double hr1[5] = {h10, h11, 0, h1l, 1.0};
                double hp0[5], hp1[5];
                for (int b = 0; b < 5; b++) {
                    double s0 = 0.0, s1 = 0.0;
                    for (int a = 0; a < 5; a++) {
                        const double p = P_pre[(size_t)idx[a] * n + idx[b]];
                        s0 += hr0[a] * p;
                        s1 += hr1[a] * p;
                    }
                    hp0[b] = s0;
                    hp1[b] = s1;
                }
                for (int b = 0; b < 5; b++) {
                    S[0] += hp0[b] * hr0[b];
                    S[1] += hp0[b] * hr1[b];
                    S[2] += hp1[b] * hr0[b];
                    S[3] += hp1[b] * hr1[b];
                }
            }
            for (int e = 0; e < 4; e++) S[e] += R[e];

            /* z, h (Robot.cpp:411-426) */
            double z[2] = {lines[i].alpha, lines[i].r};
            double h[2] = {ma - x_pre[2], mr - (x_pre[0] * cos(ma) + x_pre[1] * sin(ma))};
            h[0] = oracle_normalize_radian(h[0]);
            /* inv(S) (Robot.cpp:443-457) */
            double S_inv[4] = {0, 0, 0, 0};
            if (oracle_lu_invert2(S, S_inv)) o->status |= 1;
            /* v = z − h, 2π fold (Robot.cpp:465-475) */
            z[0] -= h[0];
            z[1] -= h[1];
            if (fabs(z[0] - 2.0 * M_PI) < fabs(z[0])) z[0] -= 2.0 * M_PI;
            else if (fabs(z[0] + 2.0 * M_PI) < fabs(z[0])) z[0] += 2.0 * M_PI;
            /* vᵀ S⁻¹ v (Robot.cpp:479-486) */
            double vS[2], d2;
            oracle_dgemm(1, 0, 1, 2, 2, 1.0, z, 1, S_inv, 2, 0.0, vS, 2);
            oracle_dgemm(0, 0, 1, 1, 2, 1.0, vS, 2, z, 1, 0.0, &d2, 1);

            if (fabs(sqrt(fabs(d2)) - MAHALANOBIS) < o->gate_margin) o->gate_margin = fabs(sqrt(fabs(d2)) - MAHALANOBIS);
            if (o->pred_eta > 0.0) {
                /* The gate distance against a state within pred_eta of this one: |ΔS_ab| <=
                 * eta·s_a·s_b with s_a = Σ_k |H_ak|·√P_kk over rows 0, 1, 2, l0, l1 (H0 = (0, 0, −1,
                 * 1, 0), H1 = (h10, h11, 0, h1l, 1)), so to first order |Δd²| <= eta·(|w0|·s0 +
                 * |w1|·s1)², w = S⁻¹v: a distance that close to the gate is not resolved (the
                 * reference's own evaluation order: Robot.cpp:313-489, every candidate up to the
                 * winner) */
                const double* Pd = P_pre;
                const double s0 = sqrt(fabs(Pd[(size_t)2 * n + 2])) + sqrt(fabs(Pd[(size_t)l0 * n + l0]));
                const double s1 = fabs(h10) * sqrt(fabs(Pd[0])) + fabs(h11) * sqrt(fabs(Pd[(size_t)n + 1])) +
                                  fabs(h1l) * sqrt(fabs(Pd[(size_t)l0 * n + l0])) + sqrt(fabs(Pd[(size_t)l1 * n + l1]));
                const double wv = fabs(vS[0]) * s0 + fabs(vS[1]) * s1;
                if (fabs(d2 - MAHALANOBIS * MAHALANOBIS) <= o->pred_eta * wv * wv) o->pred |= ORACLE_PRED_GATE;
            }
            if (sqrt(fabs(d2)) > MAHALANOBIS) {                  /* Robot.cpp:489-498 */
                if (j == s - 1) { extra[nextra++] = i; break; }
                continue;
            }
            /* match (Robot.cpp:500-641) */
            o->matched[nmatched++] = j;
            matchesNum++;
            if (match_out) match_out[i] = j;
            double* W = o->W;
            double* K = o->K;
            double* KS = o->KS;
            if (!fast) {
                /* Robot.cpp:522: P_pre·Hxᵀ (NT), 526: ·S⁻¹ */
                oracle_dgemm(0, 1, n, 2, n, 1.0, P_pre, n, o->Hs, n, 0.0, W, 2);
            } else {
                ORACLE_PAR_ROWS
                for (int r = 0; r < n; r++) {
                    const double* pr = P_pre + (size_t)r * n;
                    W[2 * r + 0] = -1.0 * pr[2] + 1.0 * pr[l0] + 0.0 * pr[l1];
                    W[2 * r + 1] = h10 * pr[0] + h11 * pr[1] + h1l * pr[l0] + 1.0 * pr[l1];
                }
            }
            oracle_dgemm(0, 0, n, 2, 2, 1.0, W, 2, S_inv, 2, 0.0, K, 2);
            const double dlt[2] = {z[0], z[1]};                  /* Robot.cpp:550 */
            /* Robot.cpp:560-572: P_pre −= (K·S)·Kᵀ ; P_t0 ← P_pre (deferred to the end) */
            oracle_dgemm(0, 0, n, 2, 2, 1.0, K, 2, S, 2, 0.0, KS, 2);
            if (!fast) {
                double* KSK = o->tmpA;
                oracle_dgemm(0, 1, n, n, 2, 1.0, KS, 2, K, 2, 0.0, KSK, n);
                for (size_t e = 0; e < (size_t)n * n; e++) P_pre[e] -= KSK[e];
            } else {
                ORACLE_PAR_ROWS
                for (int r = 0; r < n; r++) {
                    const double a0 = KS[2 * r], a1 = KS[2 * r + 1];
                    double* pr = P_pre + (size_t)r * n;
                    for (int cc = 0; cc < n; cc++) {
                        double t = 0.0;
                        t += a0 * K[2 * cc];
                        t += a1 * K[2 * cc + 1];
                        pr[cc] -= t;
                    }
                }
            }
            /* Robot.cpp:579-602 */
            y[0] = x_pre[0];
            y[1] = x_pre[1];
            y[2] = x_pre[2];
            for (int r = 0; r < n; r++) {
                double t = 0.0;
                t += K[2 * r] * dlt[0];
                t += K[2 * r + 1] * dlt[1];
                y[r] += t;
            }
            y[2] = oracle_normalize_radian(y[2]);
            o->pose[0] = y[0];
            o->pose[1] = y[1];
            o->pose[2] = y[2];
            x_pre[0] = y[0];
            x_pre[1] = y[1];
            x_pre[2] = y[2];
            break;                                               /* Robot.cpp:641 */
        }
    }

    if (L == 0 || matchesNum == 0) {                             /* Robot.cpp:702-716 */
        y[0] = x_pre[0];
        y[1] = x_pre[1];
        y[2] = x_pre[2];
        o->pose[0] = y[0];
        o->pose[1] = y[1];
        o->pose[2] = oracle_normalize_radian(y[2]);
    }
    int canc = 0;   /* (a scan that ends in the map reset updates no landmark it keeps) */
    if (o->pred_eta > 0.0 && matchesNum > 0) {
        /* An update that shrinks a landmark's variance trace by more than pred_cancel (more than
         * log2 of it of the stored precision's bits cancel) or leaves it non-positive: P still
         * holds the state before the scan (the landmark block is not predicted), P_pre after */
        for (int j = 0; j < s_in; j++) {
            const size_t a = (size_t)(3 + 2 * j), b = a + 1;
            const double tb = P[a * n + a] + P[b * n + b];
            const double ta = P_pre[a * n + a] + P_pre[b * n + b];
            if (!(ta > 0.0) || tb > o->pred_cancel * ta) { canc = 1; break; }
        }
    }
    /* P_t0 ← P_pre (Robot.cpp:572 per match / :713 no match) */
    ORACLE_PAR_ROWS
    for (int r = 0; r < n; r++) memcpy(P + (size_t)r * n, P_pre + (size_t)r * n, sizeof(double) * (size_t)n);

    /* augmentation (Robot.cpp:776-866) */
    for (int e = 0; e < nextra; e++) {
        const oracle_line* lin = &lines[extra[e]];
        const int s = o->saved;
        if (3 + 2 * s + 2 > n) { o->status |= 2; continue; }    /* capacity overflow: UB in ref */
        double alfa = lin->alpha;
        double r = lin->r + (o->pose[0] * cos(alfa) + o->pose[1] * sin(alfa));
        alfa += o->pose[2];
        const double Gx[6] = {0, 0, 1, cos(alfa), sin(alfa), 0};
        const double Gl[4] = {1.0, 0, y[1] * cos(alfa) - y[0] * sin(alfa), 1};
        alfa = oracle_normalize_radian(alfa);
        y[3 + 2 * s] = alfa;
        y[3 + 2 * s + 1] = r;
        const double* R = lin->R;                                /* Robot.cpp:807-811 */
        double GxPrr[6], Pll[4], GlR[4], GlRGl[4];
        oracle_dgemm(0, 0, 2, 3, 3, 1.0, Gx, 3, P, n, 0.0, GxPrr, 3);
        oracle_dgemm(0, 1, 2, 2, 3, 1.0, GxPrr, 3, Gx, 3, 0.0, Pll, 2);
        oracle_dgemm(0, 0, 2, 2, 2, 1.0, Gl, 2, R, 2, 0.0, GlR, 2);
        oracle_dgemm(0, 1, 2, 2, 2, 1.0, GlR, 2, Gl, 2, 0.0, GlRGl, 2);
        for (int q = 0; q < 4; q++) Pll[q] += GlRGl[q];
        if (o->pred_eta > 0.0)   /* fp32 storage's range, with 2x of slack (the library's bound: 2^120) */
            for (int q = 0; q < 4; q++)
                if (!(fabs(Pll[q]) <= 0x1p119)) o->pred |= ORACLE_PRED_RANGE;
        const int l0 = 3 + 2 * s;
        P[(size_t)l0 * n + l0] = Pll[0];
        P[(size_t)l0 * n + l0 + 1] = Pll[1];
        P[(size_t)(l0 + 1) * n + l0] = Pll[2];
        P[(size_t)(l0 + 1) * n + l0 + 1] = Pll[3];
        /* Robot.cpp:852-862: P[l0:l0+2, 0:l0] = Gx·P[0:3, 0:l0], then its transpose */
        oracle_dgemm(0, 0, 2, l0, 3, 1.0, Gx, 3, P, n, 0.0, P + (size_t)l0 * n, n);
        for (int q = 0; q < l0; q++) {
            P[(size_t)q * n + l0] = P[(size_t)l0 * n + q];
            P[(size_t)q * n + l0 + 1] = P[(size_t)(l0 + 1) * n + q];
        }
        o->saved = s + 1;
    }

    /* reset (Robot.cpp:893-904) */
    if (canc && !(o->saved > N - 10)) o->pred |= ORACLE_PRED_CANCEL;
    if (o->saved > N - 10) {
        o->saved = 0;
        for (int i = 3; i < n; ++i) y[i] = 0;
        ORACLE_PAR_ROWS
        for (int i = 0; i < n; i++)
            for (int j = 0; j < n; j++)
                if (i >= 3 || j >= 3) P[(size_t)i * n + j] = 0.0;
    }
    free(extra);
    return matchesNum;
}
