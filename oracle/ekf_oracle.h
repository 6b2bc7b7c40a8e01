/*
 * ekf_oracle.h — CPU restatement of the reference EKF-SLAM update (TEST INFRASTRUCTURE).
 *
 * This is the parity CHECKER for the MI355X path, never the product: only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it.
 *
 * It restates HuaiLeiTang/slam_ros `Robot::localize()` (slam_ros/Robot.cpp:126-904) with a
 * runtime landmark capacity N (the reference hard-wires LINESIZE 100, Robot.h:13-14) and
 * heap buffers instead of the reference's stack arrays.
 *
 * Parity pinning: the reference cannot be built in this image (it needs GSL headers/libs and
 * ROS, neither present). The only known-answer data the reference holds is the
 * MATLAB self-evaluation quiz in Robot.h:146-178 (generic EKF prediction + update), which
 * tests/golden/kat_matlab.json pins through oracle_dgemm / oracle_lu_invert2. The
 * SLAM-specific structure (H, gating, augmentation, reset) is "parity unpinned" by reference
 * vectors: it is pinned only by this statement-by-statement restatement and by the
 * faithful-vs-fast cross-check in tests/test_oracle.py.
 *
 * Two modes share every scalar formula:
 *   ORACLE_FAITHFUL — dense n×n GSL-equivalent arithmetic in the reference's call order,
 *                      including the n³ Fx·P·Fxᵀ predict (Robot.cpp:242-258) and dense
 *                      per-candidate H·P·Hᵀ (Robot.cpp:397-405). The dead Hx fill
 *                      (Robot.cpp:344-362) and debug printing are not reproduced.
 *   ORACLE_FAST     — algebraically identical, sparse-aware (O(n) predict, 5×5 gating blocks,
 *                      O(n²) per match). Used as the CPU baseline and as the checker at N≥1024.
 */
#ifndef EKF_ORACLE_H
#define EKF_ORACLE_H

#ifdef __cplusplus
extern "C" {
#endif

enum { ORACLE_FAITHFUL = 0, ORACLE_FAST = 1 };
/* R (line covariance) source inside the association loop:
 *   INTENDED  — R = line.C_AR, as in the augmentation at Robot.cpp:807-811.
 *   AS_WRITTEN — the reference's loop at Robot.cpp:302-304 (`R[i] = C_AR->data[j]`) under
 *                zero-initialised stack: R = 0 except R[i] = C_AR[3] for line index i < 4
 *                (i >= 4 is an out-of-bounds write in the reference; here it is dropped). */
enum { ORACLE_R_INTENDED = 0, ORACLE_R_AS_WRITTEN = 1 };

typedef struct oracle_line {
    double alpha;   /* line.alfa (robot frame), simplifyPath.h:67 */
    double r;       /* line.r, simplifyPath.h:68 */
    double R[4];    /* line.C_AR->data, 2x2 row-major, simplifyPath.h:71 */
} oracle_line;

typedef struct oracle_robot oracle_robot;

/* Robot::Robot(x, y, theta), Robot.cpp:20-35, with zero-initialised y / P / savedLineCount. */
oracle_robot* oracle_create(int capacity, double x, double y, double theta, int mode, int r_mode);
void oracle_destroy(oracle_robot* o);

/* Robot::localize(lines, rot, encoder), Robot.cpp:126-904 (SIMULATIONOFF == true branch).
 * match_out[i] (optional, length L): saved-landmark index matched by line i, or -1 when the
 * line was appended to extraLines. Returns the number of matches (matchesNum). */
int oracle_localize(oracle_robot* o, const oracle_line* lines, int L, const double enc[3],
                    int* match_out);

int oracle_n(const oracle_robot* o);
int oracle_capacity(const oracle_robot* o);
int oracle_saved(const oracle_robot* o);
int oracle_status(const oracle_robot* o);
/* min |sqrt(|d²|) − 0.4| over the candidates the last localize evaluated (INFINITY: none) */
double oracle_gate_margin(const oracle_robot* o);
/* Test instrumentation (not in the reference): the decisions of the last localize that a stored
 * state within relative precision eta of this one could not resolve — a gate distance within
 * eta·(|w0|·s0 + |w1|·s1)² of the gate (ORACLE_PRED_GATE), an update that shrinks some landmark's
 * variance trace by more than `cancel` or to <= 0 (ORACLE_PRED_CANCEL), a new landmark variance
 * past 2^119 (ORACLE_PRED_RANGE). The GPU library reports the same conditions on its own state as
 * EKF_ST_PRECISION / EKF_ST_RANGE; the tests check its flags against these. eta = 0: off. */
enum { ORACLE_PRED_GATE = 1, ORACLE_PRED_CANCEL = 2, ORACLE_PRED_RANGE = 4 };
void oracle_set_pred(oracle_robot* o, double eta, double cancel);
int oracle_pred_flags(const oracle_robot* o);
/* threads the O(n^2) loops run on: 1 in libekf_oracle.so, the OpenMP team in libekf_oracle_omp.so */
int oracle_threads(void);   /* OR of GSL-like error codes seen in last call */
void oracle_pose(const oracle_robot* o, double pose[3]);
double* oracle_P(oracle_robot* o);          /* n*n row-major P_t0 (Robot.h:62) */
double* oracle_y(oracle_robot* o);          /* n state vector y (Robot.h:26) */
void oracle_set_state(oracle_robot* o, const double* P, const double* y, int saved,
                      const double pose[3]);

/* ---- primitives (exposed for the known-answer tests) ---- */
/* gslcblas row-major dgemm loop semantics (GSL cblas/source_gemm_r.h, recalled; GSL absent). */
void oracle_dgemm(int transA, int transB, int M, int N, int K, double alpha,
                  const double* A, int lda, const double* B, int ldb, double beta,
                  double* C, int ldc);
/* gsl_linalg_LU_decomp + gsl_linalg_LU_invert on a 2x2 (Robot.cpp:449-457).
 * Returns 0, or 1 (GSL_EDOM) when U is singular, leaving Sinv untouched. */
int oracle_lu_invert2(const double S[4], double Sinv[4]);
/* Robot::normalizeRadian, Robot.cpp:62-71 (non-standard for |rad| >= 2π). */
double oracle_normalize_radian(double rad);

#ifdef __cplusplus
}
#endif
#endif
