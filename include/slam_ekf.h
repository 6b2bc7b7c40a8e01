/*
 * slam_ekf.h — C-ABI of the MI355X-native EKF-SLAM update (libslam_ekf.so).
 *
 * Drop-in boundary for HuaiLeiTang/slam_ros `class Robot` (slam_ros/Robot.h:21-77). The
 * reference has no FFI: its interface is the C++ class, so every entry point below names the
 * member (file:line) it replaces. Plain pointers and sizes only; no GSL/ROS/torch types.
 *
 * One context = E independent EKF instances (an ensemble) of capacity N landmarks on one
 * HIP device, one HIP stream. State n = 3 + 2N (Robot.h:13-14 LINESIZE/SLAMSIZE, runtime here).
 * Contexts are not thread-safe (the reference is single-threaded, main.cpp:130-179).
 *
 * Errors: every call returns an int status (EKF_OK == 0). The reference's localize() returns
 * void and only prints GSL error codes (Robot.cpp:128, 909-917); per-instance numeric
 * conditions (singular S, capacity overflow, fp16 range) are reported in ekf_result.status
 * instead and the state is committed, as in the reference. One condition the reference cannot
 * have is handled differently: EKF_ST_SYNC_TIMEOUT (an instance spread over G > 1 cooperating
 * workgroups lost one of them) rolls that instance's call back instead of committing it. A
 * context whose instances fit one workgroup (N <= 192, e.g. the drop-in's N = 100) cannot time
 * out, so there every call commits.
 *
 * The library reads no environment variables: diagnostics and test hooks are per-context
 * options (ekf_set_option), all off by default.
 */
#ifndef SLAM_EKF_H
#define SLAM_EKF_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ekf_debug_scan_stamps fills 32 slots (was 16); ekf_config.arith (formerly reserved) selects
 *    the fp32 flush arithmetic and EKF_ARITH_BF16X6 is rejected (EKF_EINVAL) for configurations
 *    that can never use it; EKF_ST_SYNC_TIMEOUT rolls the call back instead of committing it.
 * 3: ekf_set_option / ekf_get_option replace the environment variables the library used to read
 *    (EKF_SPECULATE, EKF_SPIN_LOG2, EKF_TEST_DROP_WG, EKF_MFREP, EKF_SCAN_STAMPS,
 *    EKF_DD_BLOCKS_PER_CU, EKF_FLUSH_VARIANT); EKF_ARITH_F16X3; the row shard replaced by a
 *    partitioned instance (ekf_shard_create ... ekf_shard_end: tiles partitioned, O(n) state
 *    replicated). */
#define SLAM_EKF_ABI_VERSION 3
#define EKF_MAX_LINES 64 /* lines per scan per instance; main.cpp:99 reserves 20 */

/* status codes */
enum {
    EKF_OK = 0,
    EKF_EINVAL = 1,   /* bad argument */
    EKF_ENOMEM = 2,   /* device / host allocation failed */
    EKF_EDEVICE = 3,  /* HIP runtime error / no device */
    EKF_ERANGE = 4,   /* instance index / line count out of range */
};
/* ekf_result.status bits (per instance, per call) */
enum {
    EKF_ST_SINGULAR_S = 1, /* gsl_linalg_LU_invert → GSL_EDOM on some candidate (Robot.cpp:454) */
    EKF_ST_CAPACITY = 2,   /* augmentation beyond capacity (UB in the reference, Robot.cpp:802) */
    EKF_ST_NONSYM = 4,     /* EKF_R_AS_WRITTEN only: a line with index 1 or 2 matched. Its R has a
                              single off-diagonal entry (Robot.cpp:302-304), so the reference's
                              K·S·Kᵀ — and from then on its P — is not symmetric; the packed
                              symmetric storage keeps the upper triangle. */
    EKF_ST_SYNC_TIMEOUT = 8, /* the instance's cooperating workgroups did not all arrive at an
                                exchange within the spin bound: the call is rolled back (the
                                instance keeps its state from before the call, as if the scan had
                                not been received; the result record reports no matches) */
    EKF_ST_RANGE = 16,     /* EKF_PREC_F16: a landmark this call added has a variance above a
                              quarter of the fp16 range at the instance's storage exponent
                              (2^exp·P stored; values are still finite). ekf_rescale re-chooses
                              the exponent; ignoring it lets later landmarks saturate to ±inf.
                              EKF_PREC_F32: a new landmark variance above 2^120, within 2^8 of
                              fp32's range (a diverged filter: the fp64 storage holds it) */
    EKF_ST_PRECISION = 32, /* EKF_PREC_F32: the call's update shrank some landmark's variance (the
                              trace of its 2x2 block) by more than 2^4, or left it non-positive:
                              more than 4 of fp32's 24 significant bits cancel, so the stored
                              block is no longer guaranteed to resolve the fp64 reference to the
                              1e-6 bar (informational: the state commits; EKF_PREC_F64 holds any
                              filter). Every precision: a gate distance the call evaluated (up to
                              the winner) lies within the storage precision of the gate of the
                              threshold (|ΔP_ab| up to eta·sqrt(P_aa·P_bb), eta 2^-16 for F32,
                              2^-8 F16, 2^-44 F64, first order), so the reference's state may decide
                              that line differently. In SURVEY §8d's world the reference's own
                              motion model runs away and this is how a diverging
                              instance shows */
};

/* storage precision of the landmark-landmark covariance block (robot rows, mean: always fp64).
 * F16: fp16 storage, fp32 MFMA accumulation, the block rounded to fp16 after every scan
 * (BASELINE config 5); the tolerance it meets is stated in tests/test_gpu_parity.py. */
enum { EKF_PREC_F64 = 0, EKF_PREC_F32 = 1, EKF_PREC_F16 = 2 };
/* R source inside the association loop (SURVEY.md §8a parity-mode flags) */
enum { EKF_R_INTENDED = 0, EKF_R_AS_WRITTEN = 1 };
/* arithmetic of the fp32 covariance flush (ekf_config.arith).
 * EXACT: v_mfma_f32_32x32x2_f32; the flush's per-element chain is the ordered fp32 FMA chain the
 *   association kernel replays on read, so the state is bit-identical for every flush interval
 *   and schedule (default; the C++ drop-in uses it).
 * BF16X6: requires EKF_PREC_F32 or EKF_PREC_F16, EKF_R_INTENDED and max_lines <= 8; any other
 *   configuration is rejected by ekf_create with EKF_EINVAL. Every fp32 operand is split exactly
 *   into three bf16 parts (hi + mid + lo), six v_mfma_f32_32x32x16_bf16 per product (all part
 *   products down to 2^-16 relative; the dropped ones are below 2^-24), accumulated in fp32; fp16
 *   storage is scaled out of its exponent on load and rounded to fp16 once per group on store.
 *   Within fp32 rounding of EXACT (the 1e-6 bound of BASELINE holds; fp16: its re-stated 1e-3) but
 *   no longer bit-identical across flush intervals: the state depends on T at the level of fp32
 *   rounding. The association kernel applies pending steps by the same bf16 MFMAs on the planes
 *   (EKF_OPT_MFMA_REPLAY) and keeps the diagonal blocks in fp64. Groups of an even number of steps
 *   (2..16) take the split-bf16 flush, augmentation and resets included: the wave-tiles holding a
 *   landmark the group added are recomputed by the exact general loop in a second pass, and those
 *   of an instance whose map was reset in the group are stored as zero; the wave-tiles past every
 *   step's nonzero operand rows are skipped (EKF_OPT_ACTIVE_FLUSH). An odd-sized group (a partial
 *   group flushed by a drain) takes the EXACT forms (ekf_flush_kernel_name reports the form).
 * F16X3: the same requirements, schedule and fallbacks as BF16X6, with a two-part fp16 split
 *   instead: every operand row is scaled by 2^σ (σ per instance, from the largest landmark variance
 *   vmax: |2^σ·V| <= 2^12 because each step's downdate V·Vᵀ is bounded by the variances it reduces;
 *   σ is chosen at the first scan of a flush group and changes mid-group only on a reset or a new
 *   landmark 64x above the variance it was set for; an instance whose σ changes inside a group,
 *   or one with a landmark whose variance is below 2^-4·4^-σ (the planes would lose bits relative
 *   to that landmark's own scale: PLANE_SIGMA_EXACT, a filter spanning more than 2^28 in
 *   variance), runs that group's flush and on-read replay in the exact forms), split into hi + lo
 *   fp16 parts (22 significant bits), and each product runs as three v_mfma_f32_32x32x16_f16 —
 *   (lo, hi), (hi, lo), (hi, hi) — accumulated in fp32, the accumulators holding P·2^(2σ)
 *   (power-of-two scalings, exact). Half the MFMA work and two thirds of the plane bytes of BF16X6;
 *   per product within ≈2^-21 of the rows' own scale (BF16X6: 2^-23), held to the same bar per scan
 *   from identical inputs (tests/test_bench_config.py, SURVEY §8d's world included). */
enum { EKF_ARITH_EXACT = 0, EKF_ARITH_BF16X6 = 1, EKF_ARITH_F16X3 = 2 };

typedef struct ekf_config {
    int32_t capacity;      /* N = LINESIZE (Robot.h:13); landmarks per instance */
    int32_t instances;     /* E: independent EKF instances in this context */
    int32_t precision;     /* EKF_PREC_* for the landmark block of P */
    int32_t device;        /* HIP device ordinal, -1 = current */
    int32_t max_lines;     /* per-scan line capacity per instance, <= EKF_MAX_LINES */
    int32_t r_mode;        /* EKF_R_* */
    int32_t reset_margin;  /* map wiped when savedLineCount > N - margin (Robot.cpp:893: 10) */
    int32_t pipeline;      /* 1: double-buffer the landmark block so that association kernels
                              may overlap the covariance downdate of earlier scans (applying it on
                              read, bit-identically); 0: in-place, strictly sequential. Overlap
                              happens only when an instance fits one association workgroup
                              (N <= 192): otherwise its cooperating workgroups must not wait on
                              CUs a flush holds, so its association kernels are ordered after the
                              flush in flight, and the second buffer is not allocated */
    int32_t flush_interval;/* T >= 1: the landmark block is rewritten once per T scans by one
                              rank-2·Σm MFMA pass; scans in between read it with the pending
                              downdates applied on read. With EKF_ARITH_EXACT the state is
                              bit-identical for every T (the MFMA chain is an ordered FMA chain);
                              the split arithmetics are within fp32 rounding of it instead.
                              T = 1: once per scan. <= 16 (<= 24 with EKF_ARITH_F16X3) */
    int32_t arith;         /* EKF_ARITH_* (fp32 flush arithmetic); formerly reserved, 0 = EXACT */
    double mahalanobis;    /* MAHALANOBIS gate, Robot.h:15 (0.4) */
    double encoder_noise;  /* ENCODERNOISE, Robot.h:17 (0.024) */
} ekf_config;

/* One observed line: the fields of `line` (simplifyPath.h:62-79) that localize reads. */
typedef struct ekf_line {
    double alpha; /* line.alfa, robot frame */
    double r;     /* line.r */
    double R[4];  /* *line.C_AR, 2x2 row-major */
} ekf_line;

/* Per-instance outcome of one localize (what Robot exposes after the call). */
typedef struct ekf_result {
    double pose[3];            /* xPos, yPos, thetaPos (Robot.h:54-56) */
    int32_t matches;           /* matchesNum (Robot.h:36) */
    int32_t new_landmarks;     /* extraLines.size() (Robot.cpp:291) */
    int32_t saved;             /* savedLineCount after the call (Robot.h:28) */
    int32_t reset;             /* 1 if the capacity reset ran (Robot.cpp:893-904) */
    int32_t status;            /* EKF_ST_* bits */
    int32_t nlines;
    int32_t match[EKF_MAX_LINES]; /* matched saved index per line, -1 = appended as new */
} ekf_result;

typedef struct ekf_ctx ekf_ctx;

void ekf_config_init(ekf_config* cfg);
const char* ekf_strerror(int status);
int ekf_abi_version(void);

/* Robot::Robot(x, y, theta) for every instance (Robot.cpp:20-35), y/P/savedLineCount zeroed. */
int ekf_create(const ekf_config* cfg, ekf_ctx** out);
int ekf_destroy(ekf_ctx* ctx);
/* Order all work after/before the caller's stream (e.g. torch's current stream). NULL = own. */
int ekf_set_stream(ekf_ctx* ctx, void* hip_stream);
int ekf_sync(ekf_ctx* ctx);

/* Per-context options: diagnostics, alternative (result-identical or parity-equivalent) kernel
 * forms and test hooks. A new context has every option at its default; nothing is read from the
 * environment. ekf_set_option drains the context first (the option applies from the next call)
 * and returns EKF_EINVAL for an unknown option, EKF_ERANGE for a value out of range. */
enum {
    /* association path: 1 speculative (default), 0 the sequential chain on every scan (one
     * cross-workgroup exchange per line), 2 test hook: every guess wrong (the speculative path,
     * a failed verdict and the sequential restart on every scan), 3 test hook: the guesses of
     * lines L/2 .. L-1 wrong (a failed verdict keeps the lines before the first wrong one).
     * Identical results. */
    EKF_OPT_SPECULATE = 1,
    /* spin bound of the association's cross-workgroup waits: 2^v polls, 8 <= v <= 24 (24) */
    EKF_OPT_SPIN_LOG2 = 2,
    /* fp32 / fp16 flush form, all bit-identical within an arithmetic: 0 automatic (default),
     * 2 the super-tile form for every group, 8 the wave form also for groups of 2 and 4 steps,
     * 24 the split-bf16 flush on 2 x 4 wave-tiles, 44 the split-fp16 flush on groups of 2 x 2
     * wave-tiles sharing their operand planes through LDS (groups of 6 or more steps) */
    EKF_OPT_FLUSH_FORM = 3,
    /* workgroups per CU of the grid-strided flush forms, 1..16 (8) */
    EKF_OPT_FLUSH_BLOCKS_PER_CU = 4,
    /* pending steps applied on read by MFMA. 1 (default): split arithmetics by their own split
     * products on the operand planes (a step whose planes cannot carry the instance's dynamic
     * range is replayed exactly, PLANE_SIGMA_EXACT), fp64 storage by the flush's own f64 MFMA
     * (bit-identical); 2: split arithmetics by fp32 MFMA on the fp32 operand rows (exact
     * products: within a flush group the association reads the block at the EXACT arithmetic's
     * precision, ≈3 µs per scan more at T = 20); 0: the per-element replay forms */
    EKF_OPT_MFMA_REPLAY = 5,
    /* 1: the association kernel's instrumented instantiation with phase timers
     * (ekf_debug_scan_stamps); 0 (default) the product kernel */
    EKF_OPT_SCAN_STAMPS = 6,
    /* test hook: e + 1 = the last association workgroup of instance e never runs (its exchanges
     * time out and the instance's calls roll back); 0 off (default) */
    EKF_OPT_TEST_DROP_WG = 7,
    /* test hook: e + 1 = on the speculative path, association workgroup 1 of instance e treats
     * its verdict poll as timed out while every other workgroup completes; 0 off (default) */
    EKF_OPT_TEST_VERDICT_TIMEOUT = 8,
    /* 1 (default): the split-arithmetic flush skips the wave-tiles whose columns lie past every
     * landmark with a nonzero operand row or new row in the group (unchanged by it: a partly
     * filled map streams only its active part); 0: every wave-tile */
    EKF_OPT_ACTIVE_FLUSH = 9,
    /* landmarks per association workgroup: 0 automatic (default: the narrowest that fits), 192,
     * or 128 / 64 (more workgroups per instance, each with fewer landmarks, on more CUs: fp32 /
     * fp16 storage with EKF_R_INTENDED and max_lines <= 8, every flush arithmetic, when an
     * instance then needs at most 64 workgroups and the instances still fit the device in one
     * launch; otherwise 192). Identical results for every value. */
    EKF_OPT_SCAN_THREADS = 10,
};
int ekf_set_option(ekf_ctx* ctx, int option, int value);
int ekf_get_option(const ekf_ctx* ctx, int option, int* value);

/* Robot::Robot(x, y, theta) on one instance (e < 0: all instances). */
int ekf_reset_instance(ekf_ctx* ctx, int e, double x, double y, double theta);

/* Robot::localize(lines, rot, encoder) (Robot.h:74, Robot.cpp:126-904) on every instance.
 * Host buffers: encoder[E*3] (realRoboPose, main.cpp:84-89), lines[E*max_lines] (instance e
 * uses lines[e*max_lines ... + nlines[e]-1]), nlines[E]. out[E] optional. Synchronous.
 * `rot` (wheel rotations) is not an input: SIMULATIONOFF == true (Robot.h:18) never uses it. */
int ekf_localize(ekf_ctx* ctx, const double* encoder, const ekf_line* lines,
                 const int32_t* nlines, ekf_result* out);
/* Same, with all three inputs already resident in device memory; asynchronous on the
 * context stream. Results stay on the device until ekf_read_results(). */
int ekf_localize_device(ekf_ctx* ctx, const double* d_encoder, const ekf_line* d_lines,
                        const int32_t* d_nlines);
/* The two halves of localize: predict = Robot.cpp:130-286 (motion model and
 * P_pre), update = Robot.cpp:288-904 (association, Kalman updates, augmentation, reset).
 * predict followed by update == localize. */
int ekf_predict(ekf_ctx* ctx, const double* encoder);
int ekf_update(ekf_ctx* ctx, const ekf_line* lines, const int32_t* nlines, ekf_result* out);
int ekf_read_results(ekf_ctx* ctx, ekf_result* out);

/* State transfer (fixtures, tests, checkpoints). P_full is the reference's dense row-major
 * n×n P_t0 (Robot.h:62) in fp64; y is Robot::y (Robot.h:26); pose = xPos/yPos/thetaPos. */
int ekf_upload_state(ekf_ctx* ctx, int e, const double* P_full, const double* y, int saved,
                     const double pose[3]);
/* Any pointer may be NULL. With P_full the call drains first (the pending downdates are flushed);
 * without it, it only waits for the context's stream: the mean, pose and savedLineCount are
 * committed by every scan, and the flush schedule is left as it is. */
int ekf_download_state(ekf_ctx* ctx, int e, double* P_full, double* y, int* saved,
                       double pose[3]);
/* Device-side initialisation P = diag(d) + U·Uᵀ (U: n×rank row-major, host pointers). */
int ekf_init_lowrank(ekf_ctx* ctx, int e, const double* diag, const double* U, int rank,
                     const double* y, int saved, const double pose[3]);
/* EKF_PREC_F16 storage exponent: the landmark block is stored as fp16(2^exp·P). Upload and
 * init_lowrank choose it from the largest landmark variance v (exp = min(10, ⌊log2(4096/v)⌋),
 * at least -24; 10 for an empty map); ekf_rescale(ctx, e, EKF_EXP_AUTO) re-chooses it from the
 * current P (EKF_ST_RANGE), or sets the given exponent. Power-of-two rescaling is exact except
 * for values that leave fp16's normal range. For f32 / f64 storage the exponent is 0 and
 * rescale is a no-op. */
#define EKF_EXP_AUTO (-1000)
int ekf_storage_exponent(const ekf_ctx* ctx, int e);
int ekf_rescale(ekf_ctx* ctx, int e, int exp);
/* P_t0[0:3,0:3] of instance e (what getEllipse reads, Robot.cpp:75-77). */
int ekf_get_pose_cov(ekf_ctx* ctx, int e, double P33[9]);
/* Robot::getEllipse(axii, angle) (Robot.h:73, Robot.cpp:73-124): axii sorted by |eigenvalue|,
 * angle = atan2 of the larger eigenvalue's unit eigenvector in GSL's sign convention. Returns 1
 * on success, 0 if the 2x2 eigenproblem failed (as the reference's bool), negative on API error. */
int ekf_get_ellipse(ekf_ctx* ctx, int e, float axii[2], float* angle);
/* The same computation on a given 2x2 block P22 = {P00, P01, P10, P11} (host only, no device):
 * gsl_eigen_nonsymmv + GSL_EIGEN_SORT_ABS_ASC restated (sign convention included). Returns 1,
 * 0 for a non-finite block or a complex eigenvalue pair, negative on API error. Divergence: for a
 * complex pair (only a non-symmetric block has one; P's pose block is symmetric) the reference's
 * nonsymmv succeeds and it publishes |Re λ| and an angle from the real parts of the complex
 * eigenvector; that branch of GSL is not restated here, axii and angle are left untouched. */
int ekf_ellipse_of_block(const double P22[4], float axii[2], float* angle);

/* One instance with its landmark block partitioned over ranks, for maps
 * whose packed P should not (or cannot) live on one GPU. No reference member maps to these: they
 * replace the single call Robot::localize (Robot.h:34, Robot.cpp:126-904) for an instance spread over
 * processes. ekf_shard_create makes rank `rank` of `world` a context of one instance (instances =
 * 1, EKF_ARITH_EXACT, fp32 or fp64 with flush_interval <= 8, no pipeline, max_lines <= 8)
 * that stores only its share of the packed landmark block: the tiles of tile rows [row_begin,
 * row_end) (ekf_shard_tiles), a contiguous slice balanced by tile count, about 1/world of it
 * (ekf_landmark_block_bytes). Everything of size O(n) (robot strip, mean, the landmarks' scan
 * state and diagonal blocks, the downdate operands) is replicated and evolves identically on every
 * rank. ekf_upload_state / ekf_init_lowrank store the rank's tiles; ekf_download_state returns the
 * full robot rows and mean and the rank's tiles, zero elsewhere (the ranks' landmark blocks sum to
 * the instance's).
 * Per scan (Robot.cpp:126-904, the sequential association), every call asynchronous on the context
 * stream except ekf_shard_end; buf is the caller's device buffer of ekf_shard_buffer_words doubles
 * ([N][4] 2x2 blocks), which the caller sums over the ranks where marked (each rank fills the
 * blocks its tiles hold, zeros elsewhere: the sum is exact):
 *   ekf_shard_begin(enc, lines, L, buf)     predict (Robot.cpp:130-286); the rank's diagonal blocks
 *   SUM buf over ranks
 *   for each line i < L, in order:
 *     ekf_shard_line(i, buf)                gate of every landmark (Robot.cpp:313-498: the first
 *                                           passing unmatched one, found by every rank alike), the
 *                                           winner's package, the rank's blocks of its column
 *     SUM buf over ranks
 *     ekf_shard_apply(i, buf)               gain rows of every landmark, robot update (Robot.cpp:522-602)
 *   ekf_shard_end(out)                      augmentation (Robot.cpp:776-866), the capacity reset
 *                                           (Robot.cpp:893-904), commit; the step joins the flush,
 *                                           which rewrites the rank's tiles only; out[0] as
 *                                           ekf_read_results (synchronous)
 * With the same inputs the state is bit-identical to a single context's (exact arithmetic). A
 * partitioned context rejects ekf_localize, ekf_localize_device, ekf_predict and ekf_update. */
int ekf_shard_create(const ekf_config* cfg, int rank, int world, ekf_ctx** out);
int ekf_shard_tiles(const ekf_ctx* ctx, int* row_begin, int* row_end);
size_t ekf_shard_buffer_words(const ekf_ctx* ctx);
int ekf_shard_begin(ekf_ctx* ctx, const double enc[3], const ekf_line* lines, int nlines, double* buf);
int ekf_shard_line(ekf_ctx* ctx, int line, double* buf);
int ekf_shard_apply(ekf_ctx* ctx, int line, const double* buf);
int ekf_shard_end(ekf_ctx* ctx, ekf_result* out);
/* Abandons the open scan (before ekf_shard_end nothing of the committed state has been written),
 * e.g. after a failed exchange; a phase that fails abandons it too. */
int ekf_shard_abort(ekf_ctx* ctx);
/* The speculative association of a partitioned instance: the per-line exchanges replaced by one.
 *   ekf_shard_begin(enc, lines, L, buf); SUM buf over ranks
 *   ekf_shard_speculate(buf, cols)          every line's first passing landmark at the scan's start
 *                                           (its guess, found by every rank alike), the rank's
 *                                           blocks of every guessed column into cols
 *                                           (ekf_shard_spec_buffer_words doubles, [L][N][4])
 *   SUM cols over ranks
 *   ekf_shard_run(cols, next)               lines 0 .. L−1 as the per-line phases compute them, each
 *                                           winner's column from cols; stops at the first line
 *                                           whose first passing landmark is not its guess and
 *                                           writes that line (or L) as a double to next, device
 *                                           memory of the caller (asynchronous, stream-ordered;
 *                                           L + 1 when its cooperating workgroups' exchange timed
 *                                           out: abandon the scan, ekf_shard_abort)
 *   ekf_shard_resume(line)                  the host's copy of next (every rank reads the same)
 *   for each line i from next: ekf_shard_line, SUM buf, ekf_shard_apply (the per-line protocol)
 *   ekf_shard_end(out)
 * Bit-identical to the per-line protocol; every rank stops at the same line (replicated state).
 * EKF_OPT_SPECULATE = 2 (test hook) makes every line guess landmark 0. */
/* The same scan as one call, with the exchanges on the library's own RCCL communicator (RCCL is
 * loaded on first use; EKF_EDEVICE if it is not available): rank 0 gets an id with
 * ekf_rccl_unique_id, the host hands it to every rank, and each attaches with its (rank, world)
 * of ekf_shard_create. ekf_shard_localize then runs begin, SUM, speculate, SUM, run, MAX, end on
 * the context's stream before its one host read: the end phase commits only if the agreement says
 * every line ran on every rank, and otherwise changes nothing, when resume / the per-line phases
 * and the end follow (a second host read). It is bit-identical to the sequence above (Robot::localize,
 * Robot.cpp:126-904). A phase failing on any rank, or a run whose workgroups timed out, abandons
 * the scan on every rank alike (the error, or EKF_EDEVICE on the ranks where nothing failed);
 * a failed collective returns EKF_EDEVICE. */
int ekf_rccl_unique_id(unsigned char out[128]);
int ekf_shard_attach_rccl(ekf_ctx* ctx, const unsigned char id[128], int rank, int world);
int ekf_shard_localize(ekf_ctx* ctx, const double enc[3], const ekf_line* lines, int nlines, ekf_result* out);
size_t ekf_shard_spec_buffer_words(const ekf_ctx* ctx);
int ekf_shard_speculate(ekf_ctx* ctx, const double* buf, double* cols);
int ekf_shard_run(ekf_ctx* ctx, const double* cols, double* next_line);
int ekf_shard_resume(ekf_ctx* ctx, int line);

/* Introspection for the benchmark's roofline accounting. */
size_t ekf_landmark_block_bytes(const ekf_ctx* ctx); /* stored bytes of P_ll per instance */
int ekf_state_dim(const ekf_ctx* ctx);                /* n */
/* Per-kernel HIP-event timing on the stream each kernel runs on: enable 0 = off, 1 = the flush
 * only (2 events per flush), 2 = also every association kernel. Averages are over the launches
 * recorded since the last enable: scan_ms = association kernel (level 2), downdate_ms = the
 * landmark-block flush, augment_ms = 0 (augmentation is fused into the flush), launches =
 * flushes. */
int ekf_profile_enable(ekf_ctx* ctx, int enable);
int ekf_profile_read(ekf_ctx* ctx, double* scan_ms, double* downdate_ms, double* augment_ms,
                     int* launches);
/* Per-launch flush timing of the launches recorded since the last enable (level >= 1): fills
 * nsteps[k] (steps the launch applied) and ms[k] for k < min(cap, count); returns the count
 * (negative on error). ekf_flush_kernel_name: the kernel form a flush of nsteps steps runs. */
int ekf_profile_flushes(ekf_ctx* ctx, int cap, int* nsteps, float* ms);
const char* ekf_flush_kernel_name(const ekf_ctx* ctx, int nsteps);
/* Diagnostic: association-kernel phase timers (sum over instances, 100 MHz ticks), collected
 * only while EKF_OPT_SCAN_STAMPS is 1. 32 slots (ABI 2; ABI 1 had 16):
 * 0 predict, 1 diagonal gather + barrier, 2 gating, 3 min-reduction barrier, 4 winner package,
 * 5 broadcast barrier, 6 gain rows, 7 commit/augmentation, 8 total, 9 launches; 16-19 per-line
 * phases of the first landmark wave (gate, wait for the package, gain rows, robot update);
 * 20-22 gate-filter counts; the rest scripts/assoc_probe.py names. */
int ekf_debug_scan_stamps(ekf_ctx* ctx, unsigned long long out[32]);
/* Diagnostic: words 0..15 of instance e's result record as of the last ekf_read_results
 * (word 9: association path code, 10..14: the first five guessed winners, 15: 1 if the call was
 * rolled back after EKF_ST_SYNC_TIMEOUT). */
int ekf_debug_result_words(ekf_ctx* ctx, int e, int out[16]);

#ifdef __cplusplus
}
#endif
#endif /* SLAM_EKF_H */
