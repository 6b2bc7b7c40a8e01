// ekf_api.hip — C-ABI (include/slam_ekf.h) over the gfx950 kernels in ekf_kernels.hip.
//
// A context owns E instances' state in HBM and two HIP streams:
//   S  association/gain kernels (scan_kernel) — all state except the landmark block — and, on
//      the sequential schedule, the flushes too (stream order is the only dependency);
//   D  the landmark-block flush of the pipelined schedule.
// Every update step k writes its downdate operands, augmented rows and result record into slot
// k mod R of a ring. The landmark block is rewritten by a flush once per group of T =
// flush_interval steps; association kernels read the last materialised block ("base") with the
// steps not yet in it applied on read (bit-identical to flushing first, see ekf_kernels.hip).
//   sequential (pipeline = 0): one buffer, flushed in place on S after the group's last scan;
//     R = T.
//   pipelined  (pipeline = 1): flush f reads X[in] and writes X[out] = the other buffer while the
//     next group's scans run on S reading X[in] — the output of flush f-1 — with the steps of
//     groups f and f+1 pending (< 2T); R = 2T.
// Any call that reads or replaces the landmark block drains (flushes the partial group, syncs).
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <dlfcn.h>

#include <algorithm>
#include <new>
#include <vector>

#include <rccl/rccl.h>   // (types only: the library loads RCCL on first use, ekf_rccl_unique_id)

#include "../../include/slam_ekf.h"
#include "ekf_kernels.h"

using ekf::Dims;

struct EvPair {
    hipEvent_t a, b;
};

struct ekf_ctx {
    ekf_config cfg;
    Dims d;
    int device;
    hipStream_t own_stream;   // S unless the caller supplies one
    hipStream_t stream;       // S
    hipStream_t dstream;      // D
    size_t elem;              // bytes per stored landmark-block element
    size_t op_elem;           // bytes per downdate operand element (fp32 for fp16 storage)
    size_t pll_inst;          // elements per instance (the whole packed block)
    long long t0 = 0, t1 = 0; // tiles stored per instance [t0, t1): all, unless partitioned (ekf_shard_create)
    size_t xinst;             // stored landmark-block elements per instance ((t1 − t0)·TILE_ELEMS)
    size_t op_inst;           // operand elements per instance
    void* X[2];
    double* Rs;               // [2][E][3][n] robot strip, two copies (the association kernel reads
    double* y;                // [2][E][n]    copy cur[e] and writes the other; the lead commits it)
    int* cur;                 // [E] committed copy per instance (device; read back when needed)
    double* dense = nullptr;   // n × n fp64 scratch of upload / download / rescale (allocated on first use, kept)
    // partitioned instance (ekf_shard_create): rank sh_rank of sh_world stores tile rows [sh_r0, sh_r1);
    // the running scan's replicated state
    int sh_rank = -1, sh_world = 0, sh_r0 = 0, sh_r1 = 0;
    double* sh_rob = nullptr;
    double* sh_rec = nullptr;
    double* sh_hist = nullptr;
    double* sh_pkg = nullptr;
    int* sh_flags = nullptr;
    int* sh_ctl = nullptr;
    int sh_L = 0, sh_line = 0, sh_open = 0;   // sh_open: 1 during a scan; sh_line: the next line expected
    int sh_diag = 0;                           // begin's exchange consumed (SH_DIAG ran) in this scan
    ekf::Slot sh_null;        // a step that applies nothing (pads an odd partial group to the wave flush)
    double* pose;
    double* xpre;
    int* saved;
    double* D;                // [2][E][N][4] diagonal landmark blocks after the last committed step
                              // (split-bf16 contexts: the association kernel's MFMA replay)
    std::vector<ekf::Slot> ring;   // R per-step slots
    double* Ust;              // fp64 gain scratch of the running scan
    double* Vst;
    int2* tile_rc;
    int2* stile_rc;
    int2* stile2_rc;
    int nstiles2;
    ekf::WtEntry* wt;
    int nwt;
    ekf::WtEntry* wt64;
    int nwt64;
    int* wt24;                // split-bf16 wave-tiles of 2 × 4 tiles (wr | wc << 16), panel order
    int nwt24;
    ekf::WtEntry* wtq;        // split-fp16 quad form: groups of 2 × 2 wave-tiles (four entries each)
    int nwtq;
    double* d_enc;            // the scan inputs: views of d_in, staged from h_in by one copy
    ekf_line* d_lines;
    int* d_nlines;
    char* d_in;
    char* h_in;               // pinned
    size_t in_lines, in_nlines, in_bytes;   // byte offsets of the lines and counts, the total
    int in_pending;           // a copy from h_in was enqueued (ev_in)
    hipEvent_t ev_in;
    void* rccl_comm;          // ekf_shard_attach_rccl: the partitioned instance's own communicator
    double* sh_xbuf;          // ... and ekf_shard_localize's exchange buffers (device): [N][4] + flag,
    double* sh_xcols;         // [L][N][4] + flag + stopping line
    double* h_agree;          // pinned: the agreement pair and a flag word
    int sh_dirty;             // a failed scan left nonzero flag words
    int* h_res;
    double* h_pose;
    // the synchronous calls' result mirror (ScanParams::res_host): pinned, written by the scan's
    // lead; h_r33 the robot block, h_ep the epoch of each instance's last mirrored commit
    double* h_r33;
    unsigned* h_ep;
    int* hd_res;              // (their device pointers)
    double* hd_pose;
    double* hd_r33;
    unsigned* hd_ep;
    int mirror_on;            // the association launch being enqueued writes the mirror
    unsigned mirror_epoch;    // scan_epoch of the mirrored robot blocks (0: none valid)
    int dd_grid;
    int dd_per_cu;            // flush workgroups per CU of the grid-strided forms (EKF_OPT_FLUSH_BLOCKS_PER_CU)
    int dd_variant;           // f32 flush kernel form (EKF_OPT_FLUSH_FORM)
    int ncu;
    int G;                    // association workgroups per instance
    int mbw;                  // mailbox words per workgroup slot
    int spec;                 // speculative association (EKF_OPT_SPECULATE)
    int spin_log2;            // spin bound of the association kernel's waits (EKF_OPT_SPIN_LOG2)
    int test_drop;            // test hook (EKF_OPT_TEST_DROP_WG = e + 1): instance e's last workgroup never runs
    int test_verdict;         // test hook (EKF_OPT_TEST_VERDICT_TIMEOUT = e + 1)
    int mfrep_opt;            // EKF_OPT_MFMA_REPLAY
    int active_flush;         // EKF_OPT_ACTIVE_FLUSH
    int mfrep;                // split-bf16 contexts: MFMA replay of pending steps (bf && mfrep_opt)
    int scan_batch;           // instances per association launch (co-residency bound), 192 wide
    int resident;             // association workgroups the device holds at once
    int nt_opt;               // EKF_OPT_SCAN_THREADS
    int Gmax;                 // workgroups per instance at the narrowest width (mailbox, sync words)
    int last_G;               // workgroups per instance of the last association launch
    unsigned scan_epoch;      // association launches so far (mailbox tags)
    double* mbox;
    int* sync;
    int sync_stride;
    unsigned long long* dbg;  // association-kernel phase timers (EKF_OPT_SCAN_STAMPS = 1, else null)
    int* pexp;                // [E] fp16 storage exponents (device), host copy below
    void* sink;               // scratch tile for the wave flushes (DowndateParams::sink)
    void* ops_u;              // operand rows of every ring slot (U), slot_bytes apart
    void* ops_v;              // ... (V)
    long long slot_bytes;
    void* ops_b;              // split-plane arithmetics: the planes of V of every ring slot (else null)
    long long bslot_bytes;
    bool bf;                  // a split-plane flush applies (arith, fp32 operands, symmetric R, kmax 16)
    int pmode;                // its plane arithmetic: 1 EKF_ARITH_BF16X6, 2 EKF_ARITH_F16X3 (0: none)
    int* psig;                // [E] EKF_ARITH_F16X3 plane exponent σ (device; the association kernel's
    double* pvmax;            // [E] lead lowers it when a new landmark raises the largest variance)
    std::vector<int> pexp_h;
    // flush scheduling (see the top of this file)
    int T;                    // flush interval
    long long nsteps;         // update steps enqueued
    long long unflushed0;     // first step not covered by an enqueued flush
    long long pend0;          // first step not contained in X[base]
    int base;                 // buffer the association kernels read
    int last_out;             // buffer the newest enqueued flush writes (materialised after drain)
    long long nflush;
    hipEvent_t ev_scan;       // recorded on S after each update scan
    hipEvent_t ev_flush[2];   // recorded on D after flush f (f & 1)
    hipEvent_t ev_base;       // event guarding X[base] and the ring (nullptr: none pending)
    // profiling
    int prof;
    std::vector<EvPair> ev[3];   // scan, downdate, patch
    std::vector<int> ev_nsteps;  // steps applied by each timed flush (ev[1])
    std::vector<EvPair> pool;
};

#define HIP_TRY(expr)                                                                       \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            fprintf(stderr, "slam_ekf: %s failed: %s\n", #expr, hipGetErrorString(_e));     \
            return EKF_EDEVICE;                                                             \
        }                                                                                   \
    } while (0)

extern "C" {

void ekf_config_init(ekf_config* c)
{
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->capacity = 100;        // Robot.h:13
    c->instances = 1;
    c->precision = EKF_PREC_F64;
    c->device = -1;
    c->max_lines = 20;        // main.cpp:99 lines.reserve(20)
    c->r_mode = EKF_R_INTENDED;
    c->reset_margin = 10;     // Robot.cpp:893
    c->mahalanobis = 0.4;     // Robot.h:15
    c->encoder_noise = 0.024; // Robot.h:17
}

const char* ekf_strerror(int s)
{
    switch (s) {
    case EKF_OK: return "ok";
    case EKF_EINVAL: return "invalid argument";
    case EKF_ENOMEM: return "out of memory";
    case EKF_EDEVICE: return "HIP device error";
    case EKF_ERANGE: return "index out of range";
    default: return "unknown error";
    }
}

int ekf_abi_version(void) { return SLAM_EKF_ABI_VERSION; }

}  // extern "C"

static void free_all(ekf_ctx* c)
{
    std::vector<void*> ptrs = {c->X[0], c->X[1], c->Rs, c->y, c->cur, c->pose, c->xpre, c->saved, c->D,
                               c->tile_rc, c->stile_rc, c->stile2_rc, c->wt, c->wt64, c->wt24, c->wtq, c->d_in, c->dbg, c->pexp, c->sink, c->mbox,
                               c->sync, c->Ust, c->Vst, c->dense, c->psig, c->pvmax,
                               c->sh_rob, c->sh_rec, c->sh_hist, c->sh_pkg, c->sh_flags, c->sh_ctl,
                               c->sh_null.res, c->sh_xbuf, c->sh_xcols};
    ptrs.push_back(c->ops_u);
    ptrs.push_back(c->ops_v);
    ptrs.push_back(c->ops_b);
    for (auto& sl : c->ring) {
        ptrs.push_back(sl.patch);
        ptrs.push_back(sl.patch_diag);
        ptrs.push_back(sl.res);
    }
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->h_agree) (void)hipHostFree(c->h_agree);
    if (c->h_res) (void)hipHostFree(c->h_res);
    if (c->h_pose) (void)hipHostFree(c->h_pose);
    if (c->h_r33) (void)hipHostFree(c->h_r33);
    if (c->h_in) (void)hipHostFree(c->h_in);
    if (c->ev_in) (void)hipEventDestroy(c->ev_in);
    if (c->h_ep) (void)hipHostFree(c->h_ep);
    for (auto& v : c->ev)
        for (auto& pr : v) { (void)hipEventDestroy(pr.a); (void)hipEventDestroy(pr.b); }
    for (auto& pr : c->pool) { (void)hipEventDestroy(pr.a); (void)hipEventDestroy(pr.b); }
    if (c->ev_scan) (void)hipEventDestroy(c->ev_scan);
    for (int k = 0; k < 2; k++)
        if (c->ev_flush[k]) (void)hipEventDestroy(c->ev_flush[k]);
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
    if (c->dstream) (void)hipStreamDestroy(c->dstream);
}

static int enqueue_flush(ekf_ctx* c);

// Flush the partial group and wait for both streams; afterwards X[last_out] is the materialised
// landmark block and nothing is pending.
static int drain(ekf_ctx* c)
{
    if (c->nsteps > c->unflushed0) {
        int rc = enqueue_flush(c);
        if (rc) return rc;
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipStreamSynchronize(c->dstream));
    c->base = c->last_out;
    c->pend0 = c->nsteps;
    c->ev_base = nullptr;
    return EKF_OK;
}

static inline int cur_buf(const ekf_ctx* c) { return c->last_out; }

// instance e's stored tiles in buffer buf; and the kernels' view of instance 0, in which tile t sits
// at t·TILE_ELEMS (a partitioned instance stores the tiles [t0, t1) only: the view is shifted)
static inline char* xinst_ptr(const ekf_ctx* c, int buf, int e)
{
    return (char*)c->X[buf] + (size_t)e * c->xinst * c->elem;
}
static inline void* xview(const ekf_ctx* c, int buf)
{
    return (char*)c->X[buf] - (ptrdiff_t)c->t0 * ekf::TILE_ELEMS * (ptrdiff_t)c->elem;
}

// Committed copy of instance e's robot strip and mean (the association kernel flips it when it
// commits a launch): read back after the stream has drained up to here.
static int strip_copy(ekf_ctx* c, int e, int* cb)
{
    HIP_TRY(hipMemcpyAsync(cb, c->cur + e, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (*cb != 0 && *cb != 1) return EKF_EDEVICE;
    return EKF_OK;
}

static inline double* strip_of(const ekf_ctx* c, int cb, int e)
{
    return c->Rs + ((size_t)cb * c->cfg.instances + e) * 3 * c->d.n;
}

static inline double* mean_of(const ekf_ctx* c, int cb, int e)
{
    return c->y + ((size_t)cb * c->cfg.instances + e) * c->d.n;
}

static int set_exponent(ekf_ctx* c, int e, int ex)
{
    c->pexp_h[e] = ex;
    HIP_TRY(hipMemcpy(c->pexp + e, &ex, sizeof(int), hipMemcpyHostToDevice));
    return EKF_OK;
}

// fp16 storage exponent for a landmark block whose largest variance is vmax: the largest
// 2^x <= 2^10 with 2^x·vmax <= 2^12 (16× below the fp16 range, 4× below the EKF_ST_RANGE warning)
static int choose_exponent(const ekf_ctx* c, double vmax)
{
    if (c->cfg.precision != EKF_PREC_F16) return 0;
    if (!(vmax > 0.0) || !std::isfinite(vmax)) return ekf::F16_EXP_DEFAULT;
    const int x = (int)std::floor(std::log2(4096.0 / vmax));
    return std::max(-24, std::min(ekf::F16_EXP_DEFAULT, x));
}

// EKF_ARITH_F16X3 plane exponent of instance e from its largest landmark variance (every context
// keeps it; only F16X3 reads it)
static int set_plane_scale(ekf_ctx* c, int e, double vmax)
{
    const int sg = ekf::plane_sigma(vmax);
    const double vm = (vmax > 0.0 && std::isfinite(vmax)) ? vmax : 0.0;
    HIP_TRY(hipMemcpy(c->psig + e, &sg, sizeof(int), hipMemcpyHostToDevice));
    HIP_TRY(hipMemcpy(c->pvmax + e, &vm, sizeof(double), hipMemcpyHostToDevice));
    return EKF_OK;
}

static int set_robot_ctor(ekf_ctx* c, int e, double x, double y, double th)
{
    // Robot::Robot (Robot.cpp:20-35): P_t0[0][0] = P_t0[1][1] = 0.05, P_t0[2][2] = 0, the rest
    // (and y, savedLineCount) zero.
    const Dims& d = c->d;
    HIP_TRY(hipMemsetAsync(xinst_ptr(c, cur_buf(c), e), 0, c->xinst * c->elem, c->stream));
    const int zero = 0;
    const double v = 0.05;
    HIP_TRY(hipMemcpyAsync(c->cur + e, &zero, sizeof(int), hipMemcpyHostToDevice, c->stream));
    for (int cb = 0; cb < 2; cb++) {
        HIP_TRY(hipMemsetAsync(strip_of(c, cb, e), 0, sizeof(double) * 3 * d.n, c->stream));
        HIP_TRY(hipMemsetAsync(mean_of(c, cb, e), 0, sizeof(double) * d.n, c->stream));
        HIP_TRY(hipMemcpyAsync(strip_of(c, cb, e) + 0, &v, sizeof(double), hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipMemcpyAsync(strip_of(c, cb, e) + d.n + 1, &v, sizeof(double), hipMemcpyHostToDevice,
                               c->stream));
    }
    const double pose[3] = {x, y, th};
    HIP_TRY(hipMemcpyAsync(c->pose + 3 * e, pose, sizeof(pose), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->xpre + 3 * e, pose, sizeof(pose), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->saved + e, &zero, sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    const int rc = set_plane_scale(c, e, 0.0);   // an empty map
    if (rc) return rc;
    return set_exponent(c, e, c->cfg.precision == EKF_PREC_F16 ? ekf::F16_EXP_DEFAULT : 0);
}

// One packed-tile-row partition of the landmark block over `world` ranks: boundaries on even tile
// rows (whole wave-tile rows of the flush) balancing the tiles per rank; rank's rows [r0, r1)
static void tile_partition(int nb, int world, int rank, int& r0, int& r1)
{
    const long long total = (long long)nb * (nb + 1) / 2;
    auto boundary = [&](int k) {
        if (k <= 0) return 0;
        if (k >= world) return nb;
        // the even tile row whose prefix of tiles is closest to k/world of them
        const long long want = total * k / world;
        int bi = 0;
        while (bi + 2 < nb && ekf::tile_index(bi + 2, bi + 2, nb) <= want) bi += 2;
        if (bi + 2 < nb && ekf::tile_index(bi + 2, bi + 2, nb) - want < want - ekf::tile_index(bi, bi, nb)) bi += 2;
        return bi;
    };
    r0 = boundary(rank);
    r1 = boundary(rank + 1);
}

static int create_ctx(const ekf_config* cfg, int sh_rank, int sh_world, ekf_ctx** out);

extern "C" int ekf_create(const ekf_config* cfg, ekf_ctx** out)
{
    return create_ctx(cfg, -1, 0, out);
}

extern "C" int ekf_shard_create(const ekf_config* cfg, int rank, int world, ekf_ctx** out)
{
    if (!cfg || !out) return EKF_EINVAL;
    *out = nullptr;
    // one instance, the exact arithmetic, fp32 or fp64 storage, the sequential schedule, groups the
    // wave flushes take (fp32 <= 8 steps, fp64 <= 8)
    if (world < 1 || rank < 0 || rank >= world || cfg->instances != 1 || cfg->pipeline ||
        cfg->arith != EKF_ARITH_EXACT || (cfg->precision != EKF_PREC_F32 && cfg->precision != EKF_PREC_F64) ||
        cfg->flush_interval > (cfg->precision == EKF_PREC_F64 ? ekf::F64_WAVE_MAXS : 8) || cfg->max_lines > 8)
        return EKF_EINVAL;
    return create_ctx(cfg, rank, world, out);
}

static int create_ctx(const ekf_config* cfg, int sh_rank, int sh_world, ekf_ctx** out)
{
    if (!cfg || !out) return EKF_EINVAL;
    *out = nullptr;
    // capacity bound: one association thread per landmark, at most MAX_GROUPS workgroups of
    // SCAN_THREADS per instance (N <= 32768, i.e. n <= 65539)
    if (cfg->capacity < 1 || cfg->capacity > ekf::MAX_CAPACITY ||
        cfg->instances < 1 ||
        cfg->max_lines < 1 ||
        cfg->max_lines > EKF_MAX_LINES ||
        (cfg->precision != EKF_PREC_F64 && cfg->precision != EKF_PREC_F32 &&
         cfg->precision != EKF_PREC_F16) ||
        (cfg->r_mode != EKF_R_INTENDED && cfg->r_mode != EKF_R_AS_WRITTEN) ||
        cfg->flush_interval < 0 ||
        cfg->flush_interval > (cfg->arith == EKF_ARITH_F16X3 ? ekf::F16X3_MAXS : 16) ||
        (cfg->arith != EKF_ARITH_EXACT && cfg->arith != EKF_ARITH_BF16X6 && cfg->arith != EKF_ARITH_F16X3) ||
        // the split-plane flushes need symmetric fp32 operands with kmax = 16 (slam_ekf.h)
        (cfg->arith != EKF_ARITH_EXACT &&
         (cfg->precision == EKF_PREC_F64 || cfg->r_mode != EKF_R_INTENDED || cfg->max_lines > 8)))
        return EKF_EINVAL;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return EKF_EDEVICE;
    ekf_ctx* c = new (std::nothrow) ekf_ctx();
    if (!c) return EKF_ENOMEM;
    c->cfg = *cfg;
    if (cfg->device >= 0) {
        if (cfg->device >= ndev || hipSetDevice(cfg->device) != hipSuccess) {
            delete c;
            return EKF_EDEVICE;
        }
    }
    (void)hipGetDevice(&c->device);
    c->d = ekf::make_dims(cfg->capacity, cfg->max_lines);
    const Dims& d = c->d;
    const int E = cfg->instances;
    c->elem = (cfg->precision == EKF_PREC_F64) ? 8 : (cfg->precision == EKF_PREC_F32) ? 4 : 2;
    c->op_elem = (cfg->precision == EKF_PREC_F64) ? 8 : 4;   // operands in the compute type
    c->pll_inst = (size_t)d.ntiles * ekf::TILE_ELEMS;
    c->t0 = 0;
    c->t1 = d.ntiles;
    if (sh_world > 0) {
        tile_partition(d.nb, sh_world, sh_rank, c->sh_r0, c->sh_r1);
        if (c->sh_r0 >= c->sh_r1) {   // more ranks than wave-tile rows
            delete c;
            return EKF_ERANGE;
        }
        c->sh_rank = sh_rank;
        c->sh_world = sh_world;
        c->t0 = ekf::tile_index(c->sh_r0, c->sh_r0, d.nb);
        c->t1 = c->sh_r1 < d.nb ? ekf::tile_index(c->sh_r1, c->sh_r1, d.nb) : d.ntiles;
    }
    c->xinst = (size_t)(c->t1 - c->t0) * ekf::TILE_ELEMS;
    c->op_inst = (size_t)d.nb * 64 * (d.kmax / 2);
    c->G = (d.N + ekf::SCAN_THREADS - 1) / ekf::SCAN_THREADS;
    c->Gmax = (d.N + 63) / 64;   // EKF_OPT_SCAN_THREADS = 64
    c->last_G = c->G;
    c->nt_opt = 0;
    // pipeline: the association kernels of an instance spread over G > 1 cooperating workgroups
    // must never wait on CUs a flush holds, so they are ordered after the flush in flight, and
    // nothing would overlap: such contexts run the sequential schedule (slam_ekf.h)
    if (c->G > 1) c->cfg.pipeline = 0;
    int rc = EKF_ENOMEM;
#define ALLOC(ptr, bytes)                                                       \
    do {                                                                        \
        if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess) goto fail;        \
        if (hipMemset((void*)(ptr), 0, (bytes)) != hipSuccess) goto fail;       \
    } while (0)
    ALLOC(c->X[0], c->xinst * c->elem * E);
    if (c->cfg.pipeline) ALLOC(c->X[1], c->xinst * c->elem * E);
    else c->X[1] = nullptr;
    ALLOC(c->Rs, sizeof(double) * 3 * d.n * E * 2);
    ALLOC(c->y, sizeof(double) * d.n * E * 2);
    ALLOC(c->cur, sizeof(int) * E);
    ALLOC(c->pose, sizeof(double) * 3 * E);
    ALLOC(c->xpre, sizeof(double) * 3 * E);
    ALLOC(c->saved, sizeof(int) * E);
    ALLOC(c->D, sizeof(double) * 4 * d.N * E * 2);
    ALLOC(c->Ust, sizeof(double) * d.max_lines * d.n * 2 * E);
    ALLOC(c->Vst, sizeof(double) * d.max_lines * d.n * 2 * E);
    c->T = cfg->flush_interval > 0 ? cfg->flush_interval : 1;
    c->ring.assign((size_t)c->T * (c->cfg.pipeline ? 2 : 1), ekf::Slot{});
    // the operand rows of all slots in two contiguous buffers (fixed slot stride): the wave
    // flush addresses step q's rows from one base and its ring index (DowndateParams::ubase)
    c->slot_bytes = (long long)(((c->op_inst * c->op_elem * E) + 255) / 256 * 256);
    ALLOC(c->ops_u, (size_t)c->slot_bytes * c->ring.size());
    ALLOC(c->ops_v, (size_t)c->slot_bytes * c->ring.size());
    // split-plane flushes: V's planes per slot (written by the association kernel), three bf16
    // (BF16X6) or two fp16 (F16X3) per operand element
    c->bf = cfg->arith != EKF_ARITH_EXACT;   // (validated above: fp32 / fp16, symmetric R, kmax 16)
    c->pmode = c->bf ? cfg->arith : 0;
    c->ops_b = nullptr;
    c->bslot_bytes = 0;
    if (c->bf) {
        const int npl = c->pmode == EKF_ARITH_F16X3 ? 2 : 3;
        c->bslot_bytes = (long long)((c->op_inst * npl * 2 * E + 255) / 256 * 256);
        ALLOC(c->ops_b, (size_t)c->bslot_bytes * c->ring.size());
    }
    ALLOC(c->psig, sizeof(int) * E);
    ALLOC(c->pvmax, sizeof(double) * E);
    for (size_t i = 0; i < c->ring.size(); i++) {
        ekf::Slot& sl = c->ring[i];
        sl.Uop = (char*)c->ops_u + (size_t)c->slot_bytes * i;
        sl.Vop = (char*)c->ops_v + (size_t)c->slot_bytes * i;
        sl.Bop = c->bf ? (char*)c->ops_b + (size_t)c->bslot_bytes * i : nullptr;
        ALLOC(sl.patch, sizeof(double) * d.max_lines * 2 * d.M * E);
        ALLOC(sl.patch_diag, sizeof(double) * d.max_lines * 4 * E);
        ALLOC(sl.res, sizeof(int) * ekf::RES_STRIDE * E);
    }
    ALLOC(c->tile_rc, sizeof(int2) * d.ntiles);
    {
        const int nsb = (d.nb + ekf::DD_SB - 1) / ekf::DD_SB;
        ALLOC(c->stile_rc, sizeof(int2) * (size_t)nsb * (nsb + 1) / 2);
        ALLOC(c->stile2_rc, sizeof(int2) * (size_t)nsb * ((d.nb + 1) / 2));
    }
    c->in_lines = ((sizeof(double) * 3 * E + 15) / 16) * 16;
    c->in_nlines = c->in_lines + ((sizeof(ekf_line) * d.max_lines * E + 15) / 16) * 16;
    c->in_bytes = c->in_nlines + sizeof(int) * E;
    ALLOC(c->d_in, c->in_bytes);
    c->d_enc = reinterpret_cast<double*>(c->d_in);
    c->d_lines = reinterpret_cast<ekf_line*>(c->d_in + c->in_lines);
    c->d_nlines = reinterpret_cast<int*>(c->d_in + c->in_nlines);
    ALLOC(c->pexp, sizeof(int) * E);
    ALLOC(c->sink, 8 * ekf::TILE_ELEMS);
    c->pexp_h.assign(E, 0);
    // whole 128-B lines: the package words, then 16 words for the speculative list words
    c->mbw = ((ekf::MB_WORDS_FIXED + 4 * d.max_lines + 15) / 16) * 16 + 16;
    // options (ekf_set_option): defaults, nothing from the environment
    c->spec = 1;
    c->spin_log2 = 24;
    c->test_drop = 0;
    c->test_verdict = 0;
    c->mfrep_opt = 1;
    c->active_flush = 1;
    c->mfrep = c->bf ? 1 : 0;
    c->dbg = nullptr;
    ALLOC(c->mbox, sizeof(double) * 2 * c->Gmax * c->mbw * E);
    if (c->sh_world > 0) {
        // the partitioned instance's scan state (replicated on every rank) and a step that applies
        // nothing (rolled back: every flush form skips it), which pads an odd partial group
        ALLOC(c->sh_rob, sizeof(double) * 12);
        ALLOC(c->sh_rec, sizeof(double) * d.N * ekf::SH_REC);
        ALLOC(c->sh_hist, sizeof(double) * d.N * d.max_lines * 8);
        ALLOC(c->sh_pkg, sizeof(double) * (ekf::MB_WORDS_FIXED + 4 * d.max_lines));
        ALLOC(c->sh_flags, sizeof(int) * d.N);
        ALLOC(c->sh_ctl, sizeof(int) * ekf::SC_WORDS);
        ALLOC(c->sh_null.res, sizeof(int) * ekf::RES_STRIDE);
        const int one = 1;
        if (hipMemcpy(c->sh_null.res + ekf::RES_ROLLBACK, &one, sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
            goto fail;
        c->sh_null.Uop = c->ring[0].Uop;
        c->sh_null.Vop = c->ring[0].Vop;
        c->sh_null.patch = c->ring[0].patch;
        c->sh_null.patch_diag = c->ring[0].patch_diag;
    }
    c->sync_stride = ((ekf::SYNC_WG0 + c->Gmax + 15) / 16) * 16;
    ALLOC(c->sync, sizeof(int) * c->sync_stride * E);
#undef ALLOC
    if (hipHostMalloc((void**)&c->h_res, sizeof(int) * ekf::RES_STRIDE * E) != hipSuccess) goto fail;
    if (hipHostMalloc((void**)&c->h_pose, sizeof(double) * 3 * E) != hipSuccess) goto fail;
    if (hipHostMalloc((void**)&c->h_r33, sizeof(double) * 9 * E) != hipSuccess) goto fail;
    if (hipHostMalloc((void**)&c->h_ep, sizeof(unsigned) * E) != hipSuccess) goto fail;
    if (hipHostMalloc((void**)&c->h_in, c->in_bytes) != hipSuccess) goto fail;
    if (hipEventCreateWithFlags(&c->ev_in, hipEventDisableTiming) != hipSuccess) goto fail;
    memset(c->h_ep, 0, sizeof(unsigned) * E);
    if (hipHostGetDevicePointer((void**)&c->hd_res, c->h_res, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->hd_pose, c->h_pose, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->hd_r33, c->h_r33, 0) != hipSuccess ||
        hipHostGetDevicePointer((void**)&c->hd_ep, c->h_ep, 0) != hipSuccess)
        goto fail;
    rc = EKF_EDEVICE;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) goto fail;
    if (hipStreamCreateWithFlags(&c->dstream, hipStreamNonBlocking) != hipSuccess) goto fail;
    c->stream = c->own_stream;
    if (hipEventCreateWithFlags(&c->ev_scan, hipEventDisableTiming) != hipSuccess) goto fail;
    for (int k = 0; k < 2; k++)
        if (hipEventCreateWithFlags(&c->ev_flush[k], hipEventDisableTiming) != hipSuccess) goto fail;
    {
        std::vector<int2> rcv((size_t)d.ntiles);
        for (int bi = 0; bi < d.nb; bi++)
            for (int bj = bi; bj < d.nb; bj++) {
                int2 v;
                v.x = bi;
                v.y = bj;
                rcv[(size_t)ekf::tile_index(bi, bj, d.nb)] = v;
            }
        if (hipMemcpy(c->tile_rc, rcv.data(), sizeof(int2) * d.ntiles, hipMemcpyHostToDevice) !=
            hipSuccess)
            goto fail;
        const int nsb = (d.nb + ekf::DD_SB - 1) / ekf::DD_SB;
        std::vector<int2> srcv;
        for (int bi = 0; bi < nsb; bi++)
            for (int bj = bi; bj < nsb; bj++) {
                int2 v;
                v.x = bi;
                v.y = bj;
                srcv.push_back(v);
            }
        if (hipMemcpy(c->stile_rc, srcv.data(), sizeof(int2) * srcv.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
            goto fail;
        // 4 × 2 super-tiles holding at least one stored tile (bi <= bj): sbj·2 + 1 >= sbi·4
        std::vector<int2> s2;
        for (int si = 0; si < nsb; si++)
            for (int sj = 0; sj < (d.nb + 1) / 2; sj++)
                if (sj * 2 + 1 >= si * 4) {
                    int2 v;
                    v.x = si;
                    v.y = sj;
                    s2.push_back(v);
                }
        c->nstiles2 = (int)s2.size();
        if (hipMemcpy(c->stile2_rc, s2.data(), sizeof(int2) * s2.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
            goto fail;
        // WT_R × WT_C wave-tiles holding a stored tile (wc·WT_C + WT_C − 1 >= wr·WT_R), in panels
        // of 16 wave-tile columns walked row by row (the wave-tiles an XCD has in flight share
        // operand rows); each entry carries its tile indices and operand row blocks
        const int nwr = (d.nb + ekf::WT_R - 1) / ekf::WT_R, nwc = (d.nb + ekf::WT_C - 1) / ekf::WT_C;
        std::vector<ekf::WtEntry> wt;
        for (int pc = 0; pc < nwc; pc += 16)
            for (int wr = 0; wr < nwr; wr++)
                for (int wc = pc; wc < pc + 16 && wc < nwc; wc++) {
                    if (wc * ekf::WT_C + ekf::WT_C - 1 < wr * ekf::WT_R) continue;
                    ekf::WtEntry v;
                    memset(&v, 0, sizeof(v));
                    // a stored tile of this wave-tile (its first row, last column in the block)
                    const int fbi = wr * ekf::WT_R, fbj = std::min(wc * ekf::WT_C + ekf::WT_C - 1, d.nb - 1);
                    for (int r = 0; r < ekf::WT_R; r++)
                        for (int cc = 0; cc < ekf::WT_C; cc++) {
                            const int i = r * ekf::WT_C + cc;
                            const int bi = wr * ekf::WT_R + r, bj = wc * ekf::WT_C + cc;
                            const bool ok = bi < d.nb && bj < d.nb && bi <= bj;
                            v.tile[i] = (int)(ok ? ekf::tile_index(bi, bj, d.nb) : ekf::tile_index(fbi, fbj, d.nb));
                            v.valid |= (ok ? 1 : 0) << i;
                        }
                    for (int r = 0; r < ekf::WT_R; r++)
                        v.rows[0] |= std::min(wr * ekf::WT_R + r, d.nb - 1) << (16 * r);
                    for (int cc = 0; cc < ekf::WT_C; cc++)
                        v.rows[1] |= std::min(wc * ekf::WT_C + cc, d.nb - 1) << (16 * cc);
                    v.rc = wr | (wc << 16);
                    wt.push_back(v);
                }
        if (c->sh_world > 0) {   // a partitioned instance flushes its tile rows only
            std::vector<ekf::WtEntry> keep;
            for (const auto& v : wt) {
                const int r = (v.rc & 0xffff) * ekf::WT_R;
                if (r >= c->sh_r0 && r < c->sh_r1) keep.push_back(v);
            }
            wt.swap(keep);
        }
        c->nwt = (int)wt.size();
        if (hipMalloc((void**)&c->wt, sizeof(ekf::WtEntry) * wt.size()) != hipSuccess) goto fail;
        if (hipMemcpy(c->wt, wt.data(), sizeof(ekf::WtEntry) * wt.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
            goto fail;
        // the f64 wave flush: wave-tiles of 1 × WT64_C tiles, same panel walk
        std::vector<ekf::WtEntry> w64;
        const int nwc64 = (d.nb + ekf::WT64_C - 1) / ekf::WT64_C;
        for (int pc = 0; pc < nwc64; pc += 16)
            for (int wr = 0; wr < d.nb; wr++)
                for (int wc = pc; wc < pc + 16 && wc < nwc64; wc++) {
                    if (wc * ekf::WT64_C + ekf::WT64_C - 1 < wr) continue;
                    ekf::WtEntry v;
                    memset(&v, 0, sizeof(v));
                    const int fbj = std::min(wc * ekf::WT64_C + ekf::WT64_C - 1, d.nb - 1);   // stored
                    for (int cc = 0; cc < ekf::WT64_C; cc++) {
                        const int bj = wc * ekf::WT64_C + cc;
                        const bool ok = bj < d.nb && wr <= bj;
                        v.tile[cc] = (int)(ok ? ekf::tile_index(wr, bj, d.nb) : ekf::tile_index(wr, fbj, d.nb));
                        v.valid |= (ok ? 1 : 0) << cc;
                        v.rows[1] |= std::min(bj, d.nb - 1) << (16 * cc);
                    }
                    v.rows[0] = wr;
                    v.rc = wr | (wc << 16);
                    w64.push_back(v);
                }
        if (c->sh_world > 0) {
            std::vector<ekf::WtEntry> keep;
            for (const auto& v : w64)
                if (v.rows[0] >= c->sh_r0 && v.rows[0] < c->sh_r1) keep.push_back(v);
            w64.swap(keep);
        }
        c->nwt64 = (int)w64.size();
        if (hipMalloc((void**)&c->wt64, sizeof(ekf::WtEntry) * w64.size()) != hipSuccess) goto fail;
        if (hipMemcpy(c->wt64, w64.data(), sizeof(ekf::WtEntry) * w64.size(), hipMemcpyHostToDevice) !=
            hipSuccess)
            goto fail;
        // the split-bf16 flush's 2 × 4 wave-tiles holding a stored tile (4wc + 3 >= 2wr), in panels of
        // 8 wave-tile columns walked row by row (flush_bf24_kernel)
        std::vector<int> w24;
        const int nwr2 = (d.nb + 1) / 2, nwc4 = (d.nb + 3) / 4;
        for (int pc = 0; pc < nwc4; pc += 8)
            for (int wr = 0; wr < nwr2; wr++)
                for (int wc = pc; wc < pc + 8 && wc < nwc4; wc++)
                    if (4 * wc + 3 >= 2 * wr) w24.push_back(wr | (wc << 16));
        c->nwt24 = (int)w24.size();
        if (hipMalloc((void**)&c->wt24, sizeof(int) * w24.size()) != hipSuccess) goto fail;
        if (hipMemcpy(c->wt24, w24.data(), sizeof(int) * w24.size(), hipMemcpyHostToDevice) != hipSuccess)
            goto fail;
        // the split-fp16 quad form's groups of 2 × 2 wave-tiles holding a stored tile (group column
        // >= group row), in panels of 8 group columns walked row by row; entry 2a + b of a group is
        // its wave-tile (2R + a, 2C + b). Wave-tiles wholly below the diagonal or past the block stay
        // in their group (the group's operand rows are loaded alike): no valid tile, indices of a
        // stored tile of the group, rows clamped to the block. A partitioned context has none.
        if (c->sh_world <= 0) {
            std::vector<ekf::WtEntry> wq;
            const int ngr = (nwr + 1) / 2, ngc = (nwc + 1) / 2;
            for (int pc = 0; pc < ngc; pc += 8)
                for (int R = 0; R < ngr; R++)
                    for (int Cg = pc; Cg < pc + 8 && Cg < ngc; Cg++) {
                        if (Cg < R) continue;
                        // a stored tile of the group: its first tile row, last tile column in the block
                        const long long any = ekf::tile_index(4 * R, std::min(4 * Cg + 3, d.nb - 1), d.nb);
                        for (int a = 0; a < 2; a++)
                            for (int b = 0; b < 2; b++) {
                                const int wr = 2 * R + a, wc = 2 * Cg + b;
                                ekf::WtEntry v;
                                memset(&v, 0, sizeof(v));
                                for (int r = 0; r < ekf::WT_R; r++)
                                    for (int cc = 0; cc < ekf::WT_C; cc++) {
                                        const int i = r * ekf::WT_C + cc;
                                        const int bi = wr * ekf::WT_R + r, bj = wc * ekf::WT_C + cc;
                                        const bool ok = bi < d.nb && bj < d.nb && bi <= bj;
                                        v.tile[i] = (int)(ok ? ekf::tile_index(bi, bj, d.nb) : any);
                                        v.valid |= (ok ? 1 : 0) << i;
                                    }
                                for (int r = 0; r < ekf::WT_R; r++)
                                    v.rows[0] |= std::min(wr * ekf::WT_R + r, d.nb - 1) << (16 * r);
                                for (int cc = 0; cc < ekf::WT_C; cc++)
                                    v.rows[1] |= std::min(wc * ekf::WT_C + cc, d.nb - 1) << (16 * cc);
                                v.rc = wr | (wc << 16);
                                wq.push_back(v);
                            }
                    }
            c->nwtq = (int)wq.size();
            if (hipMalloc((void**)&c->wtq, sizeof(ekf::WtEntry) * wq.size()) != hipSuccess) goto fail;
            if (hipMemcpy(c->wtq, wq.data(), sizeof(ekf::WtEntry) * wq.size(), hipMemcpyHostToDevice) != hipSuccess)
                goto fail;
        }
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) goto fail;
        c->dd_per_cu = 8;   // downdate workgroups per CU (4 waves each; EKF_OPT_FLUSH_BLOCKS_PER_CU)
        c->dd_grid = prop.multiProcessorCount * c->dd_per_cu;
        c->ncu = prop.multiProcessorCount;
        // automatic flush form (EKF_OPT_FLUSH_FORM); a partitioned instance: the wave form for every
        // group (its wave tables hold the rank's tile rows only; the other forms walk every tile)
        c->dd_variant = c->sh_world > 0 ? 8 : 0;
        // all G workgroups of an instance must be co-resident (they exchange per line). A plain
        // launch gets the same residency as a cooperative one for the same grid
        // (cdna_hip_programming.md §1; the cooperative form only adds a launch-time check of the
        // same occupancy query, which can over-report, for ≈17 µs per launch), so the grid is
        // sized from a bound that cannot over-report: the LDS the kernel declares (one block per
        // CU at 128 KB of 160 KB), capped by the occupancy query less one block of margin when
        // the query allows more than one.
        int per_cu = ekf::scan_blocks_per_cu(cfg->precision);
        if (per_cu > 1) per_cu -= 1;
        const size_t lds = ekf::scan_lds_bytes(cfg->precision);
        if (lds > 0 && prop.maxSharedMemoryPerMultiProcessor > 0) {
            const int by_lds = (int)(prop.maxSharedMemoryPerMultiProcessor / lds);
            if (by_lds < per_cu) per_cu = by_lds;
        }
        if (per_cu < 1) {
            rc = EKF_EINVAL;
            goto fail;
        }
        const int resident = prop.multiProcessorCount * per_cu;
        c->resident = resident;
        c->scan_batch = resident / c->G;
        if (c->scan_batch < 1) {
            rc = EKF_EINVAL;   // one instance does not fit the device
            goto fail;
        }
        if (c->scan_batch > E) c->scan_batch = E;
    }
    c->base = c->last_out = 0;
    for (int e = 0; e < E; e++)
        if (set_robot_ctor(c, e, 0.0, 0.0, 0.0) != EKF_OK) goto fail;
    *out = c;
    return EKF_OK;
fail:
    free_all(c);
    delete c;
    return rc;
}

static void rccl_destroy(ekf_ctx* c);

extern "C" int ekf_destroy(ekf_ctx* c)
{
    if (!c) return EKF_EINVAL;
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->dstream);
    rccl_destroy(c);
    free_all(c);
    delete c;
    return EKF_OK;
}

extern "C" int ekf_set_stream(ekf_ctx* c, void* s)
{
    if (!c) return EKF_EINVAL;
    int rc = drain(c);
    if (rc) return rc;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return EKF_OK;
}

extern "C" int ekf_sync(ekf_ctx* c)
{
    if (!c) return EKF_EINVAL;
    return drain(c);
}

extern "C" int ekf_set_option(ekf_ctx* c, int opt, int v)
{
    if (!c) return EKF_EINVAL;
    const int E = c->cfg.instances;
    switch (opt) {
    case EKF_OPT_SPECULATE: if (v < 0 || v > 3) return EKF_ERANGE; break;
    case EKF_OPT_SPIN_LOG2: if (v < 8 || v > 24) return EKF_ERANGE; break;
    case EKF_OPT_FLUSH_FORM:
        if (v != 0 && v != 2 && v != 8 && v != 24 && v != 44) return EKF_ERANGE;
        // a partitioned context stores only its tile rows; only the wave forms walk the rank's
        // wave tables (the super-tile and tile forms walk every tile of the block)
        if (c->sh_world > 0 && v != 8) return EKF_EINVAL;
        break;
    case EKF_OPT_FLUSH_BLOCKS_PER_CU: if (v < 1 || v > 16) return EKF_ERANGE; break;
    case EKF_OPT_MFMA_REPLAY: if (v < 0 || v > 2) return EKF_ERANGE; break;
    case EKF_OPT_ACTIVE_FLUSH:
    case EKF_OPT_SCAN_STAMPS: if (v < 0 || v > 1) return EKF_ERANGE; break;
    case EKF_OPT_SCAN_THREADS: if (v != 0 && v != 64 && v != 128 && v != 192) return EKF_ERANGE; break;
    case EKF_OPT_TEST_DROP_WG:
    case EKF_OPT_TEST_VERDICT_TIMEOUT: if (v < 0 || v > E) return EKF_ERANGE; break;
    default: return EKF_EINVAL;
    }
    int rc = drain(c);
    if (rc) return rc;
    switch (opt) {
    case EKF_OPT_SPECULATE: c->spec = v; break;
    case EKF_OPT_SPIN_LOG2: c->spin_log2 = v; break;
    case EKF_OPT_FLUSH_FORM: c->dd_variant = v; break;
    case EKF_OPT_FLUSH_BLOCKS_PER_CU:
        c->dd_per_cu = v;
        c->dd_grid = c->ncu * v;
        break;
    case EKF_OPT_MFMA_REPLAY:
        c->mfrep_opt = v;
        c->mfrep = c->bf ? v : 0;
        break;
    case EKF_OPT_SCAN_STAMPS:
        if (v && !c->dbg) {
            const size_t bytes = sizeof(unsigned long long) * 32 * E;
            if (hipMalloc((void**)&c->dbg, bytes) != hipSuccess) {
                c->dbg = nullptr;
                return EKF_ENOMEM;
            }
            HIP_TRY(hipMemset(c->dbg, 0, bytes));
        } else if (!v && c->dbg) {
            HIP_TRY(hipFree(c->dbg));
            c->dbg = nullptr;
        }
        break;
    case EKF_OPT_TEST_DROP_WG: c->test_drop = v; break;
    case EKF_OPT_TEST_VERDICT_TIMEOUT: c->test_verdict = v; break;
    case EKF_OPT_ACTIVE_FLUSH: c->active_flush = v; break;
    case EKF_OPT_SCAN_THREADS: c->nt_opt = v; break;
    }
    return EKF_OK;
}

extern "C" int ekf_get_option(const ekf_ctx* c, int opt, int* v)
{
    if (!c || !v) return EKF_EINVAL;
    switch (opt) {
    case EKF_OPT_SPECULATE: *v = c->spec; break;
    case EKF_OPT_SPIN_LOG2: *v = c->spin_log2; break;
    case EKF_OPT_FLUSH_FORM: *v = c->dd_variant; break;
    case EKF_OPT_FLUSH_BLOCKS_PER_CU: *v = c->dd_per_cu; break;
    case EKF_OPT_MFMA_REPLAY: *v = c->mfrep_opt; break;
    case EKF_OPT_SCAN_STAMPS: *v = c->dbg ? 1 : 0; break;
    case EKF_OPT_TEST_DROP_WG: *v = c->test_drop; break;
    case EKF_OPT_TEST_VERDICT_TIMEOUT: *v = c->test_verdict; break;
    case EKF_OPT_ACTIVE_FLUSH: *v = c->active_flush; break;
    case EKF_OPT_SCAN_THREADS: *v = c->nt_opt; break;
    default: return EKF_EINVAL;
    }
    return EKF_OK;
}

extern "C" int ekf_reset_instance(ekf_ctx* c, int e, double x, double y, double th)
{
    if (c) c->mirror_epoch = 0;   // (the robot block changes without a scan)
    if (!c) return EKF_EINVAL;
    if (e >= c->cfg.instances) return EKF_ERANGE;
    int rc = drain(c);
    if (rc) return rc;
    if (e < 0) {
        for (int k = 0; k < c->cfg.instances; k++) {
            rc = set_robot_ctor(c, k, x, y, th);
            if (rc) return rc;
        }
        return EKF_OK;
    }
    return set_robot_ctor(c, e, x, y, th);
}

// profiling level 1 times the flush only (what the roofline needs, 2 events per group);
// level 2 also every association kernel. record = false: the caller hands the pair to the launch
// (hipExtLaunchKernelGGL timestamps the dispatch itself; no marker packets around the flush)
static EvPair* prof_begin(ekf_ctx* c, int kind, hipStream_t st, bool record = true)
{
    if (!c->prof || (kind == 0 && c->prof < 2)) return nullptr;
    EvPair pr;
    if (!c->pool.empty()) {
        pr = c->pool.back();
        c->pool.pop_back();
    } else {
        if (hipEventCreate(&pr.a) != hipSuccess) return nullptr;
        if (hipEventCreate(&pr.b) != hipSuccess) return nullptr;
    }
    c->ev[kind].push_back(pr);
    if (record) (void)hipEventRecord(pr.a, st);
    return &c->ev[kind].back();
}

static void prof_end(ekf_ctx* c, EvPair* pr, hipStream_t st)
{
    if (pr) (void)hipEventRecord(pr->b, st);
}

// Landmarks per association workgroup (EKF_OPT_SCAN_THREADS): the narrow widths exist for the
// HOT instantiations of the kernel only (symmetric fp32 / fp16 operands, kmax = 16, every flush
// arithmetic; launch_scan) and need the instance's workgroups
// within the speculative path's bound, no pipelined overlap and every instance in one launch.
// Automatic: the narrowest of 64 and 128 that fits (measured, DESIGN §4.1: N = 256 / 1024 / 2048
// +8 / +9 / +5 % updates/s at 64, N = 4096 with 8 instances +1.4 % at 128).
// Symmetric fp32 operands (sym_factor: every EKF_R_INTENDED fp32 / fp16 context; U = −2^x·V
// exactly): the association kernel stores the V rows only and every reader of U rows scales them
// (ScanParams / DowndateParams::usym). The partitioned instance stores both.
static int usym_of(const ekf_ctx* c)
{
    return c->sh_world == 0 && c->cfg.precision != EKF_PREC_F64 && c->cfg.r_mode == EKF_R_INTENDED;
}

static int scan_width(const ekf_ctx* c)
{
    constexpr int W = ekf::SCAN_THREADS;
    if (c->dbg || c->sh_world > 0 || c->cfg.precision == EKF_PREC_F64 || c->cfg.r_mode != EKF_R_INTENDED ||
        c->d.kmax != 16)
        return W;
    auto fits = [&](int nt) {
        const int G = (c->d.N + nt - 1) / nt;
        return G <= ekf::SPEC_GMAX && !(G > 1 && c->cfg.pipeline) && G * c->cfg.instances <= c->resident;
    };
    if (c->nt_opt) return c->nt_opt != W && fits(c->nt_opt) ? c->nt_opt : W;
    return fits(64) ? 64 : fits(128) ? 128 : W;
}

static ekf::ScanParams scan_params(ekf_ctx* c, int phase, const double* enc,
                                   const ekf_line* lines, const int* nlines)
{
    ekf::ScanParams p;
    memset(&p, 0, sizeof(p));
    p.d = c->d;
    p.E = c->cfg.instances;
    p.phase = phase;
    p.r_mode = c->cfg.r_mode;
    p.reset_margin = c->cfg.reset_margin;
    p.gate = c->cfg.mahalanobis;
    p.enc_noise = c->cfg.encoder_noise;
    p.Rs = c->Rs;
    p.y = c->y;
    p.live = c->cur;
    p.Dd = c->D;
    p.mfrep = c->mfrep;
    p.mfrep64 = (c->cfg.precision == EKF_PREC_F64 && c->mfrep_opt) ? 1 : 0;
    p.bf = c->pmode;
    p.psig = c->psig;
    p.pvmax = c->pvmax;
    p.Etot = c->cfg.instances;
    p.spin_log2 = c->spin_log2;
    p.test_drop = c->test_drop;
    p.test_verdict = c->test_verdict;
    p.pose = c->pose;
    p.xpre = c->xpre;
    p.saved = c->saved;
    p.enc = enc;
    p.lines = lines;
    p.nlines = nlines;
    p.dbg = c->dbg;
    p.pexp = c->pexp;
    p.nt = scan_width(c);
    p.usym = usym_of(c);
    p.G = (c->d.N + p.nt - 1) / p.nt;
    c->last_G = p.G;
    p.mbw = c->mbw;
    p.spec = c->spec;
    p.mbox = c->mbox;
    p.sync = c->sync;
    p.sync_stride = c->sync_stride;
    if (c->mirror_on) {
        p.res_host = c->hd_res;
        p.pose_host = c->hd_pose;
        p.r33_host = c->hd_r33;
        p.ep_host = c->hd_ep;
    }
    return p;
}

// The association kernel in batches of co-resident instances: grid (G, batch). Its per-line
// exchange counters are zeroed on the stream first.
static hipError_t launch_scans(ekf_ctx* c, ekf::ScanParams sp)
{
    const int E = c->cfg.instances;
    sp.epoch = ++c->scan_epoch;
    hipError_t err = hipSuccess;
    // (scan_width keeps a narrow launch within one batch)
    const int batch = sp.nt == ekf::SCAN_THREADS ? c->scan_batch : E;
    for (int e0 = 0; err == hipSuccess && e0 < E; e0 += batch) {
        sp.e0 = e0;
        sp.E = (E - e0 < batch) ? E - e0 : batch;
        err = ekf::launch_scan(sp, c->cfg.precision, c->stream);
    }
    return err;
}

static const ekf::Slot& slot_of(const ekf_ctx* c, long long k)
{
    return c->ring[(size_t)(k % (long long)c->ring.size())];
}

// One pass over the landmark block applying steps [unflushed0, nsteps) (stream D).
static int enqueue_flush(ekf_ctx* c)
{
    const int nst = (int)(c->nsteps - c->unflushed0);
    if (nst <= 0) return EKF_OK;
    // sequential schedule: the flush follows the scans on S (no cross-stream events); pipelined:
    // on D after the group's last scan
    hipStream_t fs = c->cfg.pipeline ? c->dstream : c->stream;
    if (c->cfg.pipeline) HIP_TRY(hipStreamWaitEvent(c->dstream, c->ev_scan, 0));
    ekf::DowndateParams dp;
    memset(&dp, 0, sizeof(dp));
    dp.d = c->d;
    dp.E = c->cfg.instances;
    dp.nsteps = nst;
    dp.variant = c->dd_variant;
    dp.ncu = c->ncu;
    dp.tile_rc = c->tile_rc;
    dp.stile_rc = c->stile_rc;
    dp.stile2_rc = c->stile2_rc;
    dp.nstiles2 = c->nstiles2;
    dp.wt = c->wt;
    dp.nwt = c->nwt;
    dp.wt64 = c->wt64;
    dp.nwt64 = c->nwt64;
    dp.wt24 = c->wt24;
    dp.nwt24 = c->nwt24;
    dp.wtq = c->wtq;
    dp.nwtq = c->nwtq;
    dp.pexp = c->pexp;
    dp.usym = usym_of(c);
    dp.sink = c->sink;
    dp.ubase = c->ops_u;
    dp.vbase = c->ops_v;
    dp.slot_bytes = c->slot_bytes;
    dp.nslots = (int)c->ring.size();
    dp.slot0 = (int)(c->unflushed0 % (long long)c->ring.size());
    dp.dbg = c->dbg;
    dp.bf = c->pmode;
    dp.bbase = c->ops_b;
    dp.bslot_bytes = c->bslot_bytes;
    for (int q = 0; q < nst; q++) dp.steps[q] = slot_of(c, c->unflushed0 + q);
    if (c->sh_world > 0 && c->cfg.precision == EKF_PREC_F32 && (nst & 1)) {
        // a partitioned instance flushes with the wave form only (even groups): pad with a step
        // that applies nothing
        dp.steps[nst] = c->sh_null;
        dp.nsteps = nst + 1;
    }
    const int in = c->last_out;
    const int out = c->cfg.pipeline ? 1 - in : in;
    dp.Pin = xview(c, in);
    dp.Pout = xview(c, out);
    // the association kernel's RES_ZMAX bound (partitioned contexts write other records). A
    // skipped wave-tile is neither loaded nor stored, so it stays valid only in place: a
    // double-buffered (pipelined) flush would leave X[out]'s copy from two flushes earlier
    dp.zskip = (c->active_flush && c->sh_world == 0 && in == out) ? 1 : 0;
    EvPair* pr = prof_begin(c, 1, fs, false);
    if (pr) c->ev_nsteps.push_back(nst);
    HIP_TRY(ekf::launch_downdate(dp, c->cfg.precision, c->dd_grid, fs, pr ? pr->a : nullptr,
                                 pr ? pr->b : nullptr));
    hipEvent_t ev = c->ev_flush[c->nflush & 1];
    if (c->cfg.pipeline) HIP_TRY(hipEventRecord(ev, fs));
    if (c->cfg.pipeline) {
        // next scans read X[in] (= output of the previous flush) with both groups pending
        c->base = in;
        c->ev_base = c->nflush > 0 ? c->ev_flush[(c->nflush - 1) & 1] : nullptr;
        c->pend0 = c->unflushed0;
    } else {
        c->base = in;
        c->ev_base = nullptr;   // same stream
        c->pend0 = c->nsteps;
    }
    c->last_out = out;
    c->unflushed0 = c->nsteps;
    c->nflush++;
    return EKF_OK;
}

// Enqueue one localize step (or its predict / update half).
static int enqueue(ekf_ctx* c, int phase, const double* enc, const ekf_line* lines,
                   const int* nlines)
{
    // a row-sharded context keeps only its own rows current: the whole-instance scan would read
    // stale ones (slam_ekf.h ekf_shard_abort)
    if (c->sh_world > 0) return EKF_EINVAL;
    ekf::ScanParams sp = scan_params(c, phase, enc, lines, nlines);
    if (!(phase & ekf::PHASE_UPDATE)) {
        EvPair* pr = prof_begin(c, 0, c->stream);
        HIP_TRY(launch_scans(c, sp));
        prof_end(c, pr, c->stream);
        return EKF_OK;
    }
    // X[base] and the ring slot this step reuses are released by the event guarding base
    if (c->ev_base) HIP_TRY(hipStreamWaitEvent(c->stream, c->ev_base, 0));
    const int np = (int)(c->nsteps - c->pend0);
    if (np > ekf::PMAX) return EKF_EINVAL;   // unreachable: T <= 24
    sp.Pread = xview(c, c->base);
    sp.npend = np;
    for (int q = 0; q < np; q++) sp.pend[q] = slot_of(c, c->pend0 + q);
    sp.cur = slot_of(c, c->nsteps);
    sp.Ust = c->Ust;
    sp.Vst = c->Vst;
    EvPair* pr = prof_begin(c, 0, c->stream);
    HIP_TRY(launch_scans(c, sp));
    prof_end(c, pr, c->stream);
    if (c->cfg.pipeline || c->mirror_on) HIP_TRY(hipEventRecord(c->ev_scan, c->stream));
    c->nsteps++;
    if (c->nsteps - c->unflushed0 >= c->T) return enqueue_flush(c);
    return EKF_OK;
}

static int stage_inputs(ekf_ctx* c, const double* enc, const ekf_line* lines, const int* nlines)
{
    const int E = c->cfg.instances;
    if (nlines)
        for (int e = 0; e < E; e++)
            if (nlines[e] < 0 || nlines[e] > c->d.max_lines) return EKF_ERANGE;
    // into the pinned staging buffer (once the previous copy out of it has been done), then one
    // stream-ordered copy of the sections given: the device buffers are rewritten after the
    // association kernels that read them
    if (c->in_pending) HIP_TRY(hipEventSynchronize(c->ev_in));
    size_t lo = c->in_bytes, hi = 0;
    if (enc) {
        memcpy(c->h_in, enc, sizeof(double) * 3 * E);
        lo = 0;
        hi = sizeof(double) * 3 * E;
    }
    if (lines) {
        memcpy(c->h_in + c->in_lines, lines, sizeof(ekf_line) * c->d.max_lines * E);
        lo = std::min(lo, c->in_lines);
        hi = c->in_nlines;
    }
    if (nlines) {
        memcpy(c->h_in + c->in_nlines, nlines, sizeof(int) * E);
        lo = std::min(lo, c->in_nlines);
        hi = c->in_bytes;
    }
    if (hi > lo) {
        HIP_TRY(hipMemcpyAsync(c->d_in + lo, c->h_in + lo, hi - lo, hipMemcpyHostToDevice, c->stream));
        HIP_TRY(hipEventRecord(c->ev_in, c->stream));
        c->in_pending = 1;
    }
    return EKF_OK;
}

static void fill_results(const ekf_ctx* c, ekf_result* out);

extern "C" int ekf_read_results(ekf_ctx* c, ekf_result* out)
{
    if (!c) return EKF_EINVAL;
    const int E = c->cfg.instances;
    if (c->nsteps == 0) {
        if (out) memset(out, 0, sizeof(ekf_result) * E);
        return EKF_OK;
    }
    HIP_TRY(hipMemcpyAsync(c->h_res, slot_of(c, c->nsteps - 1).res, sizeof(int) * ekf::RES_STRIDE * E,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_pose, c->pose, sizeof(double) * 3 * E, hipMemcpyDeviceToHost,
                           c->stream));
    std::vector<int> hs((size_t)c->sync_stride * E);
    HIP_TRY(hipMemcpyAsync(hs.data(), c->sync, sizeof(int) * hs.size(), hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    // every workgroup's completion word of the last association launch (commit_fold: a word of
    // another launch — a workgroup that never ran or never finished — reads as a timeout, not as
    // the status bits an earlier launch left in it). A partitioned context never launches the
    // association kernel (scan_epoch counts its shard runs, which write no completion words): its
    // status bits are already in the record SH_END wrote
    if (c->scan_epoch > 0 && c->sh_world <= 0)
        for (int e = 0; e < E; e++) {
            int st = 0;
            for (int gq = 0; gq < c->last_G; gq++)
                st = ekf::commit_fold(st, (unsigned)hs[(size_t)e * c->sync_stride + ekf::SYNC_WG0 + gq],
                                      c->scan_epoch);
            c->h_res[(size_t)e * ekf::RES_STRIDE + ekf::RES_STATUS] |= st & ekf::DONE_STATUS_MASK;
        }
    fill_results(c, out);
    return EKF_OK;
}

// ekf_result of every instance from the host copies of the last step's records and poses
static void fill_results(const ekf_ctx* c, ekf_result* out)
{
    const int E = c->cfg.instances;
    if (!out) return;
    for (int e = 0; e < E; e++) {
        const int* r = c->h_res + (size_t)e * ekf::RES_STRIDE;
        ekf_result& o = out[e];
        memset(&o, 0, sizeof(o));
        o.pose[0] = c->h_pose[3 * e];
        o.pose[1] = c->h_pose[3 * e + 1];
        o.pose[2] = c->h_pose[3 * e + 2];
        o.matches = r[ekf::RES_M];
        o.new_landmarks = r[ekf::RES_NEXTRA];
        o.saved = r[ekf::RES_SAVED];
        o.reset = r[ekf::RES_RESET];
        o.status = r[ekf::RES_STATUS];
        o.nlines = r[ekf::RES_NLINES];
        for (int i = 0; i < EKF_MAX_LINES; i++)
            o.match[i] = (i < o.nlines) ? r[ekf::RES_MATCH + i] : -1;
    }
}

// A synchronous call's update: the scan's lead mirrors a committed result into pinned host memory
// (ScanParams::res_host), so the call waits for the association kernel only (not for a flush queued
// behind it) and reads the result without a copy; the robot blocks it mirrored serve
// ekf_get_pose_cov until the next launch. Any instance without this launch's epoch in its mirror
// (a rollback, a lead that never finished) takes the copies and the host fold of ekf_read_results.
static int enqueue_mirrored(ekf_ctx* c, int phase, ekf_result* out)
{
    c->mirror_on = 1;
    const int rc = enqueue(c, phase, c->d_enc, c->d_lines, c->d_nlines);
    c->mirror_on = 0;
    if (rc) return rc;
    c->mirror_epoch = 0;
    HIP_TRY(hipEventSynchronize(c->ev_scan));
    const int E = c->cfg.instances;
    bool all = true;
    for (int e = 0; e < E; e++) all = all && __atomic_load_n(c->h_ep + e, __ATOMIC_ACQUIRE) == c->scan_epoch;
    if (!all) return ekf_read_results(c, out);
    c->mirror_epoch = c->scan_epoch;
    fill_results(c, out);
    return EKF_OK;
}

extern "C" int ekf_localize(ekf_ctx* c, const double* enc, const ekf_line* lines,
                            const int32_t* nlines, ekf_result* out)
{
    if (!c || !enc || !lines || !nlines || c->sh_world > 0) return EKF_EINVAL;
    int rc = stage_inputs(c, enc, lines, nlines);
    if (rc) return rc;
    return enqueue_mirrored(c, ekf::PHASE_BOTH, out);
}

extern "C" int ekf_localize_device(ekf_ctx* c, const double* d_enc, const ekf_line* d_lines,
                                   const int32_t* d_nlines)
{
    if (!c || !d_enc || !d_lines || !d_nlines) return EKF_EINVAL;
    return enqueue(c, ekf::PHASE_BOTH, d_enc, d_lines, d_nlines);
}

extern "C" int ekf_predict(ekf_ctx* c, const double* enc)
{
    if (!c || !enc || c->sh_world > 0) return EKF_EINVAL;
    int rc = stage_inputs(c, enc, nullptr, nullptr);
    if (rc) return rc;
    return enqueue(c, ekf::PHASE_PREDICT, c->d_enc, c->d_lines, c->d_nlines);
}

extern "C" int ekf_update(ekf_ctx* c, const ekf_line* lines, const int32_t* nlines,
                          ekf_result* out)
{
    if (!c || !lines || !nlines || c->sh_world > 0) return EKF_EINVAL;
    int rc = stage_inputs(c, nullptr, lines, nlines);
    if (rc) return rc;
    return enqueue_mirrored(c, ekf::PHASE_UPDATE, out);
}

// The dense n × n fp64 scratch of the state transfers: allocated on first use and kept, so that a
// caller mirroring P after every scan (the drop-in's full mirror) does not allocate per call
static hipError_t dense_scratch(ekf_ctx* c, double** out)
{
    if (!c->dense) {
        const hipError_t err = hipMalloc((void**)&c->dense, sizeof(double) * c->d.n * c->d.n);
        if (err != hipSuccess) {
            c->dense = nullptr;
            return err;
        }
    }
    *out = c->dense;
    return hipSuccess;
}

extern "C" int ekf_upload_state(ekf_ctx* c, int e, const double* P, const double* y, int saved,
                                const double pose[3])
{
    if (c) c->mirror_epoch = 0;   // (the robot block changes without a scan)
    if (!c) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    if (saved < 0 || saved > c->d.N) return EKF_ERANGE;
    int rc = drain(c);
    if (rc) return rc;
    const Dims& d = c->d;
    int cb = 0;
    rc = strip_copy(c, e, &cb);
    if (rc) return rc;
    if (P) {
        double vmax = 0.0;
        for (int i = 3; i < d.n; i++) vmax = std::max(vmax, std::fabs(P[(size_t)i * d.n + i]));
        rc = set_exponent(c, e, choose_exponent(c, vmax));
        if (rc) return rc;
        rc = set_plane_scale(c, e, vmax);
        if (rc) return rc;
        double* tmp = nullptr;
        HIP_TRY(dense_scratch(c, &tmp));
        hipError_t err = hipMemcpyAsync(tmp, P, sizeof(double) * d.n * d.n, hipMemcpyHostToDevice,
                                        c->stream);
        if (err == hipSuccess)
            err = ekf::launch_pack(d, c->cfg.precision, tmp, xinst_ptr(c, cur_buf(c), e),
                                   strip_of(c, cb, e), c->tile_rc, c->pexp_h[e], c->stream, c->t0, c->t1);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        HIP_TRY(err);
    }
    if (y)
        HIP_TRY(hipMemcpyAsync(mean_of(c, cb, e), y, sizeof(double) * d.n,
                               hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->saved + e, &saved, sizeof(int), hipMemcpyHostToDevice, c->stream));
    if (pose) {
        HIP_TRY(hipMemcpyAsync(c->pose + 3 * e, pose, sizeof(double) * 3, hipMemcpyHostToDevice,
                               c->stream));
        HIP_TRY(hipMemcpyAsync(c->xpre + 3 * e, pose, sizeof(double) * 3, hipMemcpyHostToDevice,
                               c->stream));
    }
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

extern "C" int ekf_download_state(ekf_ctx* c, int e, double* P, double* y, int* saved,
                                  double pose[3])
{
    if (!c) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    // P drains (the pending downdates are flushed first); the mean, pose and savedLineCount are
    // committed by every association kernel, so without P the call only waits for the stream and
    // leaves the flush schedule as it is
    int rc = EKF_OK;
    if (P) rc = drain(c);
    else HIP_TRY(hipStreamSynchronize(c->stream));
    if (rc) return rc;
    const Dims& d = c->d;
    int cb = 0;
    rc = strip_copy(c, e, &cb);
    if (rc) return rc;
    if (P) {
        double* tmp = nullptr;
        HIP_TRY(dense_scratch(c, &tmp));
        hipError_t err = ekf::launch_unpack(d, c->cfg.precision, tmp, xinst_ptr(c, cur_buf(c), e),
                                            strip_of(c, cb, e), c->pexp_h[e], c->stream, c->t0, c->t1);
        if (err == hipSuccess)
            err = hipMemcpyAsync(P, tmp, sizeof(double) * d.n * d.n, hipMemcpyDeviceToHost,
                                 c->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        HIP_TRY(err);
    }
    if (y)
        HIP_TRY(hipMemcpyAsync(y, mean_of(c, cb, e), sizeof(double) * d.n,
                               hipMemcpyDeviceToHost, c->stream));
    if (saved)
        HIP_TRY(hipMemcpyAsync(saved, c->saved + e, sizeof(int), hipMemcpyDeviceToHost, c->stream));
    if (pose)
        HIP_TRY(hipMemcpyAsync(pose, c->pose + 3 * e, sizeof(double) * 3, hipMemcpyDeviceToHost,
                               c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

extern "C" int ekf_init_lowrank(ekf_ctx* c, int e, const double* diag, const double* U, int rank,
                                const double* y, int saved, const double pose[3])
{
    if (c) c->mirror_epoch = 0;   // (the robot block changes without a scan)
    if (!c || !diag || (rank > 0 && !U) || rank < 0) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    int rc = drain(c);
    if (rc) return rc;
    const Dims& d = c->d;
    int cb = 0;
    rc = strip_copy(c, e, &cb);
    if (rc) return rc;
    double vmax = 0.0;
    for (int i = 3; i < d.n; i++) {
        double v = diag[i];
        for (int k = 0; k < rank; k++) v += U[(size_t)i * rank + k] * U[(size_t)i * rank + k];
        vmax = std::max(vmax, std::fabs(v));
    }
    rc = set_exponent(c, e, choose_exponent(c, vmax));
    if (rc) return rc;
    rc = set_plane_scale(c, e, vmax);
    if (rc) return rc;
    double *dd = nullptr, *du = nullptr;
    HIP_TRY(hipMalloc((void**)&dd, sizeof(double) * d.n));
    hipError_t err = hipMalloc((void**)&du, sizeof(double) * d.n * (rank > 0 ? rank : 1));
    if (err == hipSuccess)
        err = hipMemcpyAsync(dd, diag, sizeof(double) * d.n, hipMemcpyHostToDevice, c->stream);
    if (err == hipSuccess && rank > 0)
        err = hipMemcpyAsync(du, U, sizeof(double) * d.n * rank, hipMemcpyHostToDevice, c->stream);
    if (err == hipSuccess)
        err = ekf::launch_lowrank(d, c->cfg.precision, dd, du, rank, xinst_ptr(c, cur_buf(c), e),
                                  strip_of(c, cb, e), c->tile_rc, c->pexp_h[e], c->stream, c->t0, c->t1);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    (void)hipFree(dd);
    if (du) (void)hipFree(du);
    HIP_TRY(err);
    return ekf_upload_state(c, e, nullptr, y, saved, pose);
}

extern "C" int ekf_storage_exponent(const ekf_ctx* c, int e)
{
    if (!c) return 0;
    if (e < 0 || e >= c->cfg.instances) return 0;
    return c->pexp_h[e];
}

extern "C" int ekf_rescale(ekf_ctx* c, int e, int ex)
{
    if (c) c->mirror_epoch = 0;   // (the robot block changes without a scan)
    if (!c) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    if (c->cfg.precision != EKF_PREC_F16) return EKF_OK;
    if (ex != EKF_EXP_AUTO && (ex < -24 || ex > 24)) return EKF_ERANGE;
    int rc = drain(c);
    if (rc) return rc;
    const Dims& d = c->d;
    int cb = 0;
    rc = strip_copy(c, e, &cb);
    if (rc) return rc;
    void* X = xinst_ptr(c, cur_buf(c), e);
    double* Rs = strip_of(c, cb, e);
    double* tmp = nullptr;
    HIP_TRY(dense_scratch(c, &tmp));
    std::vector<double> dg(d.n);
    hipError_t err = ekf::launch_unpack(d, c->cfg.precision, tmp, X, Rs, c->pexp_h[e], c->stream);
    if (err == hipSuccess)   // the diagonal of the dense copy (stride n + 1)
        err = hipMemcpy2DAsync(dg.data(), sizeof(double), tmp, sizeof(double) * (d.n + 1), sizeof(double),
                               d.n, hipMemcpyDeviceToHost, c->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    if (err == hipSuccess) {
        double vmax = 0.0;
        for (int i = 3; i < d.n; i++) vmax = std::max(vmax, std::fabs(dg[i]));
        rc = set_exponent(c, e, ex == EKF_EXP_AUTO ? choose_exponent(c, vmax) : ex);
        if (rc == EKF_OK) rc = set_plane_scale(c, e, vmax);
        if (rc == EKF_OK) {
            err = ekf::launch_pack(d, c->cfg.precision, tmp, X, Rs, c->tile_rc, c->pexp_h[e], c->stream);
            if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        }
    }
    HIP_TRY(err);
    return rc;
}

extern "C" int ekf_get_pose_cov(ekf_ctx* c, int e, double P33[9])
{
    if (!c || !P33) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    if (c->mirror_epoch != 0 && c->mirror_epoch == c->scan_epoch) {
        // the robot block the last synchronous call's scan committed (no launch since)
        memcpy(P33, c->h_r33 + 9 * (size_t)e, sizeof(double) * 9);
        return EKF_OK;
    }
    const Dims& d = c->d;
    int cb = 0;
    const int rc = strip_copy(c, e, &cb);
    if (rc) return rc;
    for (int a = 0; a < 3; a++)
        HIP_TRY(hipMemcpyAsync(P33 + 3 * a, strip_of(c, cb, e) + (size_t)a * d.n,
                               sizeof(double) * 3, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

// ---- Robot::getEllipse (Robot.cpp:73-124) on the 2×2 pose block -------------------------
// The reference calls gsl_eigen_nonsymmv on [[P00, P01], [P10, P11]] (GSL is not vendored and its
// version is unpinned, CMakeLists.txt:43-51), sorts with GSL_EIGEN_SORT_ABS_ASC and publishes
// atan2(Re v0, Re v1) of the eigenvector of the larger |λ|. Restated from GSL's published
// algorithm (gsl/eigen/nonsymmv.c with its defaults: no balancing; gsl/eigen/francis.c):
//   * a 2×2 matrix is already Hessenberg (Z = I); the Francis QR of a 2×2 block is the
//     standardisation francis_schur_standardize (LAPACK dlanv2): [a b; c d] = Z [a' b'; 0 d'] Zᵀ
//     with Z = [[cs, -sn], [sn, cs]] (gsl_blas_drot applied to the columns of I);
//   * right eigenvectors of the Schur form by back substitution, x = (1, 0) for a' and
//     x = (-b'/(a'-d'), 1) for d' (denominator floored at smin), back-transformed v = Z·x and
//     scaled to unit 2-norm (gslcblas dnrm2) — positive scalings only, so the sign is Z's;
//   * eigenvalues in diagonal order (a', d'), then sorted by |λ| ascending (selection sort,
//     ties keep their order).
// A complex pair (c' != 0: not produced by a symmetric covariance block) returns 0.
namespace {
inline double gsl_sign(double x) { return x >= 0.0 ? 1.0 : -1.0; }

inline double gsl_hypot_(double x, double y)
{
    const double xa = fabs(x), ya = fabs(y);
    const double mn = xa < ya ? xa : ya, mx = xa < ya ? ya : xa;
    if (mn == 0.0) return mx;
    const double u = mn / mx;
    return mx * sqrt(1.0 + u * u);
}

inline double cblas_dnrm2_2(double x0, double x1)
{
    double scale = 0.0, ssq = 1.0;
    const double xs[2] = {x0, x1};
    for (int i = 0; i < 2; i++) {
        if (xs[i] != 0.0) {
            const double ax = fabs(xs[i]);
            if (scale < ax) {
                ssq = 1.0 + ssq * (scale / ax) * (scale / ax);
                scale = ax;
            } else {
                ssq += (ax / scale) * (ax / scale);
            }
        }
    }
    return scale * sqrt(ssq);
}

int gsl_ellipse_2x2(const double P[4], float axii[2], float* angle)
{
    for (int k = 0; k < 4; k++)
        if (!isfinite(P[k])) return 0;
    double a = P[0], b = P[1], c = P[2], d = P[3];
    double cs, sn;
    const double eps = 2.220446049250313e-16;   // GSL_DBL_EPSILON
    if (c == 0.0) {
        cs = 1.0;
        sn = 0.0;
    } else if (b == 0.0) {
        cs = 0.0;
        sn = 1.0;
        const double t = d;
        d = a;
        a = t;
        b = -c;
        c = 0.0;
    } else if ((a - d) == 0.0 && gsl_sign(b) != gsl_sign(c)) {
        cs = 1.0;
        sn = 0.0;
    } else {
        const double tmp = a - d;
        double p = 0.5 * tmp;
        const double bcmax = fmax(fabs(b), fabs(c));
        const double bcmis = fmin(fabs(b), fabs(c)) * gsl_sign(b) * gsl_sign(c);
        const double scale = fmax(fabs(p), bcmax);
        double z = (p / scale) * p + (bcmax / scale) * bcmis;
        if (z >= 4.0 * eps) {
            z = p + gsl_sign(p) * fabs(sqrt(scale) * sqrt(z));
            a = d + z;
            d -= (bcmax / z) * bcmis;
            const double tau = gsl_hypot_(c, z);
            cs = z / tau;
            sn = c / tau;
            b -= c;
            c = 0.0;
        } else {
            const double sigma = b + c;
            const double tau = gsl_hypot_(sigma, tmp);
            cs = sqrt(0.5 * (1.0 + fabs(sigma) / tau));
            sn = -(p / (tau * cs)) * gsl_sign(sigma);
            const double aa = a * cs + b * sn, bb = -a * sn + b * cs;
            const double cc = c * cs + d * sn, dd = -c * sn + d * cs;
            a = aa * cs + cc * sn;
            b = bb * cs + dd * sn;
            c = -aa * sn + cc * cs;
            d = -bb * sn + dd * cs;
            const double t2 = 0.5 * (a + d);
            a = d = t2;
            if (c != 0.0) {
                if (b != 0.0) {
                    if (gsl_sign(b) == gsl_sign(c)) {
                        const double sab = sqrt(fabs(b)), sac = sqrt(fabs(c));
                        p = gsl_sign(c) * fabs(sab * sac);
                        const double tau2 = 1.0 / sqrt(fabs(b + c));
                        a = t2 + p;
                        d = t2 - p;
                        b -= c;
                        c = 0.0;
                        const double cs1 = sab * tau2, sn1 = sac * tau2;
                        const double t3 = cs * cs1 - sn * sn1;
                        sn = cs * sn1 + sn * cs1;
                        cs = t3;
                    }
                } else {
                    b = -c;
                    c = 0.0;
                    const double t3 = cs;
                    cs = -sn;
                    sn = t3;
                }
            }
        }
    }
    if (c != 0.0) return 0;   // complex pair
    // eigenvectors: Z = [[cs, -sn], [sn, cs]]
    double v[2][2];
    v[0][0] = cs;
    v[0][1] = sn;
    {
        const double smlnum = 2.2250738585072014e-308 * (2.0 / eps);
        const double smin = fmax(eps * fabs(d), smlnum);
        double den = a - d;
        if (fabs(den) < smin) den = smin;
        const double x0 = -b / den;
        v[1][0] = x0 * cs + (-sn);
        v[1][1] = x0 * sn + cs;
    }
    for (int k = 0; k < 2; k++) {
        // back substitution ends with a max-norm scaling (as LAPACK dtrevc), the workspace
        // normalises to unit 2-norm afterwards (nonsymmv_normalize_eigenvectors)
        const double emax = fmax(fabs(v[k][0]), fabs(v[k][1]));
        if (emax > 0.0) {
            const double remax = 1.0 / emax;
            v[k][0] *= remax;
            v[k][1] *= remax;
        }
        const double nr = cblas_dnrm2_2(v[k][0], v[k][1]);
        if (nr > 0.0) {
            const double sc = 1.0 / nr;
            v[k][0] *= sc;
            v[k][1] *= sc;
        }
    }
    double lam[2] = {a, d};
    int ord[2] = {0, 1};
    if (fabs(lam[1]) < fabs(lam[0])) {
        ord[0] = 1;
        ord[1] = 0;
    }
    for (int i = 0; i < 2; i++) axii[i] = 2.f * (float)sqrt(5.991 * fabs(lam[ord[i]]));
    *angle = (float)atan2(v[ord[1]][0], v[ord[1]][1]);
    return 1;
}
}  // namespace

extern "C" int ekf_ellipse_of_block(const double P22[4], float axii[2], float* angle)
{
    if (!P22 || !axii || !angle) return -EKF_EINVAL;
    return gsl_ellipse_2x2(P22, axii, angle);
}

extern "C" int ekf_get_ellipse(ekf_ctx* c, int e, float axii[2], float* angle)
{
    // Robot::getEllipse (Robot.cpp:73-124) on P_t0[0:2, 0:2] of instance e (see above)
    if (!c || !axii || !angle) return -EKF_EINVAL;
    double P33[9];
    int rc = ekf_get_pose_cov(c, e, P33);
    if (rc) return -rc;
    const double P22[4] = {P33[0], P33[1], P33[3], P33[4]};
    return gsl_ellipse_2x2(P22, axii, angle);
}

extern "C" size_t ekf_landmark_block_bytes(const ekf_ctx* c)
{
    return c ? c->xinst * c->elem : 0;
}

extern "C" int ekf_state_dim(const ekf_ctx* c) { return c ? c->d.n : 0; }

// ---------------------------------------------------------------------------------------
// One instance with its landmark block partitioned over ranks: this
// context (ekf_shard_create) stores the packed tiles of its tile rows only; the scan runs as
// phases of ekf::shard_kernel over every landmark (replicated state), and the caller sums the
// [N][4] exchange buffer over the ranks between phases: the diagonal blocks after begin, the
// winner's column after each line. Everything is stream-ordered on the context stream: no host
// round trip until ekf_shard_end.

static ekf::ShardParams shard_params(ekf_ctx* c, int phase, double* buf, double* cols = nullptr)
{
    ekf::ShardParams p;
    memset(&p, 0, sizeof(p));
    p.d = c->d;
    p.phase = phase;
    p.line = c->sh_line;
    p.L = c->sh_L;
    p.r_mode = c->cfg.r_mode;
    p.gate = c->cfg.mahalanobis;
    p.enc_noise = c->cfg.encoder_noise;
    const int np = (int)(c->nsteps - c->pend0);
    p.npend = np;
    p.Pread = xview(c, c->base);
    p.t0 = c->t0;
    p.t1 = c->t1;
    for (int q = 0; q < np; q++) p.pend[q] = slot_of(c, c->pend0 + q);
    p.cur = slot_of(c, c->nsteps);
    p.Rs = strip_of(c, 0, 0);
    p.y = mean_of(c, 0, 0);
    p.pose = c->pose;
    p.saved = c->saved;
    p.rob = c->sh_rob;
    p.rec = c->sh_rec;
    p.hist = c->sh_hist;
    p.flags = c->sh_flags;
    p.pkg = c->sh_pkg;
    p.ctl = c->sh_ctl;
    p.col = buf;
    p.cols = cols;
    p.enc = c->d_enc;
    p.lines = c->d_lines;
    p.pexp = c->pexp;
    p.reset_margin = c->cfg.reset_margin;
    return p;
}

// a HIP failure inside a scan abandons it (slam_ekf.h ekf_shard_abort)
#define SH_TRY(expr)                                                                        \
    do {                                                                                    \
        hipError_t _e = (expr);                                                             \
        if (_e != hipSuccess) {                                                             \
            fprintf(stderr, "slam_ekf: %s failed: %s\n", #expr, hipGetErrorString(_e));     \
            c->sh_open = 0;                                                                 \
            return EKF_EDEVICE;                                                             \
        }                                                                                   \
    } while (0)

extern "C" int ekf_shard_tiles(const ekf_ctx* c, int* row_begin, int* row_end)
{
    if (!c || c->sh_world <= 0 || !row_begin || !row_end) return EKF_EINVAL;
    *row_begin = c->sh_r0;
    *row_end = c->sh_r1;
    return EKF_OK;
}

extern "C" size_t ekf_shard_buffer_words(const ekf_ctx* c) { return (c && c->sh_world > 0) ? 4 * (size_t)c->d.N : 0; }

extern "C" int ekf_shard_begin(ekf_ctx* c, const double enc[3], const ekf_line* lines, int nlines, double* buf)
{
    if (!c || c->sh_world <= 0 || !enc || !buf || (nlines > 0 && !lines) || c->sh_open) return EKF_EINVAL;
    if (nlines < 0 || nlines > c->d.max_lines) return EKF_ERANGE;
    c->sh_line = 0;
    c->sh_L = nlines;
    c->sh_open = 1;
    c->sh_diag = 0;
    // the inputs travel as kernel arguments of the first phase, which stores them for the later
    // ones (stream-ordered: no host staging copy, no wait for the previous scan)
    ekf::ShardParams p = shard_params(c, ekf::SH_BEGIN, buf);
    for (int k = 0; k < 3; k++) p.enc_v[k] = enc[k];
    for (int i = 0; i < c->d.max_lines; i++) {
        if (i < nlines) p.lines_v[i] = lines[i];
        else memset(&p.lines_v[i], 0, sizeof(ekf_line));
    }
    SH_TRY(ekf::launch_shard(p, c->cfg.precision, c->stream));
    return EKF_OK;
}

extern "C" int ekf_shard_line(ekf_ctx* c, int line, double* buf)
{
    if (!c || c->sh_open != 1 || !buf || line != c->sh_line) return EKF_EINVAL;
    if (line < 0 || line >= c->sh_L) return EKF_ERANGE;
    if (!c->sh_diag) {   // the summed diagonal blocks of begin's exchange
        SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_DIAG, buf), c->cfg.precision, c->stream));
        c->sh_diag = 1;
    }
    SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_GATE, buf), c->cfg.precision, c->stream));
    SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_COLUMN, buf), c->cfg.precision, c->stream));
    return EKF_OK;
}

extern "C" int ekf_shard_apply(ekf_ctx* c, int line, const double* buf)
{
    if (!c || c->sh_open != 1 || !buf || line != c->sh_line) return EKF_EINVAL;
    double* b = const_cast<double*>(buf);   // (read only by these phases)
    SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_APPLY, b), c->cfg.precision, c->stream));
    SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_ROBOT, b), c->cfg.precision, c->stream));
    c->sh_line++;
    return EKF_OK;
}

extern "C" size_t ekf_shard_spec_buffer_words(const ekf_ctx* c)
{
    return (c && c->sh_world > 0) ? 4 * (size_t)c->d.N * (size_t)c->d.max_lines : 0;
}

extern "C" int ekf_shard_speculate(ekf_ctx* c, const double* buf, double* cols)
{
    if (!c || c->sh_open != 1 || !buf || !cols || c->sh_line != 0 || c->sh_L == 0) return EKF_EINVAL;
    double* b = const_cast<double*>(buf);   // (read only by SH_DIAG)
    ekf::ShardParams pg = shard_params(c, ekf::SH_GUESS, b);
    pg.diag_first = !c->sh_diag;   // (SH_DIAG fused into the guesses' launch)
    c->sh_diag = 1;
    SH_TRY(ekf::launch_shard(pg, c->cfg.precision, c->stream));
    if (c->spec == 2)   // test hook (EKF_OPT_SPECULATE = 2): every line guesses landmark 0
        SH_TRY(hipMemsetAsync(c->sh_ctl + ekf::SC_GUESS, 0, sizeof(int) * c->d.max_lines, c->stream));
    SH_TRY(ekf::launch_shard(shard_params(c, ekf::SH_SPEC_COLS, b, cols), c->cfg.precision, c->stream));
    return EKF_OK;
}

extern "C" int ekf_shard_run(ekf_ctx* c, const double* cols, double* next_line)
{
    if (!c || c->sh_open != 1 || !cols || !next_line || !c->sh_diag || c->sh_line != 0 || c->sh_L == 0)
        return EKF_EINVAL;
    ekf::ShardParams p = shard_params(c, ekf::SH_GATE, nullptr, const_cast<double*>(cols));
    p.next_out = next_line;
    // the run's workgroups exchange through the association kernel's mailbox (unused by a
    // partitioned context: ⌈N/64⌉ ≥ shard_run_workgroups(N) slots per parity)
    p.mbox = c->mbox;
    p.mbw = c->mbw;
    p.epoch = ++c->scan_epoch;
    p.spin_log2 = c->spin_log2;
    SH_TRY(ekf::launch_shard_run(p, c->cfg.precision, c->stream));
    c->sh_line = -1;   // until ekf_shard_resume
    return EKF_OK;
}

extern "C" int ekf_shard_resume(ekf_ctx* c, int line)
{
    if (!c || c->sh_open != 1 || c->sh_line != -1 || line < 0 || line > c->sh_L) return EKF_EINVAL;
    c->sh_line = line;
    return EKF_OK;
}

// SH_END with its results mirrored into the pinned host buffers (one instance), so the result
// needs no copy: only the wait for this kernel, not for a flush behind it. gate (ekf_shard_localize):
// the ranks' agreement [failure flag, stopping line] on the device; the phase commits only if it
// says every line ran, and mirrors the pair into h_agree either way
static int shard_end_launch(ekf_ctx* c, const double* gate)
{
    ekf::ShardParams p = shard_params(c, ekf::SH_END, nullptr);
    int* rh = nullptr;
    double* ph = nullptr;
    HIP_TRY(hipHostGetDevicePointer((void**)&rh, c->h_res, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&ph, c->h_pose, 0));
    p.res_host = rh;
    p.pose_host = ph;
    if (gate) {
        double* ah = nullptr;
        HIP_TRY(hipHostGetDevicePointer((void**)&ah, c->h_agree, 0));
        p.end_gate = gate;
        p.end_gate_host = ah;
    }
    SH_TRY(ekf::launch_shard(p, c->cfg.precision, c->stream));
    HIP_TRY(hipEventRecord(c->ev_scan, c->stream));
    return EKF_OK;
}

// after a committed SH_END: the step joins the deferred flush of the rank's tiles; the results
// from the mirror once the phase has finished (flushed: the wait was before the flush's launch)
static int shard_end_finish(ekf_ctx* c, ekf_result* out, bool waited)
{
    c->sh_open = 0;
    c->nsteps++;
    if (c->nsteps - c->unflushed0 >= c->T) {
        const int rc = enqueue_flush(c);
        if (rc) return rc;
    }
    if (!waited) HIP_TRY(hipEventSynchronize(c->ev_scan));
    fill_results(c, out);
    return EKF_OK;
}

extern "C" int ekf_shard_end(ekf_ctx* c, ekf_result* out)
{
    if (!c || c->sh_open != 1 || c->sh_line != c->sh_L) return EKF_EINVAL;
    // (with no line, begin's exchange is not consumed: the end needs no diagonal block)
    const int rc = shard_end_launch(c, nullptr);
    if (rc) return rc;
    return shard_end_finish(c, out, false);
}

extern "C" int ekf_shard_abort(ekf_ctx* c)
{
    // before ekf_shard_end nothing of the committed state is written (the phases use the scan's
    // scratch and the current ring slot, which only ekf_shard_end adds to the schedule)
    if (!c || c->sh_world <= 0) return EKF_EINVAL;
    c->sh_open = 0;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

// The partitioned instance's scan as one call (ekf_shard_localize): the protocol above with the
// exchanges on the library's own RCCL communicator (ekf_shard_attach_rccl), so a C++ host (the
// drop-in Robot over ranks) needs no collective library of its own and a scan costs one call, two
// host reads (the agreement pair, then the results) and no host staging. RCCL is loaded on first
// use (dlopen): the library itself does not depend on it.
namespace {
struct RcclApi {
    ncclResult_t (*get_unique_id)(ncclUniqueId*);
    ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int);
    ncclResult_t (*all_reduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t);
    ncclResult_t (*comm_destroy)(ncclComm_t);
    const char* (*error_string)(ncclResult_t);
};
const RcclApi* rccl_api()
{
    static RcclApi api;
    static int state = 0;   // 0 not tried, 1 loaded, -1 unavailable (one thread: the context's)
    if (state == 0) {
        state = -1;
        void* h = nullptr;
        for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if ((h = dlopen(name, RTLD_NOW | RTLD_LOCAL)) != nullptr) break;
        if (h) {
            api.get_unique_id = (decltype(api.get_unique_id))dlsym(h, "ncclGetUniqueId");
            api.comm_init_rank = (decltype(api.comm_init_rank))dlsym(h, "ncclCommInitRank");
            api.all_reduce = (decltype(api.all_reduce))dlsym(h, "ncclAllReduce");
            api.comm_destroy = (decltype(api.comm_destroy))dlsym(h, "ncclCommDestroy");
            api.error_string = (decltype(api.error_string))dlsym(h, "ncclGetErrorString");
            if (api.get_unique_id && api.comm_init_rank && api.all_reduce && api.comm_destroy && api.error_string)
                state = 1;
        }
        if (state != 1) fprintf(stderr, "slam_ekf: RCCL (librccl.so) not available\n");
    }
    return state == 1 ? &api : nullptr;
}
}  // namespace

static void rccl_destroy(ekf_ctx* c)
{
    const RcclApi* r = c->rccl_comm ? rccl_api() : nullptr;
    if (r) (void)r->comm_destroy((ncclComm_t)c->rccl_comm);
    c->rccl_comm = nullptr;
}

extern "C" int ekf_rccl_unique_id(unsigned char out[128])
{
    const RcclApi* r = rccl_api();
    if (!out) return EKF_EINVAL;
    if (!r) return EKF_EDEVICE;
    ncclUniqueId id;
    if (r->get_unique_id(&id) != ncclSuccess) return EKF_EDEVICE;
    static_assert(sizeof(id) == 128, "ncclUniqueId");
    memcpy(out, &id, sizeof(id));
    return EKF_OK;
}

extern "C" int ekf_shard_attach_rccl(ekf_ctx* c, const unsigned char id[128], int rank, int world)
{
    if (!c || c->sh_world <= 0 || !id || rank != c->sh_rank || world != c->sh_world || c->sh_open) return EKF_EINVAL;
    const RcclApi* r = rccl_api();
    if (!r) return EKF_EDEVICE;
    HIP_TRY(hipSetDevice(c->device));
    rccl_destroy(c);
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm;
    const ncclResult_t e = r->comm_init_rank(&comm, world, uid, rank);
    if (e != ncclSuccess) {
        fprintf(stderr, "slam_ekf: ncclCommInitRank: %s\n", r->error_string(e));
        return EKF_EDEVICE;
    }
    c->rccl_comm = comm;
    const size_t words = 4 * (size_t)c->d.N, swords = words * (size_t)c->d.max_lines;
    if (!c->sh_xbuf || !c->sh_xcols || !c->h_agree) {
        // all three or none: a failure part way frees what was allocated, so a later attach
        // allocates again instead of finding one pointer set and the others null
        auto drop = [c]() {
            if (c->sh_xbuf) (void)hipFree(c->sh_xbuf);
            if (c->sh_xcols) (void)hipFree(c->sh_xcols);
            if (c->h_agree) (void)hipHostFree(c->h_agree);
            c->sh_xbuf = c->sh_xcols = c->h_agree = nullptr;
        };
        drop();
        if (hipMalloc((void**)&c->sh_xbuf, sizeof(double) * (words + 1)) != hipSuccess ||
            hipMalloc((void**)&c->sh_xcols, sizeof(double) * (swords + 2)) != hipSuccess ||
            hipHostMalloc((void**)&c->h_agree, sizeof(double) * 4) != hipSuccess ||
            hipMemset(c->sh_xbuf, 0, sizeof(double) * (words + 1)) != hipSuccess ||
            hipMemset(c->sh_xcols, 0, sizeof(double) * (swords + 2)) != hipSuccess) {
            drop();
            rccl_destroy(c);
            return EKF_EDEVICE;
        }
    }
    c->sh_dirty = 0;
    return EKF_OK;
}

extern "C" int ekf_shard_localize(ekf_ctx* c, const double enc[3], const ekf_line* lines, int nlines, ekf_result* out)
{
    if (!c || c->sh_world <= 0 || !c->rccl_comm || !enc || (nlines > 0 && !lines) || c->sh_open) return EKF_EINVAL;
    if (nlines < 0 || nlines > c->d.max_lines) return EKF_ERANGE;
    const RcclApi* r = rccl_api();
    const int L = nlines;
    const size_t words = 4 * (size_t)c->d.N, swords = words * (size_t)c->d.max_lines;
    double* buf = c->sh_xbuf;
    double* cols = c->sh_xcols;
    double* agree = cols + swords;   // [failure flag (the columns' flag word), stopping line]
    ncclComm_t comm = (ncclComm_t)c->rccl_comm;
    auto sum = [&](double* b, size_t n, ncclRedOp_t op) {
        return r->all_reduce(b, b, n, ncclFloat64, op, comm, c->stream) == ncclSuccess;
    };
    // a phase that fails on one rank must not leave the others waiting in an exchange: every rank
    // runs the whole exchange sequence, a failed one without further phases, and the summed flag
    // words tell every rank alike whether to abandon the scan
    static const double one_l[2] = {1.0, 0.0};
    auto flag = [&](double* w) {
        c->sh_dirty = 1;
        return hipMemcpyAsync(w, one_l, sizeof(double), hipMemcpyHostToDevice, c->stream) == hipSuccess;
    };
    if (c->sh_dirty) {
        HIP_TRY(hipMemsetAsync(buf + words, 0, sizeof(double), c->stream));
        HIP_TRY(hipMemsetAsync(agree, 0, 2 * sizeof(double), c->stream));
        c->sh_dirty = 0;
    }
    int err = ekf_shard_begin(c, enc, lines, L, buf);
    if (err && !flag(buf + words)) return EKF_EDEVICE;
    if (!sum(buf, words + 1, ncclSum)) return EKF_EDEVICE;
    int first = 0;
    bool abandon = false, spec_all = false;
    if (c->spec && L > 0) {
        if (!err) err = ekf_shard_speculate(c, buf, cols);
        if (err && !flag(agree)) return EKF_EDEVICE;
        if (!sum(cols, swords + 1, ncclSum)) return EKF_EDEVICE;
        if (!err) err = ekf_shard_run(c, cols, agree + 1);
        if (err) {
            const double v[2] = {1.0, (double)L};
            HIP_TRY(hipMemcpyAsync(agree, v, sizeof(v), hipMemcpyHostToDevice, c->stream));
            c->sh_dirty = 1;
        }
        if (!sum(agree, 2, ncclMax)) return EKF_EDEVICE;
        // the end phase goes behind the run before the host reads the agreement: it commits only if
        // every line ran on every rank (the common case: one host round trip per scan), and leaves
        // everything untouched otherwise, when the lines from the agreed one follow as below
        bool gated = false;
        if (!err) {
            c->sh_line = L;
            err = shard_end_launch(c, agree);
            gated = !err;
        }
        if (!gated)
            HIP_TRY(hipMemcpyAsync(c->h_agree, agree, 2 * sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        abandon = c->h_agree[0] > 0.0 || c->h_agree[1] > (double)L;   // (past L: a run timed out)
        first = abandon ? L : (int)c->h_agree[1];
        if (gated && !abandon && first == L) return shard_end_finish(c, out, true);
        if (gated) c->sh_line = -1;   // (not committed: the run's state stands, as after ekf_shard_run)
        // (host bookkeeping only, on the agreed line: it fails on every rank alike or on none)
        if (!abandon && !err) err = ekf_shard_resume(c, first);
        spec_all = first == L;
    }
    for (int i = first; i < L; i++) {
        if (!err) err = ekf_shard_line(c, i, buf);
        if (err && !flag(buf + words)) return EKF_EDEVICE;
        if (!sum(buf, words + 1, ncclSum)) return EKF_EDEVICE;
        if (!err) err = ekf_shard_apply(c, i, buf);
    }
    double failed;
    if (spec_all) {
        failed = c->h_agree[0];   // (the agreement carried every failure flag)
    } else {
        if (L > first) {
            // the last line's apply ran after its exchange: one more word, the MAX over the ranks
            // of the summed flags and of every rank's failure since, so that a rank whose apply
            // failed does not abandon the scan alone while its peers commit it
            if (err && !flag(buf + words)) return EKF_EDEVICE;
            if (!sum(buf + words, 1, ncclMax)) return EKF_EDEVICE;
        }
        HIP_TRY(hipMemcpyAsync(c->h_agree + 2, buf + words, sizeof(double), hipMemcpyDeviceToHost, c->stream));
        HIP_TRY(hipStreamSynchronize(c->stream));
        failed = c->h_agree[2];
    }
    if (abandon || failed > 0.0 || err) {
        c->sh_dirty = 1;
        (void)ekf_shard_abort(c);
        return err ? err : EKF_EDEVICE;   // (a peer's phase failed, or the run's exchange timed out)
    }
    return ekf_shard_end(c, out);
}

extern "C" int ekf_profile_enable(ekf_ctx* c, int enable)
{
    if (!c) return EKF_EINVAL;
    (void)hipStreamSynchronize(c->stream);
    (void)hipStreamSynchronize(c->dstream);
    for (auto& v : c->ev) {
        for (auto& pr : v) c->pool.push_back(pr);
        v.clear();
    }
    c->ev_nsteps.clear();
    c->prof = enable < 0 ? 0 : (enable > 2 ? 2 : enable);
    return EKF_OK;
}

extern "C" int ekf_profile_read(ekf_ctx* c, double* scan_ms, double* dd_ms, double* aug_ms,
                                int* launches)
{
    if (!c) return EKF_EINVAL;
    HIP_TRY(hipStreamSynchronize(c->stream));
    HIP_TRY(hipStreamSynchronize(c->dstream));
    double avg[3] = {0, 0, 0};
    for (int k = 0; k < 3; k++) {
        double sum = 0;
        for (auto& pr : c->ev[k]) {
            float ms = 0;
            HIP_TRY(hipEventElapsedTime(&ms, pr.a, pr.b));
            sum += ms;
        }
        avg[k] = c->ev[k].empty() ? 0.0 : sum / (double)c->ev[k].size();
    }
    if (scan_ms) *scan_ms = avg[0];
    if (dd_ms) *dd_ms = avg[1];
    if (aug_ms) *aug_ms = avg[2];
    if (launches) *launches = (int)c->ev[1].size();
    return EKF_OK;
}

extern "C" int ekf_profile_flushes(ekf_ctx* c, int cap, int* nsteps, float* ms)
{
    if (!c || cap < 0 || (cap > 0 && (!nsteps || !ms))) return -EKF_EINVAL;
    if (hipStreamSynchronize(c->stream) != hipSuccess || hipStreamSynchronize(c->dstream) != hipSuccess)
        return -EKF_EDEVICE;
    const int n = (int)c->ev[1].size();
    for (int k = 0; k < n && k < cap; k++) {
        float t = 0.f;
        if (hipEventElapsedTime(&t, c->ev[1][k].a, c->ev[1][k].b) != hipSuccess) return -EKF_EDEVICE;
        ms[k] = t;
        nsteps[k] = k < (int)c->ev_nsteps.size() ? c->ev_nsteps[k] : 0;
    }
    return n;
}

extern "C" const char* ekf_flush_kernel_name(const ekf_ctx* c, int nsteps)
{
    if (!c || nsteps < 1) return "";
    if (c->cfg.precision == EKF_PREC_F64) {
        static const char* f64w[ekf::F64_WAVE_MAXS + 1] = {
            "", "flush_f64_wave_kernel<1>", "flush_f64_wave_kernel<2>", "flush_f64_wave_kernel<3>",
            "flush_f64_wave_kernel<4>", "flush_f64_wave_kernel<5>", "flush_f64_wave_kernel<6>",
            "flush_f64_wave_kernel<7>", "flush_f64_wave_kernel<8>"};
        if (nsteps <= ekf::F64_WAVE_MAXS && c->d.kmax == 16 && c->dd_variant != 2) return f64w[nsteps];
        return "downdate_f64_kernel";
    }
    const bool half = c->cfg.precision == EKF_PREC_F16;
    if (c->pmode == EKF_ARITH_F16X3 && nsteps >= 2 && nsteps <= ekf::F16X3_MAXS && nsteps % 2 == 0) {
        struct Names {
            char n[3][2][ekf::F16X3_MAXS / 2 + 1][64];
            Names()
            {
                static const char* fmt[3] = {"flush_f32_wave_kernel<%s, %d, true, true>", "flush_bf24_kernel<%s, %d, true>",
                                             "flush_f16q_kernel<%s, %d>"};
                for (int f = 0; f < 3; f++)
                    for (int h = 0; h < 2; h++)
                        for (int k = 0; k <= ekf::F16X3_MAXS / 2; k++)
                            snprintf(n[f][h][k], sizeof n[f][h][k], fmt[f], h ? "_Float16" : "float", 2 * k);
            }
        };
        static const Names f16n;   // (initialised once, thread-safe)
        const int form = c->dd_variant == 24 ? 1 : (c->dd_variant == 44 && nsteps >= 6 && c->nwtq > 0) ? 2 : 0;
        return f16n.n[form][half ? 1 : 0][nsteps / 2];
    }
    if (c->bf && nsteps >= 2 && nsteps <= 16 && nsteps % 2 == 0 && c->dd_variant == 24) {
        static const char* b24[2][9] = {
            {"", "flush_bf24_kernel<float, 2>", "flush_bf24_kernel<float, 4>", "flush_bf24_kernel<float, 6>",
             "flush_bf24_kernel<float, 8>", "flush_bf24_kernel<float, 10>", "flush_bf24_kernel<float, 12>",
             "flush_bf24_kernel<float, 14>", "flush_bf24_kernel<float, 16>"},
            {"", "flush_bf24_kernel<_Float16, 2>", "flush_bf24_kernel<_Float16, 4>", "flush_bf24_kernel<_Float16, 6>",
             "flush_bf24_kernel<_Float16, 8>", "flush_bf24_kernel<_Float16, 10>", "flush_bf24_kernel<_Float16, 12>",
             "flush_bf24_kernel<_Float16, 14>", "flush_bf24_kernel<_Float16, 16>"}};
        return b24[half ? 1 : 0][nsteps / 2];
    }
    if (c->bf && nsteps >= 2 && nsteps <= 16 && nsteps % 2 == 0) {
        static const char* bfn[2][9] = {
            {"", "flush_f32_wave_kernel<float, 2, true>", "flush_f32_wave_kernel<float, 4, true>",
             "flush_f32_wave_kernel<float, 6, true>", "flush_f32_wave_kernel<float, 8, true>",
             "flush_f32_wave_kernel<float, 10, true>", "flush_f32_wave_kernel<float, 12, true>",
             "flush_f32_wave_kernel<float, 14, true>", "flush_f32_wave_kernel<float, 16, true>"},
            {"", "flush_f32_wave_kernel<_Float16, 2, true>", "flush_f32_wave_kernel<_Float16, 4, true>",
             "flush_f32_wave_kernel<_Float16, 6, true>", "flush_f32_wave_kernel<_Float16, 8, true>",
             "flush_f32_wave_kernel<_Float16, 10, true>", "flush_f32_wave_kernel<_Float16, 12, true>",
             "flush_f32_wave_kernel<_Float16, 14, true>", "flush_f32_wave_kernel<_Float16, 16, true>"}};
        return bfn[half ? 1 : 0][nsteps / 2];
    }
    const bool wave = nsteps >= 2 && nsteps <= 8 && nsteps % 2 == 0 && c->d.kmax <= 16 &&
                      (nsteps >= 6 || c->dd_variant == 8);
    if (wave) {
        static const char* names[2][5] = {
            {"", "flush_f32_wave_kernel<float, 2>", "flush_f32_wave_kernel<float, 4>",
             "flush_f32_wave_kernel<float, 6>", "flush_f32_wave_kernel<float, 8>"},
            {"", "flush_f32_wave_kernel<_Float16, 2>", "flush_f32_wave_kernel<_Float16, 4>",
             "flush_f32_wave_kernel<_Float16, 6>", "flush_f32_wave_kernel<_Float16, 8>"}};
        return names[half ? 1 : 0][nsteps / 2];
    }
    if (nsteps <= 4 && c->d.kmax <= 16 && c->dd_variant != 2)
        return half ? "flush_f32_persist2_kernel<_Float16>" : "flush_f32_persist2_kernel<float>";
    return half ? "flush_f32_sb_kernel<_Float16>" : "flush_f32_sb_kernel<float>";
}

extern "C" int ekf_debug_result_words(ekf_ctx* c, int e, int out[16])
{
    // Diagnostic: the first 16 words of instance e's last result record (as copied by the last
    // ekf_read_results), including the association path code and guessed winners (RES_DBG).
    if (!c || !out || e < 0 || e >= c->cfg.instances) return EKF_EINVAL;
    memcpy(out, c->h_res + (size_t)e * ekf::RES_STRIDE, sizeof(int) * 16);
    return EKF_OK;
}

extern "C" int ekf_debug_scan_stamps(ekf_ctx* c, unsigned long long out[32])
{
    // Diagnostic: association-kernel phase times summed over instances (100 MHz ticks) since
    // context creation, when built with EKF_SCAN_STAMPS=1 in the environment; zeros otherwise.
    if (!c || !out) return EKF_EINVAL;
    memset(out, 0, sizeof(unsigned long long) * 32);
    if (!c->dbg) return EKF_OK;
    HIP_TRY(hipStreamSynchronize(c->stream));
    std::vector<unsigned long long> h((size_t)32 * c->cfg.instances);
    HIP_TRY(hipMemcpy(h.data(), c->dbg, sizeof(unsigned long long) * h.size(), hipMemcpyDeviceToHost));
    for (int e = 0; e < c->cfg.instances; e++)
        for (int k = 0; k < 32; k++) out[k] += h[(size_t)e * 32 + k];
    return EKF_OK;
}
