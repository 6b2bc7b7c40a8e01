// ekf_api.hip — C-ABI (include/slam_ekf.h) over the gfx950 kernels in ekf_kernels.hip.
//
// A context owns E instances' state in HBM (packed landmark block, robot strip, y, pose,
// savedLineCount), the per-scan scratch, and one HIP stream. localize() enqueues three
// kernels (association/gain, MFMA downdate, augmentation); nothing is copied back unless the
// caller asks for results.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <new>
#include <vector>

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
    hipStream_t own_stream;
    hipStream_t stream;
    size_t elem;      // bytes per stored P_ll element
    size_t pll_inst;  // elements per instance
    size_t op_inst;   // operand elements per instance
    void* Pll;
    double* Rs;
    double* y;
    double* pose;
    double* xpre;
    int* saved;
    double* D;
    double* Ust;
    double* Vst;
    void* Uop;
    void* Vop;
    int* res;
    int2* tile_rc;
    double* d_enc;
    ekf_line* d_lines;
    int* d_nlines;
    int* h_res;
    double* h_pose;
    int dd_grid;
    int prof;
    std::vector<EvPair> ev[3];   // scan, downdate, augment
    std::vector<EvPair> pool;
};

#define HIP_TRY(expr)                                  \
    do {                                               \
        hipError_t _e = (expr);                        \
        if (_e != hipSuccess) {                        \
            fprintf(stderr, "slam_ekf: %s failed: %s\n", #expr, hipGetErrorString(_e)); \
            return EKF_EDEVICE;                        \
        }                                              \
    } while (0)

extern "C" {

void ekf_config_init(ekf_config* c)
{
    if (!c) return;
    memset(c, 0, sizeof(*c));
    c->capacity = 100;       // Robot.h:13
    c->instances = 1;
    c->precision = EKF_PREC_F64;
    c->device = -1;
    c->max_lines = 20;       // main.cpp:99 lines.reserve(20)
    c->r_mode = EKF_R_INTENDED;
    c->reset_margin = 10;    // Robot.cpp:893
    c->mahalanobis = 0.4;    // Robot.h:15
    c->encoder_noise = 0.024;// Robot.h:17
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
    void* ptrs[] = {c->Pll, c->Rs, c->y, c->pose, c->xpre, c->saved, c->D, c->Ust, c->Vst,
                    c->Uop, c->Vop, c->res, c->tile_rc, c->d_enc, c->d_lines, c->d_nlines};
    for (void* p : ptrs)
        if (p) (void)hipFree(p);
    if (c->h_res) (void)hipHostFree(c->h_res);
    if (c->h_pose) (void)hipHostFree(c->h_pose);
    for (auto& v : c->ev)
        for (auto& pr : v) { (void)hipEventDestroy(pr.a); (void)hipEventDestroy(pr.b); }
    for (auto& pr : c->pool) { (void)hipEventDestroy(pr.a); (void)hipEventDestroy(pr.b); }
    if (c->own_stream) (void)hipStreamDestroy(c->own_stream);
}

static int set_robot_ctor(ekf_ctx* c, int e, double x, double y, double th)
{
    // Robot::Robot (Robot.cpp:20-35): P_t0[0][0] = P_t0[1][1] = 0.05, P_t0[2][2] = 0, the rest
    // (and y, savedLineCount) zero.
    const Dims& d = c->d;
    HIP_TRY(hipMemsetAsync((char*)c->Pll + (size_t)e * c->pll_inst * c->elem, 0,
                           c->pll_inst * c->elem, c->stream));
    HIP_TRY(hipMemsetAsync(c->Rs + (size_t)e * 3 * d.n, 0, sizeof(double) * 3 * d.n, c->stream));
    HIP_TRY(hipMemsetAsync(c->y + (size_t)e * d.n, 0, sizeof(double) * d.n, c->stream));
    const double v = 0.05;
    HIP_TRY(hipMemcpyAsync(c->Rs + (size_t)e * 3 * d.n + 0, &v, sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->Rs + (size_t)e * 3 * d.n + d.n + 1, &v, sizeof(double),
                           hipMemcpyHostToDevice, c->stream));
    const double pose[3] = {x, y, th};
    HIP_TRY(hipMemcpyAsync(c->pose + 3 * e, pose, sizeof(pose), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipMemcpyAsync(c->xpre + 3 * e, pose, sizeof(pose), hipMemcpyHostToDevice, c->stream));
    const int zero = 0;
    HIP_TRY(hipMemcpyAsync(c->saved + e, &zero, sizeof(int), hipMemcpyHostToDevice, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

extern "C" int ekf_create(const ekf_config* cfg, ekf_ctx** out)
{
    if (!cfg || !out) return EKF_EINVAL;
    *out = nullptr;
    if (cfg->capacity < 1 || cfg->instances < 1 || cfg->max_lines < 1 ||
        cfg->max_lines > EKF_MAX_LINES ||
        (cfg->precision != EKF_PREC_F64 && cfg->precision != EKF_PREC_F32) ||
        (cfg->r_mode != EKF_R_INTENDED && cfg->r_mode != EKF_R_AS_WRITTEN) ||
        cfg->capacity > (1 << 20))
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
    // operands: k columns rounded to a multiple of 16 (8 f32 k-steps / 4 f64 k-steps per chunk)
    c->d.kmax = ((2 * cfg->max_lines + 15) / 16) * 16;
    const Dims& d = c->d;
    const int E = cfg->instances;
    c->elem = (cfg->precision == EKF_PREC_F64) ? 8 : 4;
    c->pll_inst = (size_t)d.ntiles * ekf::TILE_ELEMS;
    c->op_inst = (size_t)d.nb * 64 * (d.kmax / 2);
    int rc = EKF_ENOMEM;
#define ALLOC(ptr, bytes)                                                      \
    do {                                                                       \
        if (hipMalloc((void**)&(ptr), (bytes)) != hipSuccess) goto fail;       \
        if (hipMemset((ptr), 0, (bytes)) != hipSuccess) goto fail;             \
    } while (0)
    ALLOC(c->Pll, c->pll_inst * c->elem * E);
    ALLOC(c->Rs, sizeof(double) * 3 * d.n * E);
    ALLOC(c->y, sizeof(double) * d.n * E);
    ALLOC(c->pose, sizeof(double) * 3 * E);
    ALLOC(c->xpre, sizeof(double) * 3 * E);
    ALLOC(c->saved, sizeof(int) * E);
    ALLOC(c->D, sizeof(double) * 4 * d.N * E);
    ALLOC(c->Ust, sizeof(double) * d.max_lines * 2 * d.n * E);
    ALLOC(c->Vst, sizeof(double) * d.max_lines * 2 * d.n * E);
    ALLOC(c->Uop, c->op_inst * c->elem * E);
    ALLOC(c->Vop, c->op_inst * c->elem * E);
    ALLOC(c->res, sizeof(int) * ekf::RES_STRIDE * E);
    ALLOC(c->tile_rc, sizeof(int2) * d.ntiles);
    ALLOC(c->d_enc, sizeof(double) * 3 * E);
    ALLOC(c->d_lines, sizeof(ekf_line) * d.max_lines * E);
    ALLOC(c->d_nlines, sizeof(int) * E);
#undef ALLOC
    if (hipHostMalloc((void**)&c->h_res, sizeof(int) * ekf::RES_STRIDE * E) != hipSuccess) goto fail;
    if (hipHostMalloc((void**)&c->h_pose, sizeof(double) * 3 * E) != hipSuccess) goto fail;
    rc = EKF_EDEVICE;
    if (hipStreamCreateWithFlags(&c->own_stream, hipStreamNonBlocking) != hipSuccess) goto fail;
    c->stream = c->own_stream;
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
    }
    {
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, c->device) != hipSuccess) goto fail;
        c->dd_grid = prop.multiProcessorCount * 8;
    }
    for (int e = 0; e < E; e++)
        if (set_robot_ctor(c, e, 0.0, 0.0, 0.0) != EKF_OK) goto fail;
    *out = c;
    return EKF_OK;
fail:
    free_all(c);
    delete c;
    return rc;
}

extern "C" int ekf_destroy(ekf_ctx* c)
{
    if (!c) return EKF_EINVAL;
    (void)hipStreamSynchronize(c->stream);
    free_all(c);
    delete c;
    return EKF_OK;
}

extern "C" int ekf_set_stream(ekf_ctx* c, void* s)
{
    if (!c) return EKF_EINVAL;
    c->stream = s ? (hipStream_t)s : c->own_stream;
    return EKF_OK;
}

extern "C" int ekf_sync(ekf_ctx* c)
{
    if (!c) return EKF_EINVAL;
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

extern "C" int ekf_reset_instance(ekf_ctx* c, int e, double x, double y, double th)
{
    if (!c) return EKF_EINVAL;
    if (e >= c->cfg.instances) return EKF_ERANGE;
    if (e < 0) {
        for (int k = 0; k < c->cfg.instances; k++) {
            int rc = set_robot_ctor(c, k, x, y, th);
            if (rc) return rc;
        }
        return EKF_OK;
    }
    return set_robot_ctor(c, e, x, y, th);
}

static ekf::ScanParams scan_params(ekf_ctx* c, int phase, const double* enc,
                                   const ekf_line* lines, const int* nlines)
{
    ekf::ScanParams p;
    p.d = c->d;
    p.E = c->cfg.instances;
    p.phase = phase;
    p.r_mode = c->cfg.r_mode;
    p.reset_margin = c->cfg.reset_margin;
    p.gate = c->cfg.mahalanobis;
    p.enc_noise = c->cfg.encoder_noise;
    p.Pll = c->Pll;
    p.Rs = c->Rs;
    p.y = c->y;
    p.pose = c->pose;
    p.xpre = c->xpre;
    p.saved = c->saved;
    p.D = c->D;
    p.Ust = c->Ust;
    p.Vst = c->Vst;
    p.Uop = c->Uop;
    p.Vop = c->Vop;
    p.res = c->res;
    p.enc = enc;
    p.lines = lines;
    p.nlines = nlines;
    return p;
}

static EvPair* prof_begin(ekf_ctx* c, int kind)
{
    if (!c->prof) return nullptr;
    EvPair pr;
    if (!c->pool.empty()) {
        pr = c->pool.back();
        c->pool.pop_back();
    } else {
        if (hipEventCreate(&pr.a) != hipSuccess) return nullptr;
        if (hipEventCreate(&pr.b) != hipSuccess) return nullptr;
    }
    c->ev[kind].push_back(pr);
    (void)hipEventRecord(pr.a, c->stream);
    return &c->ev[kind].back();
}

static void prof_end(ekf_ctx* c, EvPair* pr)
{
    if (pr) (void)hipEventRecord(pr->b, c->stream);
}

static int enqueue(ekf_ctx* c, int phase, const double* enc, const ekf_line* lines,
                   const int* nlines)
{
    ekf::ScanParams sp = scan_params(c, phase, enc, lines, nlines);
    EvPair* pr = prof_begin(c, 0);
    HIP_TRY(ekf::launch_scan(sp, c->cfg.precision, c->stream));
    prof_end(c, pr);
    if (!(phase & ekf::PHASE_UPDATE)) return EKF_OK;
    ekf::DowndateParams dp;
    dp.d = c->d;
    dp.E = c->cfg.instances;
    dp.Pll = c->Pll;
    dp.Uop = c->Uop;
    dp.Vop = c->Vop;
    dp.res = c->res;
    dp.tile_rc = c->tile_rc;
    pr = prof_begin(c, 1);
    HIP_TRY(ekf::launch_downdate(dp, c->cfg.precision, c->dd_grid, c->stream));
    prof_end(c, pr);
    pr = prof_begin(c, 2);
    HIP_TRY(ekf::launch_augment(sp, c->cfg.precision, c->stream));
    prof_end(c, pr);
    return EKF_OK;
}

static int stage_inputs(ekf_ctx* c, const double* enc, const ekf_line* lines, const int* nlines)
{
    const int E = c->cfg.instances;
    if (enc)
        HIP_TRY(hipMemcpyAsync(c->d_enc, enc, sizeof(double) * 3 * E, hipMemcpyHostToDevice,
                               c->stream));
    if (lines)
        HIP_TRY(hipMemcpyAsync(c->d_lines, lines, sizeof(ekf_line) * c->d.max_lines * E,
                               hipMemcpyHostToDevice, c->stream));
    if (nlines) {
        for (int e = 0; e < E; e++)
            if (nlines[e] < 0 || nlines[e] > c->d.max_lines) return EKF_ERANGE;
        HIP_TRY(hipMemcpyAsync(c->d_nlines, nlines, sizeof(int) * E, hipMemcpyHostToDevice,
                               c->stream));
    }
    return EKF_OK;
}

extern "C" int ekf_read_results(ekf_ctx* c, ekf_result* out)
{
    if (!c) return EKF_EINVAL;
    const int E = c->cfg.instances;
    HIP_TRY(hipMemcpyAsync(c->h_res, c->res, sizeof(int) * ekf::RES_STRIDE * E,
                           hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipMemcpyAsync(c->h_pose, c->pose, sizeof(double) * 3 * E, hipMemcpyDeviceToHost,
                           c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    if (!out) return EKF_OK;
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
        for (int i = 0; i < EKF_MAX_LINES; i++) o.match[i] = (i < o.nlines) ? r[ekf::RES_MATCH + i] : -1;
    }
    return EKF_OK;
}

extern "C" int ekf_localize(ekf_ctx* c, const double* enc, const ekf_line* lines,
                            const int32_t* nlines, ekf_result* out)
{
    if (!c || !enc || !lines || !nlines) return EKF_EINVAL;
    int rc = stage_inputs(c, enc, lines, nlines);
    if (rc) return rc;
    rc = enqueue(c, ekf::PHASE_BOTH, c->d_enc, c->d_lines, c->d_nlines);
    if (rc) return rc;
    return ekf_read_results(c, out);
}

extern "C" int ekf_localize_device(ekf_ctx* c, const double* d_enc, const ekf_line* d_lines,
                                   const int32_t* d_nlines)
{
    if (!c || !d_enc || !d_lines || !d_nlines) return EKF_EINVAL;
    return enqueue(c, ekf::PHASE_BOTH, d_enc, d_lines, d_nlines);
}

extern "C" int ekf_predict(ekf_ctx* c, const double* enc)
{
    if (!c || !enc) return EKF_EINVAL;
    int rc = stage_inputs(c, enc, nullptr, nullptr);
    if (rc) return rc;
    return enqueue(c, ekf::PHASE_PREDICT, c->d_enc, c->d_lines, c->d_nlines);
}

extern "C" int ekf_update(ekf_ctx* c, const ekf_line* lines, const int32_t* nlines,
                          ekf_result* out)
{
    if (!c || !nlines) return EKF_EINVAL;
    int rc = stage_inputs(c, nullptr, lines, nlines);
    if (rc) return rc;
    rc = enqueue(c, ekf::PHASE_UPDATE, c->d_enc, c->d_lines, c->d_nlines);
    if (rc) return rc;
    return ekf_read_results(c, out);
}

extern "C" int ekf_upload_state(ekf_ctx* c, int e, const double* P, const double* y, int saved,
                                const double pose[3])
{
    if (!c) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    if (saved < 0 || saved > c->d.N) return EKF_ERANGE;
    const Dims& d = c->d;
    if (P) {
        double* tmp = nullptr;
        HIP_TRY(hipMalloc((void**)&tmp, sizeof(double) * d.n * d.n));
        hipError_t err = hipMemcpyAsync(tmp, P, sizeof(double) * d.n * d.n, hipMemcpyHostToDevice,
                                        c->stream);
        if (err == hipSuccess)
            err = ekf::launch_pack(d, c->cfg.precision, tmp,
                                   (char*)c->Pll + (size_t)e * c->pll_inst * c->elem,
                                   c->Rs + (size_t)e * 3 * d.n, c->tile_rc, c->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        (void)hipFree(tmp);
        HIP_TRY(err);
    }
    if (y)
        HIP_TRY(hipMemcpyAsync(c->y + (size_t)e * d.n, y, sizeof(double) * d.n,
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
    const Dims& d = c->d;
    if (P) {
        double* tmp = nullptr;
        HIP_TRY(hipMalloc((void**)&tmp, sizeof(double) * d.n * d.n));
        hipError_t err = ekf::launch_unpack(d, c->cfg.precision, tmp,
                                            (const char*)c->Pll + (size_t)e * c->pll_inst * c->elem,
                                            c->Rs + (size_t)e * 3 * d.n, c->stream);
        if (err == hipSuccess)
            err = hipMemcpyAsync(P, tmp, sizeof(double) * d.n * d.n, hipMemcpyDeviceToHost,
                                 c->stream);
        if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
        (void)hipFree(tmp);
        HIP_TRY(err);
    }
    if (y)
        HIP_TRY(hipMemcpyAsync(y, c->y + (size_t)e * d.n, sizeof(double) * d.n,
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
    if (!c || !diag || (rank > 0 && !U) || rank < 0) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    const Dims& d = c->d;
    double *dd = nullptr, *du = nullptr;
    HIP_TRY(hipMalloc((void**)&dd, sizeof(double) * d.n));
    hipError_t err = hipMalloc((void**)&du, sizeof(double) * d.n * (rank > 0 ? rank : 1));
    if (err == hipSuccess)
        err = hipMemcpyAsync(dd, diag, sizeof(double) * d.n, hipMemcpyHostToDevice, c->stream);
    if (err == hipSuccess && rank > 0)
        err = hipMemcpyAsync(du, U, sizeof(double) * d.n * rank, hipMemcpyHostToDevice, c->stream);
    if (err == hipSuccess)
        err = ekf::launch_lowrank(d, c->cfg.precision, dd, du, rank,
                                  (char*)c->Pll + (size_t)e * c->pll_inst * c->elem,
                                  c->Rs + (size_t)e * 3 * d.n, c->tile_rc, c->stream);
    if (err == hipSuccess) err = hipStreamSynchronize(c->stream);
    (void)hipFree(dd);
    if (du) (void)hipFree(du);
    HIP_TRY(err);
    return ekf_upload_state(c, e, nullptr, y, saved, pose);
}

extern "C" int ekf_get_pose_cov(ekf_ctx* c, int e, double P33[9])
{
    if (!c || !P33) return EKF_EINVAL;
    if (e < 0 || e >= c->cfg.instances) return EKF_ERANGE;
    const Dims& d = c->d;
    for (int a = 0; a < 3; a++)
        HIP_TRY(hipMemcpyAsync(P33 + 3 * a, c->Rs + (size_t)e * 3 * d.n + (size_t)a * d.n,
                               sizeof(double) * 3, hipMemcpyDeviceToHost, c->stream));
    HIP_TRY(hipStreamSynchronize(c->stream));
    return EKF_OK;
}

extern "C" int ekf_get_ellipse(ekf_ctx* c, int e, float axii[2], float* angle)
{
    // Robot::getEllipse (Robot.cpp:73-124): eigen-decomposition of P_t0[0:2,0:2], eigenvalues
    // sorted by |λ| ascending, axii[i] = 2·sqrt(5.991·|λ_i|), angle = atan2(v0, v1) of the
    // eigenvector of the larger |λ|. GSL's nonsymmv sign convention for the eigenvector is not
    // reproducible without GSL: here each eigenvector is unit-norm with its first non-zero
    // component positive (angle parity is therefore modulo π).
    if (!c || !axii || !angle) return -EKF_EINVAL;
    double P33[9];
    int rc = ekf_get_pose_cov(c, e, P33);
    if (rc) return -rc;
    const double a = P33[0], b = P33[1], cc = P33[3], dd = P33[4];
    if (!isfinite(a) || !isfinite(b) || !isfinite(cc) || !isfinite(dd)) return 0;
    const double tr = 0.5 * (a + dd);
    const double disc = 0.25 * (a - dd) * (a - dd) + b * cc;
    if (disc < 0) return 0;  // complex pair: not produced by a covariance block
    const double sq = sqrt(disc);
    double lam[2] = {tr - sq, tr + sq};
    if (fabs(lam[0]) > fabs(lam[1])) {
        double t = lam[0]; lam[0] = lam[1]; lam[1] = t;
    }
    double vx = 1.0, vy = 0.0;
    {
        const double l = lam[1];
        double x1 = b, y1 = l - a, x2 = l - dd, y2 = cc;
        const double n1 = hypot(x1, y1), n2 = hypot(x2, y2);
        if (n1 >= n2 && n1 > 0) { vx = x1 / n1; vy = y1 / n1; }
        else if (n2 > 0) { vx = x2 / n2; vy = y2 / n2; }
        if (vx < 0 || (vx == 0 && vy < 0)) { vx = -vx; vy = -vy; }
    }
    axii[0] = 2.f * (float)sqrt(5.991 * fabs(lam[0]));
    axii[1] = 2.f * (float)sqrt(5.991 * fabs(lam[1]));
    *angle = (float)atan2(vx, vy);
    return 1;
}

extern "C" size_t ekf_landmark_block_bytes(const ekf_ctx* c)
{
    return c ? c->pll_inst * c->elem : 0;
}

extern "C" int ekf_state_dim(const ekf_ctx* c) { return c ? c->d.n : 0; }

extern "C" int ekf_profile_enable(ekf_ctx* c, int enable)
{
    if (!c) return EKF_EINVAL;
    (void)hipStreamSynchronize(c->stream);
    for (auto& v : c->ev) {
        for (auto& pr : v) c->pool.push_back(pr);
        v.clear();
    }
    c->prof = enable ? 1 : 0;
    return EKF_OK;
}

extern "C" int ekf_profile_read(ekf_ctx* c, double* scan_ms, double* dd_ms, double* aug_ms,
                                int* launches)
{
    if (!c) return EKF_EINVAL;
    HIP_TRY(hipStreamSynchronize(c->stream));
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
