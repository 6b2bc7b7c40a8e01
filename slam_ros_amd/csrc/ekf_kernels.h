// ekf_kernels.h — launch parameters shared by ekf_kernels.hip and ekf_api.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/slam_ekf.h"
#include "ekf_layout.h"

namespace ekf {

enum { PHASE_PREDICT = 1, PHASE_UPDATE = 2, PHASE_BOTH = 3 };
enum { EKF_ST_SINGULAR = EKF_ST_SINGULAR_S, EKF_ST_CAP = EKF_ST_CAPACITY, EKF_ST_NSYM = EKF_ST_NONSYM };

// per-instance result record in device memory (ints)
enum {
    RES_M = 0,        // matches
    RES_NEXTRA = 1,   // lines appended as new landmarks
    RES_SAVED_IN = 2, // savedLineCount before augmentation
    RES_SAVED = 3,    // savedLineCount after the call
    RES_RESET = 4,
    RES_STATUS = 5,
    RES_NLINES = 6,
    RES_KSTEPS = 7,   // MFMA k-steps of the downdate (0 = no downdate)
    RES_MATCH = 8,                      // [EKF_MAX_LINES]
    RES_EXTRA = 8 + EKF_MAX_LINES,      // [EKF_MAX_LINES] line indices, in order
    RES_STRIDE = 8 + 2 * EKF_MAX_LINES,
};

struct ScanParams {
    Dims d;
    int E;
    int phase;
    int r_mode;
    int reset_margin;
    double gate;
    double enc_noise;
    void* Pll;        // [E][ntiles][1024] storage precision
    double* Rs;       // [E][3][n]
    double* y;        // [E][n]
    double* pose;     // [E][3]
    double* xpre;     // [E][3]
    int* saved;       // [E]
    double* D;        // [E][4][N]
    double* Ust;      // [E][max_lines][2][n]
    double* Vst;      // [E][max_lines][2][n]
    void* Uop;        // [E][nb][64][kmax/2]
    void* Vop;
    int* res;         // [E][RES_STRIDE]
    const double* enc;       // [E][3]
    const ekf_line* lines;   // [E][max_lines]
    const int* nlines;       // [E]
};

struct DowndateParams {
    Dims d;
    int E;
    void* Pll;
    const void* Uop;
    const void* Vop;
    const int* res;
    const int2* tile_rc;   // [ntiles] (bi, bj)
};

hipError_t launch_scan(const ScanParams& p, int precision, hipStream_t st);
hipError_t launch_downdate(const DowndateParams& p, int precision, int grid, hipStream_t st);
hipError_t launch_augment(const ScanParams& p, int precision, hipStream_t st);
hipError_t launch_pack(const Dims& d, int precision, const double* Pfull, void* Pll, double* Rs,
                       const int2* tile_rc, hipStream_t st);
hipError_t launch_unpack(const Dims& d, int precision, double* Pfull, const void* Pll,
                         const double* Rs, hipStream_t st);
hipError_t launch_lowrank(const Dims& d, int precision, const double* diag, const double* U,
                          int rank, void* Pll, double* Rs, const int2* tile_rc, hipStream_t st);

}  // namespace ekf
