// ekf_kernels.h — launch parameters shared by ekf_kernels.hip and ekf_api.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/slam_ekf.h"
#include "ekf_layout.h"
#include "ekf_commit.h"

namespace ekf {

enum { PHASE_PREDICT = 1, PHASE_UPDATE = 2, PHASE_BOTH = 3 };
enum { EKF_ST_SINGULAR = EKF_ST_SINGULAR_S, EKF_ST_CAP = EKF_ST_CAPACITY, EKF_ST_NSYM = EKF_ST_NONSYM,
       EKF_ST_TIMEOUT_BIT = EKF_ST_SYNC_TIMEOUT, EKF_ST_RANGE_BIT = EKF_ST_RANGE,
       EKF_ST_PRECISION_BIT = EKF_ST_PRECISION };
// fp32 storage: a scan that shrinks an owned landmark's variance trace by more than 2^4 sets
// EKF_ST_PRECISION: the cancellation leaves fewer than 20 of fp32's 24 significant bits, i.e. a
// stored result no longer guaranteed to 2^-20 ≈ 1e-6 relative (the P bar) element by element
constexpr double PREC_CANCEL = 16.0;
// fp16 storage: a stored variance above 2^14 (a quarter of the fp16 range) raises EKF_ST_RANGE
constexpr double F16_RANGE_WARN = 16384.0;
// fp32 storage: a new landmark variance above 2^120 (fp32's largest finite value is ≈2^128) sets
// EKF_ST_RANGE too
constexpr double F32_RANGE_WARN = 1.329227995784916e36;   // 2^120
constexpr int F16_EXP_DEFAULT = 10;

// per-instance synchronisation words of the association kernel (never reset): a monotonic
// start counter, then one status word per workgroup, rewritten by every launch
enum { SYNC_START = 0, SYNC_WG0 = 4 };
constexpr int MAX_GROUPS = (MAX_CAPACITY + SCAN_THREADS - 1) / SCAN_THREADS;   // workgroups per instance
constexpr int SPEC_GMAX = 64;  // speculative association: workgroups per instance (<= one wave)
constexpr int MB_WORDS_FIXED = 26; // mailbox words before the V-history (see ekf_kernels.hip)
constexpr int SH_MAX_LINES = 8;     // a partitioned context's lines per scan (ekf_shard_create)
constexpr int SH_PKG_WORDS = MB_WORDS_FIXED + 4 * SH_MAX_LINES;   // one gain package of its scan

// per-instance result record in device memory (ints)
enum {
    RES_M = 0,        // matches
    RES_NEXTRA = 1,   // lines appended to extraLines (Robot.cpp:291)
    RES_SAVED_IN = 2, // savedLineCount before augmentation (first new landmark index)
    RES_SAVED = 3,    // savedLineCount after the call
    RES_RESET = 4,
    RES_STATUS = 5,
    RES_NLINES = 6,
    RES_KSTEPS = 7,   // MFMA k-steps of the downdate (0 = no downdate)
    RES_NADD = 8,     // landmarks actually added (patch rows)
    RES_DBG = 9,      // diagnostics: association path code, then the first 5 guessed winners
    RES_ROLLBACK = 15,// 1: the call timed out and was rolled back (no downdate, rows or reset)
    RES_MATCH = 16,                     // [EKF_MAX_LINES]
    RES_EXTRA = 16 + EKF_MAX_LINES,     // [EKF_MAX_LINES] line indices, in order
    RES_PSIG = 16 + 2 * EKF_MAX_LINES,  // EKF_ARITH_F16X3: the plane exponent σ of this step's planes
    RES_ZMAX = 17 + 2 * EKF_MAX_LINES,  // landmarks at or past this index have zero operand rows and no
                                        // new rows this step (workgroup granularity)
    RES_STRIDE = 16 + 2 * EKF_MAX_LINES + 4,
};

// Per-step outputs that outlive the step's association kernel (a ring of slots): the
// downdate operands, the augmented rows and the result record. They are consumed by the flush
// (covariance downdate) of the step's group and, until then, by later association kernels
// that read the landmark block with the pending steps applied on read.
struct Slot {
    void* Uop;          // [E][nb][64][kmax/2]    -U in MFMA operand order (storage precision)
    void* Vop;          //                         V in MFMA operand order
    double* patch;      // [E][max_lines][2][M]   rows of landmarks added by this step
    double* patch_diag; // [E][max_lines][4]      their 2x2 diagonal blocks
    int* res;           // [E][RES_STRIDE]
    void* Bop;          // [E][nb][npl][64][8] V split into planes in the operand order of the 32x32x16
                        // MFMAs: EKF_ARITH_BF16X6 hi + mid + lo bf16 (npl = 3), EKF_ARITH_F16X3 hi +
                        // lo fp16 of 2^σ·V (npl = 2); nullptr for EKF_ARITH_EXACT
};

constexpr int PMAX = 32;
constexpr int WT_R = 2, WT_C = 2, WT_N = WT_R * WT_C;   // f32 wave flush: tiles per wave-tile
constexpr int WT64_C = 2;                                 // f64 wave flush: 1 × 2 tiles per wave-tile
constexpr int F64_WAVE_MAXS = 8;                          // f64 wave flush: steps per launch
constexpr int F64_RING = 4;                                // f64 wave flush: operand ring depth
constexpr int F16X3_MAXS = 24;                            // split-fp16 contexts: flush_interval <= 24

// one wave-tile of the wave flush (host-built table, read with scalar loads): the linear indices
// of its WT_N tiles (positions below the diagonal or past the block point at a stored tile of
// the same wave-tile and are not written back), their validity, the operand row blocks of its
// WT_R tile rows and WT_C tile columns (16 bits each, clamped to the block) and (wr, wc)
struct alignas(32) WtEntry {
    int tile[WT_N];
    int valid;      // bit i: tile i is stored
    int rows[2];    // [0]: A row blocks (WT_R × 16 bits), [1]: B row blocks (WT_C × 16 bits)
    int rc;         // wr | wc << 16
};
constexpr int DD_SB = 4;   // f32 flush: tiles per super-tile side (one wave per tile row)

struct ScanParams {
    Dims d;
    int E;                // instances in this launch (grid.y)
    int e0;               // first instance of this launch
    int G;                // workgroups per instance = ceil(N / nt)
    int nt;               // landmarks per workgroup: SCAN_THREADS, or 128 / 64 (the F16X3 kernel only)
    int usym;             // symmetric fp32 operands, U = −2^x·V: the U rows are not stored (Slot::Uop)
    int mbw;              // mailbox words per workgroup slot
    double* mbox;         // [E][2][G][mbw] per-line candidate exchange
    int* sync;            // [E][sync_stride]
    int sync_stride;      // SYNC_WG0 + G, rounded up
    int phase;
    int r_mode;
    int reset_margin;
    int npend;            // steps not yet in Pread, applied on read (in order)
    int spec;             // speculative association: 0 off, 1 on, 2 test hook (wrong guesses)
    unsigned epoch;       // launch sequence number: tags the mailbox words of this launch
    double gate;
    double enc_noise;
    const void* Pread;    // [E][ntiles][1024] landmark block to read
    double* Rs;           // [2][Etot][3][n]  robot strip (rows 0..2 of P), two copies: a launch reads
    double* y;            // [2][Etot][n]     copy live[e] and writes the other, which the lead commits
    int* live;            // [Etot] committed copy of Rs / y per instance (flipped by the lead)
    int Etot;             // instances of the context
    int spin_log2;        // spin bound of every wait: 2^spin_log2 polls (24; tests lower it)
    int test_drop;        // test hook: e + 1 = the last workgroup of instance e never runs (0: off)
    int test_verdict;     // test hook: e + 1 = workgroup 1 of instance e sees its verdict poll time out
    double* Dd;           // [2][Etot][N][4] diagonal landmark blocks after the last committed step
                          // (copy live[e] read, the other written and committed with Rs / y)
    int mfrep64;          // fp64 context: pending steps replayed on read by f64 MFMA (the flush's own
                          // instruction: bit-identical chains; EKF_OPT_MFMA_REPLAY)
    int mfrep;            // split-plane context: pending steps replayed on read by MFMA (1 split
                          // products on the planes, 2 fp32 MFMA on the fp32 operand rows),
                          // diagonal blocks kept in Dd; 0 the per-element forms
    int bf;               // split-plane context (1 EKF_ARITH_BF16X6, 2 EKF_ARITH_F16X3): fp16 storage
                          // rounded once per flush group, also in the on-read replay
    int* psig;            // [Etot] EKF_ARITH_F16X3 plane exponent σ (the lead lowers it when a new
    double* pvmax;        // [Etot] landmark raises the largest landmark variance vmax)
    double* pose;         // [E][3]
    double* xpre;         // [E][3]
    int* saved;           // [E]
    double* Ust;          // [E][max_lines][n][2] U_t = K_t·S_t of this scan (fp64 scratch)
    double* Vst;          // [E][max_lines][n][2] V_t = K_t
    Slot cur;             // this step's slot
    Slot pend[PMAX];      // pending steps, oldest first
    const double* enc;    // [E][3]
    const ekf_line* lines;// [E][max_lines]
    const int* nlines;    // [E]
    const int* pexp;      // [E] fp16 storage exponent (P stored as 2^pexp·P)
    unsigned long long* dbg;  // optional [E][16] phase timers (s_memrealtime ticks, 100 MHz)
    // synchronous calls (ekf_localize / ekf_update): the lead also writes a committed step's result
    // words and folded status, pose and robot 3×3 block into pinned host memory (device pointers of
    // host-mapped buffers), then the launch epoch into ep_host[e] (system-scope release); nullptr: off
    int* res_host;        // [Etot][RES_STRIDE]
    double* pose_host;    // [Etot][3]
    double* r33_host;     // [Etot][9]
    unsigned* ep_host;    // [Etot]
};

// One instance whose landmark block is partitioned over ranks: rank r
// stores the packed tiles of tile rows [r0, r1) only (a contiguous slice of the packed array,
// balanced by tile count); everything of size O(n) — robot strip, mean, the landmarks' scan state,
// their diagonal blocks, the operand rows — is replicated and evolves identically on every rank.
// A scan runs the sequential association (Robot.cpp:298-641) as phases over ALL landmarks; the only
// exchanges are sums of [N][4] buffers in which every rank fills the 2×2 blocks its tiles hold:
// the diagonal blocks once per scan, the winner's column once per matched line.
enum { SH_BEGIN = 0, SH_DIAG = 1, SH_GATE = 2, SH_COLUMN = 3, SH_APPLY = 4, SH_ROBOT = 5, SH_END = 6,
       // speculative association of the partitioned instance (ekf_shard_speculate / ekf_shard_run):
       // every line's first passing landmark at the scan's start (the guesses), the rank's blocks of
       // all guessed columns, and (shard_run_kernel) the winner's package without its column
       SH_GUESS = 7, SH_SPEC_COLS = 8, SH_PACKAGE = 9 };
constexpr int SH_REC = 20;   // doubles per landmark: rr0..2 (6), yb (2), Dj (4), ma0, s0j, c0j, s0f, c0f, spare
// device control words of the running scan (no host round trip between phases)
enum { SC_WIN = 0, SC_STATUS = 1, SC_M = 2, SC_NEXTRA = 3, SC_S = 4, SC_NEXT = 5, SC_MATCH = 8,
       SC_EXTRA = 8 + EKF_MAX_LINES, SC_GUESS = 8 + 2 * EKF_MAX_LINES, SC_WORDS = 8 + 3 * EKF_MAX_LINES };
struct ShardParams {
    Dims d;
    int phase;
    int line, L;
    int r_mode;
    double gate, enc_noise;
    int npend;
    const void* Pread;    // tile t (t0 <= t < t1) of instance 0 at Pread + t·TILE_ELEMS (the slice, shifted)
    long long t0, t1;     // the rank's tiles (global packed indices)
    Slot cur;
    Slot pend[PMAX];
    double* Rs;           // [3][n] robot strip (the committed copy)
    double* y;            // [n]
    double* pose;         // [3]
    int* saved;           // [1]
    double* rob;          // [12] R33 and x_pre of the running scan (the same on every rank)
    double* rec;          // [N][SH_REC]
    double* hist;         // [N][max_lines][8] U rows and V rows of each match of the scan
    int* flags;           // [N] bit 0 matched, bit 1 singular at this line
    double* pkg;          // [MB words + 4·max_lines] the line's gain package
    int* ctl;             // [SC_WORDS]
    double* col;          // [N][4] the exchange buffer (caller's device memory)
    double* cols;         // [L][N][4] the guessed columns' exchange buffer (speculative path)
    double* next_out;     // shard_run_kernel: the line it stopped at, as a double (caller's device memory)
    const double* enc;    // [3]
    const ekf_line* lines;// [max_lines]
    const int* pexp;
    int reset_margin;
    double enc_v[3];      // SH_BEGIN: the scan's encoder pose and lines (kernel arguments; it stores
    ekf_line lines_v[EKF_MAX_LINES];   // them to enc / lines for the later phases)
    int diag_first;       // SH_GUESS: take the summed diagonal blocks first (SH_DIAG in the same launch)
    double* pkg_slot;     // SH_GATE (shard_run_kernel): a passing landmark's package into this slot
    int* res_host;        // SH_END: the step's record and pose also into pinned host memory (device
    double* pose_host;    // pointers; nullptr: not)
    double* mbox;         // shard_run_kernel: the workgroups' mailbox (2 parities × G slots of mbw words)
    int mbw;
    unsigned epoch;       // its tag epoch (one per launch)
    int spin_log2;        // its bounded waits
    const double* end_gate;   // SH_END (ekf_shard_localize): commit only if the ranks' agreement
    double* end_gate_host;    // [failure flag, stopping line] is [0, L]; the pair also into pinned host
                              // memory (device pointer) either way (nullptr: commit unconditionally)
};
hipError_t launch_shard(const ShardParams& p, int precision, hipStream_t st);
// lines [ctl[SC_NEXT], L) of the speculative path on shard_run_workgroups(N) cooperating
// workgroups (shard_run_kernel)
hipError_t launch_shard_run(const ShardParams& p, int precision, hipStream_t st);
constexpr int SH_THREADS = 64;     // shard_kernel's workgroup
#ifndef EKF_SHR_THREADS
#define EKF_SHR_THREADS 128
#endif
constexpr int SHR_THREADS = EKF_SHR_THREADS;   // shard_run_kernel's workgroup: landmarks per workgroup
constexpr int SHR_GMAX = 64;       // ... and at most this many workgroups (more landmarks per thread past it)
#ifndef EKF_SHARD_SPEC
#define EKF_SHARD_SPEC 1           // launch_shard_run: shard_spec_kernel where it applies (0: shard_run_kernel always)
#endif
inline int shard_run_workgroups(int N)
{
    const int g = (N + SHR_THREADS - 1) / SHR_THREADS;
    return g < 1 ? 1 : (g > SHR_GMAX ? SHR_GMAX : g);
}

// One pass over the landmark block applying nsteps steps in order (each: reset, or rank-2m
// downdate then its augmented rows). Pout may equal Pin (in place).
struct DowndateParams {
    Dims d;
    int E;
    int nsteps;
    int variant;          // f32 flush form (tests only, EKF_FLUSH_VARIANT; all bit-identical): 0 auto,
                          // 2 super-tile form, 8 wave form also for 2 or 4 steps
    int ncu;              // compute units (persistent grid)
    const void* Pin;
    void* Pout;
    const int2* tile_rc;  // [ntiles] (bi, bj)
    const int2* stile_rc; // [nsb(nsb+1)/2] (sbi, sbj) super-tiles of DD_SB × DD_SB tiles, sbi <= sbj
    const int2* stile2_rc;// [nstiles2] (sbi, sbj) super-tiles of DD_SB × 2 tiles holding a stored tile
    int nstiles2;
    const WtEntry* wt;    // [nwt] wave-tiles of WT_R × WT_C tiles holding a stored tile, panel order
    int nwt;
    const WtEntry* wt64;  // [nwt64] f64 wave-tiles of 1 × WT64_C tiles (tile[0..1], rows[0] = A row block)
    int nwt64;
    const int* pexp;      // [E] fp16 storage exponent
    int usym;             // the steps' U rows are −2^pexp·V (not stored): read V and scale
    void* sink;           // one scratch tile (8 KB): the wave flushes' stores of slots outside the triangle
    const void* ubase;    // operand rows of ring slot i at ubase / vbase + i·slot_bytes; the
    const void* vbase;    // group's step q is slot (slot0 + q) mod nslots (= steps[q].Uop / .Vop)
    long long slot_bytes;
    int slot0, nslots;
    unsigned long long* dbg;  // EKF_SCAN_STAMPS buffer (timing experiments of the flush only)
    const void* bbase;    // EKF_ARITH_BF16X6: bf16 operand planes of ring slot i at bbase + i·bslot_bytes
    long long bslot_bytes;
    int bf;               // plain groups of 2..16 steps (even) run the split-plane wave flush:
                          // 1 EKF_ARITH_BF16X6, 2 EKF_ARITH_F16X3 (σ of each step in RES_PSIG)
    int zskip;            // split-plane wave flush: skip wave-tiles past every step's RES_ZMAX
    const int* wt24;      // [nwt24] split-bf16 wave-tiles of 2 × 4 tiles (wr | wc << 16), panel order
    int nwt24;
    const WtEntry* wtq;   // [nwtq] the split-fp16 quad form's groups of 2 × 2 wave-tiles (four entries each)
    int nwtq;
    Slot steps[PMAX];
};

hipError_t launch_scan(const ScanParams& p, int precision, hipStream_t st);
int scan_blocks_per_cu(int precision);
size_t scan_lds_bytes(int precision);   // static LDS of the association kernel
// ev_a / ev_b (optional): events timestamped by the dispatch packet itself (hipExtLaunchKernelGGL),
// so timing a flush inserts no marker packets on the stream
hipError_t launch_downdate(const DowndateParams& p, int precision, int grid, hipStream_t st,
                           hipEvent_t ev_a = nullptr, hipEvent_t ev_b = nullptr);
// ex: fp16 storage exponent of the instance (ignored for f32 / f64)
// [t0, t1): the tiles stored (t1 < 0: all); Pll points at tile t0
hipError_t launch_pack(const Dims& d, int precision, const double* Pfull, void* Pll, double* Rs,
                       const int2* tile_rc, int ex, hipStream_t st, int64_t t0 = 0, int64_t t1 = -1);
hipError_t launch_unpack(const Dims& d, int precision, double* Pfull, const void* Pll,
                         const double* Rs, int ex, hipStream_t st, int64_t t0 = 0, int64_t t1 = -1);
hipError_t launch_lowrank(const Dims& d, int precision, const double* diag, const double* U,
                          int rank, void* Pll, double* Rs, const int2* tile_rc, int ex, hipStream_t st,
                          int64_t t0 = 0, int64_t t1 = -1);

}  // namespace ekf
