// ekf_commit.h — the association kernel's commit decision (host + device, no HIP dependency, so
// that tests/test_abi.py compiles it on the host).
#pragma once

#include "../../include/slam_ekf.h"
#include "ekf_layout.h"

namespace ekf {

// Completion word of an association workgroup (sync[SYNC_WG0 + g]): bits 31..8 the launch epoch
// (mod 2^24), 7..0 the status bits it saw. The lead commits the launch only if every workgroup's
// word carries this epoch and no timeout (commit_status); otherwise the instance keeps the state
// from before the call (the launch wrote only the inactive copy of the robot strip and mean).
EKF_HD unsigned done_word(unsigned epoch, int status) { return ((epoch & 0xffffffu) << 8) | ((unsigned)status & 0xffu); }

// bit 7 of a completion word (not a status bit): the workgroup wrote a nonzero operand row this
// step (its landmarks bound the downdate's nonzero columns: RES_ZMAX)
constexpr unsigned DONE_NZ = 128u;
// bit 6 (not a status bit): a landmark of the workgroup is below the split-fp16 planes' dynamic
// range this step (PLANE_VAR_MIN); the lead records the step's σ as PLANE_SIGMA_EXACT
constexpr unsigned DONE_PLOSS = 64u;
// the status bits of a completion word (the rest are DONE_* flags)
constexpr int DONE_STATUS_MASK = 0x3f;

// The lead's decision from the G completion words as last seen (words[0] is its own): the OR of
// the status bits, with EKF_ST_SYNC_TIMEOUT added for every word not (yet) of this epoch. The
// launch commits iff the result has no timeout bit.
EKF_HD int commit_fold(int st, unsigned word, unsigned epoch)
{
    return st | (((word >> 8) != (epoch & 0xffffffu)) ? (int)EKF_ST_SYNC_TIMEOUT : (int)(word & 0x7fu));
}

EKF_HD int commit_status(const unsigned* words, int G, unsigned epoch)
{
    int st = 0;
    for (int g = 0; g < G; g++) st = commit_fold(st, words[g], epoch);
    return st;
}

}  // namespace ekf
