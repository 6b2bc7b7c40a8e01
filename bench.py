"""Benchmark: EKF-SLAM updates/s at N=4096 landmarks on MI355X (BASELINE.json metric).

One step = one scan on every EKF instance: Robot::localize (slam_ros/Robot.cpp:126-904) with
L = m = 8 matched lines per instance, s = N - 10 active landmarks, fp32 covariance storage.
Weak scaling: 8 instances per GPU (configs[3]: batch 64 across 8 GPUs). For N > 1 GPUs, rank 0
holds the pre-generated scan payloads and broadcasts each step's payload (all instances) over
RCCL/xGMI; every rank runs its slice of instances (no other collective on the data path).

Inputs are resident in HBM before the timed region. `value` = instances × steps (all ranks)
÷ max-over-ranks wall time of the K timed steps. Before the W warm-up steps an untimed clock
pre-roll (--preroll steps of the same workload, default 200 ≈ 30 ms, reported as
`clock_preroll_steps`) lets the GPU reach the clocks it holds under this load: a step is ≈0.12 ms,
so a few warm-up steps alone measure the clock ramp (≈12 % lower with 8 warm-up steps).

Schedule (defaults): the landmark block is flushed once per T = 20 scans (flush_interval), in
place, between association kernels (--pipeline 1 overlaps them instead), by the split-fp16 flush
(--arith f16x3, slam_ekf.h EKF_ARITH_F16X3: fp32 operands scaled by 2^σ and split into hi + lo
fp16 parts, three fp16 MFMAs per product, fp32 accumulation; held to the fp32 parity bar,
tests/test_bench_config.py; --arith bf16x6 is the exact three-part bf16 split, six products).
With --arith exact (fp32 MFMA, T = 8) every schedule is
bit-identical to a per-scan in-place update (tests/test_gpu_parity.py::
test_deferred_flush_equals_drained). The timed region ends with ekf_sync, which flushes the
partial group: every step's downdate is in P. HIP events in the timed region bracket the flush
kernel only; the association-kernel time is measured on extra steps after it.

roofline: the dominant kernel is the covariance flush (rank-2m MFMA downdate of every step of the
group, one read + write of the packed block). The timed steps may end in a partial group, whose
flush runs another kernel form: every form used is listed in `roofline.launch_forms`, and the
roofline itself is computed over the launches of the form with the largest total time only. Per
launch of that form: algorithmic bytes = instances_per_gpu × n(n+1) × b,
algorithmic flops = steps_per_launch × instances_per_gpu × 2m·n(n+1). `bound` is
whichever roof is the longer ideal time; durations come from HIP events recorded on the stream
the kernel runs on. `traffic` (HBM bytes per launch of that form from FETCH_SIZE/WRITE_SIZE,
gfx950-corrected) is read from profiles/<round>/traffic.json only if it was measured on this very
library build (sha256 of libslam_ekf.so) and configuration; otherwise null.
cpu_baseline (rank 0, N=1 only): B1, the CPU restatement (oracle/, fast mode, fp64) built with
OpenMP on the host cores (bit-identical to its single-thread build), timed on a bounded sample of
the same scans of instance 0; `reference_path` carries B0 (faithful GSL-order restatement, 1 core)
at the same N from profiles/*cpu_baselines.jsonl, measured once on the GPU box's host (≈minutes
per update at N=4096). The same scans also give the per-scan parity numbers
(‖P−P_ref‖_F/‖P_ref‖_F, state, association) from identical inputs.
"""
from __future__ import annotations

import argparse
import glob
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "EKF updates/s at N=4096 landmarks, 1→8 MI355X; ‖P−P_ref‖_F rel-err"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
MFMA_F32_PEAK_TFS = 157.3   # MI355X_MICROARCH.md: dense fp32 MFMA (v_mfma_f32_32x32x2_f32)
MFMA_F64_PEAK_TFS = 78.6    # MI355X_MICROARCH.md: dense fp64 MFMA
MFMA_BF16_PEAK_TFS = 2500.0  # MI355X_MICROARCH.md: dense bf16 MFMA (v_mfma_f32_32x32x16_bf16)
MFMA_F16_PEAK_TFS = 2500.0   # MI355X_MICROARCH.md: dense fp16 MFMA (v_mfma_f32_32x32x16_f16), as bf16
L_LINES = 8


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # the GPU needs a few tens of ms of sustained work to reach its steady clocks: the default
    # warm-up (≈35 ms) is sized for that; fewer warm-up steps under-report by ≈10 %
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--capacity", type=int, default=4096)
    ap.add_argument("--instances", type=int, default=8, help="EKF instances per GPU")
    ap.add_argument("--precision", choices=["f32", "f64", "f16"], default="f32",
                    help="landmark-block storage (f16: fp32 MFMA accumulation, BASELINE config 5)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU baseline sample budget")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--pipeline", type=int, default=0,
                    help="1: overlap the association kernels with the previous group's flush")
    ap.add_argument("--flush-interval", type=int, default=0,
                    help="T: rewrite the landmark block once per T scans (0: 20 with f16x3, 12 "
                         "with bf16x6 or in the survey world, 8 exact and for f64)")
    ap.add_argument("--bcast-every", type=int, default=0,
                    help="scans per broadcast (default: the flush interval); broadcasts run one "
                         "group ahead of the scans that use them")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (= RCCL on ROCm); gloo only to rehearse ranks on one GPU")
    ap.add_argument("--preroll", type=int, default=200,
                    help="untimed clock pre-roll steps before the warm-up (steady GPU clocks)")
    ap.add_argument("--arith", choices=["exact", "bf16x6", "f16x3"], default="f16x3",
                    help="fp32 flush arithmetic (slam_ekf.h EKF_ARITH_*): exact = fp32 MFMA, the state "
                         "bit-identical for every T; bf16x6 = fp32 operands split exactly into three "
                         "bf16 parts, six bf16 MFMAs per product; f16x3 = hi + lo fp16 of 2^σ·V, "
                         "three fp16 MFMAs per product")
    ap.add_argument("--dump-state", default="",
                    help="directory: after all steps each rank writes its instances' final state "
                         "(state_<global instance>.npz: P, y, saved, pose) for multi-rank checks")
    ap.add_argument("--speculate", type=int, choices=[0, 1, 2], default=1,
                    help="association path (EKF_OPT_SPECULATE): 1 speculative (default), 0 the "
                         "sequential chain every scan, 2 every guess wrong (fallback cost)")
    ap.add_argument("--flush-form", type=int, default=0,
                    help="EKF_OPT_FLUSH_FORM (A/B runs): 0 default, 24 the 2 x 4 split flush")
    ap.add_argument("--mfma-replay", type=int, choices=[0, 1, 2], default=1,
                    help="EKF_OPT_MFMA_REPLAY: 1 the split products on the planes (default), 2 fp32 "
                         "MFMA on the fp32 operand rows, 0 the per-element forms")
    ap.add_argument("--scan-threads", type=int, choices=[0, 64, 128, 192], default=0,
                    help="EKF_OPT_SCAN_THREADS: landmarks per association workgroup, 0 automatic")
    ap.add_argument("--force-collective", action="store_true",
                    help="run the scan broadcast through the collective even at one rank (RANK=0, "
                         "WORLD_SIZE=1, MASTER_* in the env): the RCCL device branch on a one-GPU box")
    ap.add_argument("--world", choices=["bench", "survey"], default="bench",
                    help="scan_gen parameter profile: bench (default) or SURVEY.md §8d literally")
    ap.add_argument("--parity-scans", type=int, default=-1,
                    help="scans of the parity leg (-1: three flush groups or --steps if fewer; 0: all "
                         "--steps); its per-group error does not depend on the count")
    ap.add_argument("--traffic-json", default="",
                    help="HBM traffic file (default: the newest profiles/*/traffic.json)")
    args = ap.parse_args()
    if args.force_collective and not args.no_cpu:
        # the parity leg replays the timed steps from the broadcast's receive groups, which the
        # forced collective has already retired (it is a test of the RCCL branch, not a line)
        ap.error("--force-collective needs --no-cpu")
    return args


def build_info(sha, loaded):
    """How the loaded library came to be on this machine: slam_ros_amd/build.py's last_build()
    ("compiled" / "reused" by build() here, or "prebuilt": shipped, build() never ran on this copy),
    and whether that record describes the library this process loaded."""
    from slam_ros_amd import build as B
    rec = B.last_build()
    loaded_default = os.path.abspath(loaded) == os.path.abspath(B.LIB_PATH)
    return {"build_mode": rec.get("mode"), "source_sha": rec.get("source_sha"),
            "record_matches_loaded": loaded_default and rec.get("lib_sha") == sha}


def lib_sha(path):
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()[:16]


def find_traffic(explicit, sha, cfg):
    """Counter-measured HBM bytes per launch for this build and configuration, or (None, why).
    Every profiles/*/traffic.json is considered (newest first): the first one of this configuration
    measured on this very library build wins; files without a "world" key were measured in the
    bench world."""
    paths = [explicit] if explicit else sorted(glob.glob(os.path.join(ROOT, "profiles", "*", "traffic.json")),
                                                key=os.path.getmtime, reverse=True)
    why = "no counter file for this configuration"
    for pth in paths:
        try:
            tj = json.load(open(pth))
        except (OSError, ValueError):
            continue
        # (precision: "f32", or the round-5 files' dtype label "f32 storage, f16x3 products")
        got = dict(tj, precision=str(tj.get("precision", "")).split()[0] if tj.get("precision") else None)
        if all(got.get(k, "bench" if k == "world" else None) == v for k, v in cfg.items()):
            if tj.get("lib_sha") == sha:
                return tj, os.path.relpath(pth, ROOT)
            if why.startswith("no counter"):
                why = f"{os.path.relpath(pth, ROOT)}: measured on another build ({tj.get('lib_sha')})"
    return None, why


def reference_path_baseline(N):
    """B0 (faithful GSL-order restatement, 1 core) at capacity N, measured on the GPU box host."""
    best = None
    for pth in sorted(glob.glob(os.path.join(ROOT, "profiles", "*cpu_baselines.jsonl"))):
        for line in open(pth):
            try:
                r = json.loads(line)
            except ValueError:
                continue
            if r.get("N") == N and str(r.get("baseline", "")).startswith("B0"):
                best = dict(r, source=os.path.relpath(pth, ROOT))
    return best


def rel(a, b):
    nb = np.linalg.norm(b)
    return float(np.linalg.norm(a - b) / (nb if nb > 0 else 1.0))


PARITY_BAR = {"f32": 1e-6, "f16": 1e-3, "f64": 1e-10}   # ‖ΔP‖_F/‖P‖_F (fp16 re-stated)


def parity_leg(ens, O, st, step, scan_of, N, E, K, row0, T, precision, max_scans):
    """Parity of the line of record on its own schedule: this context (same arithmetic, flush
    interval and kernels), payload rows through ekf_localize_device, no drain inside a flush
    group, every instance restarted from the initial state with the payload's first rows (row0 =
    0: the trajectory the pre-roll and the timed steps continue; restarting the initial state on
    the timed rows would make the first predict jump the robot by the ≈10 m the pre-roll drove).
    Instances 0 and E-1 against the CPU restatement (oracle/, fast mode, fp64), SURVEY §8d "per
    scan from identical inputs":
      * y and the pose per scan: they are committed by every scan (read without a drain), so the
        restatement's y and pose are re-synced to the GPU's after every scan and each scan's state
        vector is compared from identical inputs;
      * P per group: at every flush-group end — the only points where the schedule materialises
        P — the restatement is re-synced to the GPU's whole state; the maximum over groups is
        held to the bar. Neither depends on how many scans are checked;
      * per group, y (reported): the state vector at the group end with only P... re-synced at
        group ends (the amplification of the reference's own dynamics over T scans is in it:
        in SURVEY §8d's world the heading error doubles on every scan without a match,
        Robot.cpp:141);
      * trajectory (reported, not barred): a second restatement never re-synced, from the same
        storage-rounded start.
    Association (both restatements) and status are checked on every scan."""
    S = K if max_scans == 0 else min(K, max_scans if max_scans > 0 else 3 * T)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
    check = sorted({0, E - 1})
    grp, traj, scn = {}, {}, {}
    for e in check:
        start = ens.download_state(e)
        grp[e] = O.OracleRobot(N, mode=O.FAST, omp=True)
        grp[e].set_state(*start)
        traj[e] = O.OracleRobot(N, mode=O.FAST, omp=True)
        traj[e].set_state(*start)
        scn[e] = O.OracleRobot(N, mode=O.FAST, omp=True)
        scn[e].set_state(*start)
        del start
    ens.profile(1)
    assoc_ok = True
    groups = []
    y_scan, pose_scan = 0.0, 0.0
    for k in range(S):
        step(row0 + k)
        r = ens.read_results()   # waits for this scan; the flush schedule is untouched
        for e in check:
            enc_e, lines_e = scan_of(row0 + k, e)
            m1 = grp[e].localize(lines_e, enc_e)
            m2 = traj[e].localize(lines_e, enc_e)
            m3 = scn[e].localize(lines_e, enc_e)
            assoc_ok &= (r[e]["match"] == m1 == m2 == m3 and r[e]["status"] == 0)
            _, yk, sk, pk = ens.download_state(e, with_P=False)   # (no drain)
            y_scan = max(y_scan, rel(yk, scn[e].y))
            pose_scan = max(pose_scan, float(np.abs(pk - scn[e].pose).max()))
            scn[e].set_state(None, yk, sk, pk)   # the next scan from the GPU's y and pose
        if (k + 1) % T and k + 1 < S:
            continue
        # a group end: its flush ran (a partial last group is flushed by the drain inside
        # download_state, as the bench's closing ekf_sync flushes it)
        g = {"end_scan": k + 1, "scans": (k % T) + 1}
        for e in check:
            Pg, yg, sg, poseg = ens.download_state(e)
            g[str(e)] = {"p_rel_err": rel(Pg, grp[e].P_t0), "y_rel_err": rel(yg, grp[e].y),
                         "pose_abs_err": float(np.abs(poseg - grp[e].pose).max()),
                         "p_rel_err_trajectory": rel(Pg, traj[e].P_t0),
                         "y_rel_err_trajectory": rel(yg, traj[e].y)}
            assoc_ok &= sg == grp[e].savedLineCount == traj[e].savedLineCount
            g[str(e)]["p_rel_err_scan_resync"] = rel(Pg, scn[e].P_t0)
            grp[e].set_state(Pg, yg, sg, poseg)   # re-sync: the next group from identical inputs
            scn[e].set_state(Pg, yg, sg, poseg)
            del Pg
        groups.append(g)
    pforms = {}
    for ns, _ in ens.profile_flushes():
        pforms[ens.flush_kernel_name(ns)] = pforms.get(ens.flush_kernel_name(ns), 0) + 1
    ens.profile(0)
    del grp, traj, scn
    worst = lambda key: max(g[str(e)][key] for g in groups for e in check)
    bar = PARITY_BAR[precision]
    out = {
        "p_rel_err": max(worst("p_rel_err"), worst("p_rel_err_scan_resync")), "y_rel_err": y_scan,
        "pose_abs_err": pose_scan, "y_rel_err_group": worst("y_rel_err"),
        "pose_abs_err_group": worst("pose_abs_err"),
        "association_identical": bool(assoc_ok),
        "bar": {"p_rel_err": bar, "y_rel_err": 1e-8},
        "trajectory": {"scans": S, "p_rel_err": max(groups[-1][str(e)]["p_rel_err_trajectory"] for e in check),
                       "y_rel_err": max(groups[-1][str(e)]["y_rel_err_trajectory"] for e in check)},
        "groups": groups,
        "scope": (f"the payload's first {S} rows from the initial state through ekf_localize_device in "
                  f"this context (T = {T}, no drain inside a group), flush forms {pforms}; instances {check} "
                  f"vs oracle/ fast mode (fp64). y_rel_err / pose_abs_err: per scan, the restatement's y and "
                  f"pose re-synced to the GPU's after every scan (read without a drain); p_rel_err: per flush "
                  f"group, re-synced at every group end (worst of: the whole state re-synced per group, and y "
                  f"re-synced per scan); y_rel_err_group: y at the group ends with the whole state re-synced "
                  f"per group only (reported); trajectory = a restatement never re-synced over the same {S} scans"),
    }
    out["within_bar"] = bool(out["p_rel_err"] <= bar and out["y_rel_err"] <= 1e-8 and assoc_ok)
    return out


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    from slam_ros_amd import dist as D, ekf, scan_gen as G

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("BENCH_SAME_DEVICE") == "1":   # rehearsal: every rank on device 0
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1 or args.force_collective:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.dist_backend)

    N, E, K, W = args.capacity, args.instances, args.steps, args.warmup
    prec = {"f32": ekf.PREC_F32, "f64": ekf.PREC_F64, "f16": ekf.PREC_F16}[args.precision]
    bpe = {"f32": 4, "f64": 8, "f16": 2}[args.precision]
    E_total = E * world
    first, count = D.shard(E_total, world, rank)
    assert count == E
    n = 3 + 2 * N

    world_map = G.make_world(N)
    profile = None if args.world == "bench" else args.world
    st = G.initial_state(world_map, profile=profile)

    arith = {"exact": ekf.ARITH_EXACT, "bf16x6": ekf.ARITH_BF16X6, "f16x3": ekf.ARITH_F16X3}[args.arith]
    if prec == ekf.PREC_F64:
        arith = ekf.ARITH_EXACT   # the split-bf16 flush serves fp32 operands (fp32 and fp16 storage)
    if args.flush_interval <= 0:
        # per capacity: the flush's pass over P is the part T amortises; below
        # N = 2048 it costs 10-60 µs per launch while every pending step adds replay to every scan
        # (sweeps: scripts/r05/tsweep2.sh)
        if prec == ekf.PREC_F64 or arith == ekf.ARITH_EXACT:
            args.flush_interval = 8
        elif arith == ekf.ARITH_F16X3:
            args.flush_interval = 20 if N > 2048 else (12 if N > 512 else 8)
        else:
            args.flush_interval = 12
    ens = ekf.Ensemble(N, E, prec, max_lines=L_LINES, device=local, pipeline=bool(args.pipeline),
                      flush_interval=args.flush_interval, arith=arith,
                      options={"speculate": args.speculate, "flush_form": args.flush_form,
                               "mfma_replay": args.mfma_replay, "scan_threads": args.scan_threads})
    # one real stream for everything (torch's default stream has handle 0, which the C-ABI reads
    # as "the context's own stream"): the payload copies, the RCCL waits (work.wait() orders the
    # current stream) and the EKF kernels are then ordered on the same queue
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ens.set_stream(stream.cuda_stream)
    for e in range(E):
        ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)

    # ---- pre-generated scan payloads, resident in HBM (rank 0 is the sensor) ----
    PR = max(0, args.preroll)
    steps_total = PR + W + K + W
    per_step = D.payload_len(E_total, L_LINES)
    payload = torch.empty((steps_total, per_step), dtype=torch.float64, device=dev)
    if rank == 0:
        host = np.zeros((steps_total, per_step))
        for s in range(steps_total):
            enc, lines, _ = G.make_scan(world_map, s + 1, instances=E_total, lines=L_LINES, profile=profile)
            host[s] = D.pack(enc, lines)
        payload.copy_(torch.from_numpy(host))
    nlines = torch.full((E,), L_LINES, dtype=torch.int32, device=dev)
    # N > 1: rank 0 broadcasts B scans (all instances) per collective, one group ahead of the
    # scans that use them (slam_ros_amd/dist.py GroupedBroadcast)
    B = max(1, args.bcast_every or args.flush_interval)
    host_coll = world > 1 and args.dist_backend != "nccl"   # rehearsal: collectives on host tensors
    bc = D.GroupedBroadcast(payload, B, dist, rank, world, src=0, host_coll=host_coll,
                            sync=lambda: torch.cuda.synchronize(dev), force=args.force_collective)
    bc.start()
    torch.cuda.synchronize(dev)

    eo, lo = D.offsets(E_total, L_LINES, first)
    nl_ptr = nlines.data_ptr()
    if bc.coll:
        def step(s):
            base = bc.step_buffer(s).data_ptr()
            ens.localize_device(base + eo * 8, base + lo * 8, nl_ptr)
    else:
        # one rank: the payload rows' addresses computed once, so the timed loop is one C-ABI call
        # per step (a slow or shared host then cannot starve the GPU of launches)
        row_bytes = payload.stride(0) * payload.element_size()
        p0 = payload.data_ptr()
        ptrs = [(p0 + s * row_bytes + eo * 8, p0 + s * row_bytes + lo * 8) for s in range(steps_total)]

        def step(s):
            e_ptr, l_ptr = ptrs[s]
            ens.localize_device(e_ptr, l_ptr, nl_ptr)

    for s in range(PR):             # clock pre-roll (untimed)
        step(s)
    for s in range(PR, PR + W):     # warm-up (untimed)
        step(s)
    ens.sync()                      # flush the partial group: the timed region starts clean
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    ens.profile(1)                  # HIP events around the flush kernel only (2 per group)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for s in range(PR + W, PR + W + K):
        step(s)
    t_enq = time.perf_counter() - t0   # host time to issue the K steps (informational)
    ens.sync()                      # every step's downdate is in the landmark block
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    prof = ens.profile_read()
    flushes = ens.profile_flushes()
    ens.profile(0)
    # association-kernel time (informational): a few more steps with every kernel timed, outside
    # the timed region
    ens.profile(2)
    for s in range(W):
        step(PR + W + K + s)
    ens.sync()
    scan_ms = ens.profile_read()["scan_ms"]
    ens.profile(0)
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device="cpu" if host_coll else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())

    if args.dump_state:
        os.makedirs(args.dump_state, exist_ok=True)
        for e in range(E):
            P_, y_, s_, pose_ = ens.download_state(e)
            np.savez(os.path.join(args.dump_state, f"state_{first + e}.npz"), P=P_, y=y_, saved=s_, pose=pose_)
        del P_
    res = ens.read_results()
    # a step counts only if it committed a valid update: every line matched, no augmentation or
    # reset, and no status bit (a timed-out exchange rolls the call back, EKF_ST_SYNC_TIMEOUT)
    all_matched = all(r["matches"] == L_LINES and r["saved"] == st.saved and not r["reset"]
                      and r["status"] == 0 for r in res)
    if world > 1:
        ok = torch.tensor([1 if all_matched else 0], dtype=torch.int32, device="cpu" if host_coll else dev)
        dist.all_reduce(ok, op=dist.ReduceOp.MIN)
        all_matched = bool(ok.item())

    value = E_total * K / elapsed
    # launch forms of the timed flushes; the roofline covers the dominant one only
    forms = {}
    for ns, ms in flushes:
        f = forms.setdefault(ns, {"kernel": ens.flush_kernel_name(ns), "steps_per_launch": ns,
                                  "launches": 0, "total_ms": 0.0})
        f["launches"] += 1
        f["total_ms"] += ms
    for f in forms.values():
        f["avg_ms"] = f["total_ms"] / f["launches"]
    dom = max(forms.values(), key=lambda f: f["total_ms"]) if forms else None
    dd_ms = dom["avg_ms"] if dom else prof["downdate_ms"]
    steps_per_launch = dom["steps_per_launch"] if dom else args.flush_interval
    alg_bytes = E * n * (n + 1) * bpe   # one read + write of the packed block per flush
    alg_flops = steps_per_launch * E * 2 * L_LINES * n * (n + 1)
    kname = dom["kernel"] if dom else ""
    # split-fp16 forms: the 2 x 2 wave form <.., true, true>, the 2 x 4 form <.., true> of
    # flush_bf24_kernel, the quad form flush_f16q_kernel; split-bf16: the other <.., true> forms
    f16_form = (kname.endswith(", true, true>") or kname.startswith("flush_f16q_kernel")
                or (kname.startswith("flush_bf24_kernel") and kname.endswith(", true>")))
    bf_form = not f16_form and (kname.endswith(", true>") or kname.startswith("flush_bf24_kernel"))
    # the MFMA roof of the instruction the flush executes: the split-bf16 flush runs six bf16
    # products per fp32 product (executed flops = 6 x algorithmic, dense bf16 peak); the exact
    # forms run v_mfma_f32_32x32x2_f32 (fp32 and fp16 storage) or v_mfma_f64_16x16x4_f64
    if f16_form:
        mfma_mult, mfma_peak, mfma_dtype = 3, MFMA_F16_PEAK_TFS, "f16 (three split products per fp32 product)"
    elif bf_form:
        mfma_mult, mfma_peak, mfma_dtype = 6, MFMA_BF16_PEAK_TFS, "bf16 (six split products per fp32 product)"
    elif prec == ekf.PREC_F64:
        mfma_mult, mfma_peak, mfma_dtype = 1, MFMA_F64_PEAK_TFS, "f64"
    else:
        mfma_mult, mfma_peak, mfma_dtype = 1, MFMA_F32_PEAK_TFS, "f32"
    t_hbm = alg_bytes / (HBM_PEAK_GBS * 1e9)
    t_mfma = mfma_mult * alg_flops / (mfma_peak * 1e12)
    bound = "hbm" if t_hbm >= t_mfma else "mfma"
    gbs = alg_bytes / (dd_ms * 1e-3) / 1e9 if dd_ms > 0 else None
    tfs = alg_flops / (dd_ms * 1e-3) / 1e12 if dd_ms > 0 else None    # fp32-equivalent (algorithmic)
    xtfs = mfma_mult * tfs if tfs else None                             # executed, in mfma_dtype
    lib_file = ekf.loaded_path or ekf.LIB_PATH
    sha = lib_sha(lib_file)
    tj, traffic_src = find_traffic(args.traffic_json, sha, {
        "capacity": N, "instances": E, "precision": args.precision, "flush_interval": args.flush_interval,
        "pipeline": bool(args.pipeline), "kernel": dom["kernel"] if dom else None, "world": args.world})
    traffic = tj.get("hbm_bytes_per_launch") if tj else None

    out = {
        "metric": METRIC,
        "value": value,
        "unit": "updates/s",
        "n_gpus": world,
        "steps": K,
        "warmup": W,
        "ms_per_step": elapsed / K * 1e3,
        "host_issue_ms_per_step": t_enq / K * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": f"{args.precision} storage, {args.arith if prec != ekf.PREC_F64 else 'exact'} products" if prec != ekf.PREC_F64 else "f64",
        "data": "synthetic (seeded line-landmark world and scans, SURVEY.md §8d)",
        "config": {
            "workload": (f"N={N} landmarks (n={n}), {E} EKF instances/GPU, L=m={L_LINES} matched "
                         f"lines/scan, s=N-10 active, {args.precision} covariance storage" if args.world == "bench" else
                         f"N={N} landmark capacity (n={n}), {E} EKF instances/GPU, L={L_LINES} lines/scan of "
                         f"SURVEY §8d's world after a {PR}-scan pre-roll (most lines new landmarks, map resets; "
                         f"the reference's motion model has run away, DESIGN §2.1), {args.precision} covariance storage"),
            "capacity": N, "instances_per_gpu": E, "global_batch": E_total,
            "lines_per_scan": L_LINES,
            "parallelism": (f"ensemble x{world} ({'RCCL' if args.dist_backend == 'nccl' else args.dist_backend} "
                            f"broadcast of {B} scans per collective)") if world > 1 else "ensemble x1",
                "pipeline": bool(args.pipeline), "flush_interval": args.flush_interval,
            "arith": {ekf.ARITH_EXACT: "exact", ekf.ARITH_BF16X6: "bf16x6", ekf.ARITH_F16X3: "f16x3"}[arith],
            "association": {0: "sequential", 1: "speculative", 2: "speculative, every guess wrong"}[args.speculate],
            "world": args.world,
        },
        "clock_preroll_steps": PR,
        "roofline": {
            "bound": bound,
            "achieved": gbs if bound == "hbm" else xtfs,
            "peak": HBM_PEAK_GBS if bound == "hbm" else mfma_peak,
            "unit": "GB/s" if bound == "hbm" else "TFLOP/s",
            "frac": ((gbs / HBM_PEAK_GBS) if bound == "hbm" else (xtfs / mfma_peak)) if dd_ms > 0 else None,
            "traffic": traffic,
            "kernel": dom["kernel"] if dom else None,
            "launch_forms": sorted(forms.values(), key=lambda f: -f["total_ms"]),
            "alg_bytes_per_launch": alg_bytes,
            "alg_flops_per_launch": alg_flops,
            "steps_per_launch": steps_per_launch,
            "hbm_gbs": gbs, "hbm_frac": (gbs / HBM_PEAK_GBS) if gbs else None,
            "mfma_tflops": xtfs, "mfma_peak": mfma_peak, "mfma_frac": (xtfs / mfma_peak) if xtfs else None,
            "mfma_dtype": mfma_dtype, "fp32_equiv_tflops": tfs,
            "mfma_frac_basis": (f"executed MFMA flops ({mfma_mult} x the algorithmic 2m·n(n+1) per step) "
                                f"vs the dense {mfma_dtype.split()[0]} MFMA peak {mfma_peak} TF/s"),
            "ideal_ms": max(t_hbm, t_mfma) * 1e3,
            # north_star's "fraction of the fp32 MFMA roofline", end to end: the algorithmic flops
            # of every update one GPU completes per second (2m·n(n+1) each) over the dense fp32 peak
            "fp32_mfma_frac_end_to_end": (value / world) * 2 * L_LINES * n * (n + 1) / (MFMA_F32_PEAK_TFS * 1e12),
            "traffic_source": traffic_src,
            "lib_sha": sha,
        },
        "build": build_info(sha, lib_file),
        "kernel_ms": {"scan": scan_ms, "flush": dd_ms, "flush_launches": prof["launches"]},
        "all_lines_matched": all_matched,
        "cpu_baseline": None,
    }
    if not all_matched:
        out["last_step_results"] = [{"matches": r["matches"], "saved": r["saved"],
                                     "reset": r["reset"], "status": r["status"]} for r in res]

    if rank == 0 and world == 1 and not args.no_cpu:
        from oracle import oracle as O
        cores = O.threads(True)
        host = payload.cpu().numpy()

        def scan_of(row, e):
            enc = host[row, 3 * (first + e): 3 * (first + e) + 3]
            lo = E_total * 3 + (first + e) * L_LINES * 6
            return enc, host[row, lo: lo + L_LINES * 6].reshape(L_LINES, 6)

        parity = parity_leg(ens, O, st, step, scan_of, N, E, K, 0, args.flush_interval,
                            args.precision, args.parity_scans)
        # CPU baseline: B1 on a bounded sample of instance 0's scans
        ens.init_lowrank(0, st.diag, st.U, st.y, st.saved, st.pose)
        P0, y0, s0, pose0 = ens.download_state(0)
        ref = O.OracleRobot(N, mode=O.FAST, omp=True)
        ref.set_state(P0, y0, s0, pose0)
        del P0
        scans = 0
        t_cpu = 0.0
        while True:
            enc, lines = scan_of(scans, 0)
            t1 = time.perf_counter()
            ref.localize(lines, enc)
            t_cpu += time.perf_counter() - t1
            scans += 1
            if t_cpu >= args.cpu_seconds or scans >= steps_total:
                break
        b0 = reference_path_baseline(N)
        out["cpu_baseline"] = {
            "value": scans / t_cpu, "unit": "updates/s", "cores": cores, "kind": "port",
            "sample": f"B1: {scans} consecutive scans of instance 0 (N={N}, L=m={L_LINES}) through "
                      f"oracle/ekf_oracle.c fast mode (fp64, sparse predict/gating, dense O(n^2) "
                      f"update per match), OpenMP build on {cores} host threads, {t_cpu:.1f} s",
            "host_cpus": O.host_cpus(),
            "reference_path": ({"name": "B0: faithful GSL-order restatement (n^3 predict, dense "
                                        "H·P·Hᵀ per candidate), 1 core", "value": b0["updates_per_s"],
                                "unit": "updates/s", "cores": 1, "host": b0.get("host_cpu"),
                                "source": b0["source"]} if b0 else None),
        }
        out["parity"] = parity
        out["speedup_vs_cpu_baseline"] = value / out["cpu_baseline"]["value"]
        if b0:
            out["speedup_vs_reference_path"] = value / b0["updates_per_s"]

    if args.force_collective:
        out["config"]["parallelism"] += f" (scan broadcast forced through the {args.dist_backend} collective)"
    if rank == 0:
        print(json.dumps(out))
    ens.close()
    if world > 1 or args.force_collective:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
