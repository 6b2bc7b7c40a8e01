"""Host enqueue cost per step vs GPU time per step (N=4096, 8 instances, f32)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch
from slam_ros_amd import dist as D, ekf, scan_gen as G

N, E, L, T = 4096, 8, 8, int(os.environ.get("T", 4))
K = 48
w = G.make_world(N); st = G.initial_state(w)
ens = ekf.Ensemble(N, E, ekf.PREC_F32, max_lines=L, flush_interval=T)
dev = torch.device("cuda", 0)
stream = torch.cuda.current_stream(dev)
ens.set_stream(stream.cuda_stream)
for e in range(E):
    ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
host = np.stack([D.pack(*G.make_scan(w, s + 1, instances=E, lines=L)[:2]) for s in range(K + 8)])
payload = torch.from_numpy(host).to(dev)
nl = torch.full((E,), L, dtype=torch.int32, device=dev)
ptrs = [(payload[s].data_ptr(), payload[s].data_ptr() + E * 3 * 8) for s in range(K + 8)]
for prof in (False, True, False, True):
    for mode in ("raw-ptrs",):
        for e in range(E):
            ens.init_lowrank(e, st.diag, st.U, st.y, st.saved, st.pose)
        ens.sync(); torch.cuda.synchronize()
        ens.profile(prof)
        t0 = time.perf_counter()
        for s in range(K):
            if mode == "torch-index":
                b = payload[s].data_ptr()
                ens.localize_device(b, b + E * 3 * 8, nl.data_ptr())
            else:
                ens.localize_device(ptrs[s][0], ptrs[s][1], nl.data_ptr())
        t1 = time.perf_counter()
        ens.sync(); torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"profile={prof} {mode}: enqueue {1e6*(t1-t0)/K:.1f} us/step, total {1e6*(t2-t0)/K:.1f} us/step")
        ens.profile(False)
