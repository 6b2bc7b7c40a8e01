"""Kernel timeline from a rocprofv3 kernel-trace CSV: per-kernel durations and the idle gaps
between consecutive kernels (the last `n` kernels)."""
import csv, sys
path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kt/run_kernel_trace.csv"
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ks = [(r["Kernel_Name"].split("(")[0][-34:], int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
prev = None
for name, s, e in ks[-n:]:
    gap = (s - prev) / 1000 if prev else 0.0
    print(f"{name:36s} dur {(e - s) / 1000:8.1f} us  gap {gap:6.1f} us")
    prev = e
