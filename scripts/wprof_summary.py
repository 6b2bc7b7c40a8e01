"""Per-kernel averages of the counter passes written by scripts/gpu_wave_prof.sh."""
import collections
import csv
import os
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/wprof"
for sub in sorted(os.listdir(src)):
    path = os.path.join(src, sub, "run_counter_collection.csv")
    if not os.path.exists(path):
        continue
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0].replace("void ekf::", "")
        if "flush" not in k and "scan" not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    for k in agg:
        n = len(disp[k])
        print(sub, k, n, {c: round(v / n) for c, v in agg[k].items()})
    kt = os.path.join(src, sub, "run_kernel_trace.csv")
    durs = collections.defaultdict(list)
    for r in csv.DictReader(open(kt)):
        k = r["Kernel_Name"].split("(")[0].replace("void ekf::", "")
        durs[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    for k, v in durs.items():
        if "flush" in k:
            print("   ", k, "us avg", round(sum(v) / len(v), 1), "n", len(v))
