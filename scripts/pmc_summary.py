"""Summarise a scripts/pmc_profile.sh run into profiles/<tag>/: kernel stats, per-kernel counter
averages, and traffic.json for the bench's dominant flush form (HBM bytes per launch =
2 × FETCH_SIZE + WRITE_SIZE, in KB × 1024: MI355X_MICROARCH.md HBM section, gfx950 FETCH_SIZE
reports half of a 16-B/lane streaming read), stamped with the sha256 of libslam_ekf.so so that
bench.py uses it only for this very build. usage: python scripts/pmc_summary.py <tag>"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def demangle(name):
    """rocprofv3 leaves some names mangled (the _Float16 instantiations)."""
    if not name.startswith("_Z"):
        return name
    try:
        import subprocess
        tool = "/opt/rocm/lib/llvm/bin/llvm-cxxfilt"
        tool = tool if os.path.exists(tool) else "c++filt"
        out = subprocess.run([tool, name], capture_output=True, text=True).stdout.strip()
        return out or name
    except OSError:
        return name


def counters(path):
    acc = defaultdict(lambda: defaultdict(list))
    if not os.path.exists(path):
        return {}
    with open(path) as f:
        for r in csv.DictReader(f):
            acc[demangle(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in acc.items()}


def main(tag, out=None):
    import bench
    from slam_ros_amd import ekf
    src = os.path.join(ROOT, "gpurun_out", tag)
    out = out or os.path.join(ROOT, "profiles", tag)
    os.makedirs(out, exist_ok=True)
    shutil.copy(os.path.join(src, "kt", "run_kernel_stats.csv"), os.path.join(out, "kernel_stats.csv"))
    shutil.copy(os.path.join(src, "bench.json"), os.path.join(out, "bench.json"))
    ctr = {}
    for sub in ("fetch", "write", "sq", "l2", "insts"):
        for k, v in counters(os.path.join(src, sub, "run_counter_collection.csv")).items():
            ctr.setdefault(k, {}).update(v)
    json.dump(ctr, open(os.path.join(out, "counters_avg_per_dispatch.json"), "w"), indent=1)
    b = json.load(open(os.path.join(out, "bench.json")))
    kern = b["roofline"]["kernel"]
    def same(k):
        if kern.split("<")[0] not in k:
            return False
        if "<" not in kern:
            return True
        if kern[kern.index("<"):].replace(" ", "") in k.replace(" ", ""):
            return True
        if k.startswith("_Z"):   # still mangled: Itanium template arguments
            args = [a.strip() for a in kern[kern.index("<") + 1:-1].split(",")]
            code = {"float": "f", "double": "d", "_Float16": "DF16_", "true": "Lb1E", "false": "Lb0E"}
            want = "I" + "".join(code.get(a, "Li%sE" % a) for a in args) + "E"
            return want in k
        return False
    match = [k for k in ctr if same(k)]
    if not match:
        print("no counters for", kern, list(ctr)[:5])
        return
    c = ctr[match[0]]
    hbm = 2 * c.get("FETCH_SIZE", 0) * 1024 + c.get("WRITE_SIZE", 0) * 1024
    cfg = b["config"]
    tj = {"capacity": cfg["capacity"], "instances": cfg["instances_per_gpu"], "precision": str(b["dtype"]).split()[0],
          "flush_interval": cfg["flush_interval"], "pipeline": cfg["pipeline"], "kernel": kern,
          "hbm_bytes_per_launch": hbm, "fetch_bytes_corrected": 2 * c.get("FETCH_SIZE", 0) * 1024,
          "write_bytes": c.get("WRITE_SIZE", 0) * 1024,
          "alg_bytes_per_launch": b["roofline"]["alg_bytes_per_launch"],
          "traffic_over_alg": hbm / b["roofline"]["alg_bytes_per_launch"],
          "sq": {k: v for k, v in c.items() if k.startswith("SQ_") or k.startswith("GRBM")},
          "l2": {k: v for k, v in c.items() if k.startswith("TCC_HIT") or k.startswith("TCC_MISS")},
          "lib_sha": bench.lib_sha(ekf.LIB_PATH), "source": f"profiles/{tag}/counters_avg_per_dispatch.json",
          "arith": cfg.get("arith"), "world": cfg.get("world", "bench")}
    json.dump(tj, open(os.path.join(out, "traffic.json"), "w"), indent=1)
    print(json.dumps({k: tj[k] for k in ("kernel", "hbm_bytes_per_launch", "traffic_over_alg")}))
    # instructions per wave of the association kernel (SQ_INSTS_* / SQ_WAVES per dispatch) and per
    # line (÷ the scan's L lines): the chain's instruction count
    scan = [k for k in ctr if "scan_kernel" in k and "SQ_WAVES" in ctr[k]]
    if scan:
        L = cfg.get("lines_per_scan", 8)
        ins = {}
        for k in scan:
            c2 = ctr[k]
            w = max(c2["SQ_WAVES"], 1.0)
            per = {n[len("SQ_INSTS_"):].lower(): c2[n] / w for n in c2 if n.startswith("SQ_INSTS_")}
            per["total"] = sum(per.get(x, 0) for x in ("valu", "salu", "lds", "smem", "vmem", "branch"))
            per["total_per_line"] = per["total"] / L
            ins[k] = {"waves_per_dispatch": c2["SQ_WAVES"], "per_wave": per}
        json.dump(ins, open(os.path.join(out, "scan_instructions.json"), "w"), indent=1)
        for k, v in ins.items():
            print("scan instructions per wave", k[:60], round(v["per_wave"]["total"]), "per line",
                  round(v["per_wave"]["total_per_line"]))
    sq = tj["sq"]
    if sq.get("SQ_WAVE_CYCLES"):
        print("SQ_WAIT_ANY/WAVE", sq.get("SQ_WAIT_ANY", 0) / sq["SQ_WAVE_CYCLES"],
              "MFMA_BUSY/BUSY", sq.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / max(sq.get("SQ_BUSY_CYCLES", 1), 1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None)
