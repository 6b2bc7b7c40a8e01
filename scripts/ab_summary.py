"""Summarise an A/B run (scripts/r03/ab.sh): per variant and repetition the bench value, scan and
flush times, and the association phase stamps. usage: python scripts/ab_summary.py <tag> [keys]"""
import glob
import json
import os
import sys

tag = sys.argv[1]
keys = sys.argv[2].split(",") if len(sys.argv) > 2 else ["records+stage", "staged_replay(w0)", "replay_wave_total",
                                                          "landmark_total", "lw_gate", "lw_gain+store", "total"]
d = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out", tag)
rows = []
for f in sorted(glob.glob(os.path.join(d, "bench_*.json"))):
    name = os.path.basename(f)[6:-5]
    b = next((json.loads(l) for l in open(f) if l.startswith("{")), None)
    pf = os.path.join(d, f"probe_{name}.txt")
    pr = next((json.loads(l) for l in open(pf) if l.startswith("{")), None) if os.path.exists(pf) else None
    row = [name]
    if b:
        row += [f"{b['value']/1e3:.1f}k", f"scan {b['kernel_ms']['scan']*1e3:.1f}", f"flush {b['kernel_ms']['flush']*1e3:.0f}"]
    if pr:
        row += [f"{k.split('(')[0]} {pr['us'].get(k, float('nan')):.2f}" for k in keys]
    rows.append("  ".join(row))
print("\n".join(rows))
