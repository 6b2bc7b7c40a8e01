"""Print the key fields of bench JSON lines (files given on the command line)."""
import json
import sys

for f in sys.argv[1:]:
    try:
        L = [l for l in open(f) if l.startswith("{")][-1]
        d = json.loads(L)
        r = d["roofline"]
        print(f, round(d["value"]), round(d["ms_per_step"], 4), {k: round(v, 4) for k, v in d["kernel_ms"].items()},
              r["bound"], round(r["frac"], 3), [(x["kernel"], round(x["avg_ms"], 3)) for x in r["launch_forms"]])
    except Exception as ex:   # noqa: BLE001
        print(f, "unreadable:", ex)
