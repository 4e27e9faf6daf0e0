"""One-line summaries of bench JSON lines (measurement helper): value, ms/step, components, Wn=8 dW, init."""
import json
import sys

for p in sys.argv[1:]:
    for l in open(p):
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        rf = d["roofline"]
        c = rf.get("component_ms_per_step", {})
        o = rf.get("others", {})
        ad = o.get("adam", {}).get("per_launch", {})
        print(d["config"]["workload"], "value", d["value"], "ms", d["ms_per_step"], "dw", d.get("dw_ms_per_step"),
              "frac", rf["frac"], "comp", c, "wn8", (d.get("dw_emulated_wn") or {}).get("ms"),
              "x", (d.get("dw_emulated_wn") or {}).get("speedup"), "ref_dw", (d.get("ref_torch_gpu") or {}).get("speedup_dw"),
              "init", d.get("init_s"), "adam_us", ad.get("avg_us"))
