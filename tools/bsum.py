"""Summarise bench JSON lines (measurement tool): python tools/bsum.py FILE..."""
import json
import sys

for path in sys.argv[1:]:
    lines = [l for l in open(path) if l.startswith("{")]
    if not lines:
        print(path, "no JSON line")
        continue
    d = json.loads(lines[-1])
    ro = d["roofline"]
    o = dict(ro.get("others", {}))
    o[ro["kernel"]] = ro
    print(f"{path}: value {d['value']} ms/step {d['ms_per_step']} dw {d['dw_ms_per_step']} host {d['host_ms_per_step']}"
          f" init {d.get('init_s')} | probe {ro['probe_total']['ms_per_step']} ms xg {ro['probe_total']['xg_once_GBps']} GB/s")
    for k in sorted(o):
        v = o[k]
        print(f"    {k:16s} {v['per_launch']['avg_us']:10.2f} us x{v['per_launch']['launches']:<6d} {v['achieved']:9.1f} {v['unit']}")
