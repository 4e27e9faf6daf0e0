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
    print(f"{path}: value {d['value']} ms/step {d['ms_per_step']} dw {d['dw_ms_per_step']} host {d['host_ms_per_step']}"
          f" | components {ro.get('component_ms_per_step')}")
    print(f"    dominant {ro['kernel']}: {ro['achieved']} {ro['unit']} frac {ro['frac']} bound {ro['bound']}")
    pl = ro.get("per_launch", {})
    if "phases_us" in pl:
        print(f"    phases (us per group): {pl['phases_us']}")
    for k, v in sorted(ro.get("others", {}).items()):
        print(f"    {k:16s} {v['per_launch']['avg_us']:10.2f} us x{v['per_launch']['launches']:<6d} {v['achieved']:9.1f} "
              f"{v['unit']} frac {v['frac']}")
