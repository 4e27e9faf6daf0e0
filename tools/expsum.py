"""Summarise tools/env_exp.sh outputs: python tools/expsum.py gpurun_out/exp_VAR_*.json"""
import json
import sys

for p in sys.argv[1:]:
    try:
        d = json.loads([l for l in open(p) if l.startswith("{")][-1])
    except Exception as e:  # noqa: BLE001
        print(p, "ERR", e)
        continue
    r = d["roofline"]
    ph = r.get("per_launch", {}).get("phases_us") or r.get("probe", {}).get("per_launch", {}).get("phases_us")
    print(f"{p}: value {d['value']} ms/step {d['ms_per_step']} dw {d['dw_ms_per_step']} comp {r.get('component_ms_per_step')}"
          f" phases {ph}")
    for k, v in sorted(r.get("others", {}).items()):
        print(f"    {k:20s} {v['per_launch']['avg_us']:10.2f} us x{v['per_launch']['launches']:<5d} {v['achieved']:8.1f} {v['unit']}")
