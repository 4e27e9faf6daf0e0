#!/bin/bash
# team kernel experiment: correctness subset, trace, bench A/B over the OUTER lag
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "team" > gpurun_out/t_team.log 2>&1 || { tail -30 gpurun_out/t_team.log; exit 1; }
tail -1 gpurun_out/t_team.log
timeout -k 10 300 python tools/team_trace.py 672 32 > gpurun_out/trace.log 2>&1 || { tail gpurun_out/trace.log; exit 1; }
cat gpurun_out/trace.log
for lag in 8 12; do
  HDP_PROBE_PATH=team HDP_TM_L=$lag timeout -k 10 300 python bench.py --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange \
    > gpurun_out/ab_L$lag.log 2>&1 || exit $?
  python - "$lag" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_L{sys.argv[1]}.log") if l.startswith("{")][-1])
r = d["roofline"]
print("L", sys.argv[1], d["value"], d["ms_per_step"], "host", d["host_ms_per_step"], r["component_ms_per_step"],
      r.get("per_launch", {}).get("avg_us"), r.get("frac"))
PY
done
