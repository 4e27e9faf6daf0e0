#!/bin/bash
# A/B of the probe paths on the bench workload (team = default vs sweep), quick bench lines
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for path in team sweep; do
  if [ $path = sweep ]; then unset HDP_PROBE_PATH; else export HDP_PROBE_PATH=$path; fi
  timeout -k 10 300 python bench.py --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange "$@" \
    > gpurun_out/ab_$path.log 2>&1 || exit $?
  python - "$path" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][-1])
r = d["roofline"]
print(sys.argv[1], d["value"], d["ms_per_step"], "host", d["host_ms_per_step"], r["component_ms_per_step"],
      r.get("per_launch", {}).get("avg_us"), r.get("frac"))
PY
done
