#!/bin/bash
# box-level spread of the headline bench line: N back-to-back runs of the default workload
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for k in $(seq 1 ${N:-3}); do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ref-torch --no-other-exchange > gpurun_out/var_$k.log 2>&1 || { tail gpurun_out/var_$k.log; exit 1; }
  python tools/bsum.py gpurun_out/var_$k.log 2>/dev/null | head -1
done
