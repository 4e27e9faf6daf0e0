#!/bin/bash
# team kernel cost breakdown (HDP_TM_DBG switches remove one cost at a time; numbers are wrong)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for dbg in 0 1 3 7 15 13; do
  HDP_TM_DBG=$dbg timeout -k 10 120 python tools/team_trace.py 672 32 > gpurun_out/tdbg_$dbg.log 2>&1 || { tail gpurun_out/tdbg_$dbg.log; exit 1; }
  echo "dbg=$dbg $(grep -E '^group' gpurun_out/tdbg_$dbg.log) | $(grep 'step period' gpurun_out/tdbg_$dbg.log | awk '{print "period p50", $8}')"
done
