#!/bin/bash
# team kernel: register-holding variants (HDP_TM_HOLD = D L) vs the re-read default
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "team" > gpurun_out/t_team.log 2>&1 || { tail -30 gpurun_out/t_team.log; exit 1; }
tail -1 gpurun_out/t_team.log
for h in 0 53 63 64; do
  HDP_TM_HOLD=$h timeout -k 10 120 python tools/team_trace.py 672 32 > gpurun_out/thold_$h.log 2>&1 || { tail gpurun_out/thold_$h.log; exit 1; }
  echo "hold=$h $(grep -E '^group' gpurun_out/thold_$h.log)"; grep -E "step period|OUTER wait" gpurun_out/thold_$h.log
done
HDP_TM_HOLD=64 HDP_TM_DBG=1 timeout -k 10 120 python tools/team_trace.py 672 32 > gpurun_out/thold_64_nowait.log 2>&1; echo "hold=64 no-wait $(grep -E '^group' gpurun_out/thold_64_nowait.log)"
