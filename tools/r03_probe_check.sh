#!/bin/bash
# round-3 probe check: shared-X kernels vs oracle, bench A/B (shared vs distinct X), host cost
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "probe" --timeout 120 --timeout-method thread > gpurun_out/r03_t_probe.log 2>&1 || { tail -30 gpurun_out/r03_t_probe.log; exit 1; }
tail -2 gpurun_out/r03_t_probe.log
timeout -k 10 120 python tools/host_probe_cost.py > gpurun_out/r03_host_cost.log 2>&1 || exit 1
head -1 gpurun_out/r03_host_cost.log
B="python bench.py --no-cpu-baseline --no-ref-torch --no-other-exchange --emulate-wn 1 --steps 20 --warmup 5"
timeout -k 10 300 $B > gpurun_out/r03_b_shared.log 2>&1 || { tail gpurun_out/r03_b_shared.log; exit 1; }
timeout -k 10 300 $B --distinct-x > gpurun_out/r03_b_distinct.log 2>&1 || { tail gpurun_out/r03_b_distinct.log; exit 1; }
python tools/bsum.py gpurun_out/r03_b_shared.log gpurun_out/r03_b_distinct.log
grep -o '"host_ms_parts": {[^}]*}' gpurun_out/r03_b_shared.log
