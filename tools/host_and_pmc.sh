#!/bin/bash
# GPU tests of the layer / queue paths, host-side cProfile of the bench's timed steps, then the
# bench-command PMC passes (FETCH x2 / WRITE / MFMA busy)
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_layer.py tests/test_trajectory.py tests/test_gpu_kernels.py -m gpu -x -q \
  --timeout 120 --timeout-method thread -k "layer or queue or step or trajectory or trainer or probe_group" > gpurun_out/t_layer.log 2>&1 \
  || { tail -30 gpurun_out/t_layer.log; exit 1; }
tail -1 gpurun_out/t_layer.log
timeout -k 10 300 python bench.py --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange \
  --profile-host > gpurun_out/hostprof.log 2>&1 || exit $?
grep -v amdgpu.ids gpurun_out/hostprof.log | head -45
[ "${1:-}" = "pmc" ] || exit 0
bash tools/pmc_bench.sh && python tools/pmc_bench_summary.py gpurun_out/pmc_bench gpurun_out/pmc_bench/summary.json
