#!/bin/bash
# K4 change check on the GPU box: the delta / plan / exchange tests, then Wn = 8 timings (tools/k4_wn8_abl.sh 0)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_kernels.py -k "delta or h2" > gpurun_out/k4_tests.log 2>&1 || { tail -30 gpurun_out/k4_tests.log; exit 1; }
tail -1 gpurun_out/k4_tests.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_configs.py -k "layer_step_plan" tests/test_gpu_exchange_full.py tests/test_gpu_ranks_one_gpu.py > gpurun_out/k4_tests2.log 2>&1 || { tail -30 gpurun_out/k4_tests2.log; exit 1; }
tail -1 gpurun_out/k4_tests2.log
bash tools/k4_wn8_abl.sh "$@"
