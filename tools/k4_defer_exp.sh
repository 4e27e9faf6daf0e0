# K4 x3w deferred W merge: parity, then Wn 8 / 4 timing (LLaMA-2-7B, 224 modules) per variant
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "delta" > gpurun_out/k4_tests.log 2>&1 || { tail -30 gpurun_out/k4_tests.log; exit 1; }
tail -1 gpurun_out/k4_tests.log
B="timeout -k 10 200 python tools/delta_bench.py --layers 32 --wn 8 4 --pol 3 --reps 3"
for d in 0 1 2; do echo "defer=$d"; HDP_K4_DEFER=$d $B || exit 1; done
