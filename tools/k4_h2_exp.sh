# K4 H2 (fp16x2 scaled split): parity, then Wn 8 / 4 timing (LLaMA-2-7B, 224 modules): H2 with
# and without the deferred merge, and bf16x3
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "delta" > gpurun_out/k4_tests.log 2>&1 || { tail -40 gpurun_out/k4_tests.log; exit 1; }
tail -1 gpurun_out/k4_tests.log
B="timeout -k 10 200 python tools/delta_bench.py --layers 32 --wn 8 4 --pol 3 --reps 3"
echo h2; $B || exit 1
echo h2-nodefer; HDP_K4_DEFER=0 $B || exit 1
echo x3; $B --math x3 || exit 1
