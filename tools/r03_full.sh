#!/bin/bash
# round-3: the whole GPU suite, smoke, the default bench line under rocprofv3 --kernel-trace --stats, K5 variants
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-v2}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_gpu_tests_$TAG.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r03_gpu_tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_$TAG.log 2>&1 || { tail gpurun_out/r03_smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/r03_smoke_$TAG.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_$TAG.log 2>&1 || { tail gpurun_out/r03_bench_$TAG.log; exit 1; }
python tools/bsum.py gpurun_out/r03_bench_$TAG.log
rm -rf /tmp/rp_$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp_$TAG -o run -- python3 bench.py --steps 10 --warmup 3 \
    --init random --no-cpu-baseline --no-ref-torch > gpurun_out/r03_bench_${TAG}_under_rocprof.log 2>&1 || exit 1
f=$(find /tmp/rp_$TAG -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r03_rocprof_bench_kernel_stats_$TAG.csv
if [ -x tools/bin/merge_bw ]; then timeout -k 10 120 tools/bin/merge_bw > gpurun_out/merge_bw_$TAG.log 2>&1; cat gpurun_out/merge_bw_$TAG.log; fi
