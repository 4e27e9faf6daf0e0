#!/bin/bash
# round-3: the whole GPU suite, smoke, and one default bench line (each step time-limited)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-v1}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_$TAG.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r03_gpu_tests_$TAG.log
[ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r03_gpu_tests_$TAG.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_$TAG.log 2>&1 || { tail gpurun_out/r03_smoke_$TAG.log; exit 1; }
tail -1 gpurun_out/r03_smoke_$TAG.log
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r03_bench_$TAG.log 2>&1 || { tail gpurun_out/r03_bench_$TAG.log; exit 1; }
python tools/bsum.py gpurun_out/r03_bench_$TAG.log
grep -o '"host[a-z_]*": [0-9.{][^,]*' gpurun_out/r03_bench_$TAG.log | head
