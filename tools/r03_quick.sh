#!/bin/bash
# quick check after a kernel change: a pytest -k selection of the GPU suite, then short bench lines
# usage: tools/r03_quick.sh TAG "pytest -k expr" "wl ..."
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; K=$2; WLS=$3
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q -k "$K" --timeout 200 --timeout-method thread > gpurun_out/q_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/q_tests_$TAG.log
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/q_tests_$TAG.log | head -20; exit $rc; }
fi
for wl in $WLS; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --no-cpu-baseline --no-ref-torch --no-other-exchange > gpurun_out/q_bench_${TAG}_$wl.log 2>&1 || { tail gpurun_out/q_bench_${TAG}_$wl.log; exit 1; }
  python tools/bsum.py gpurun_out/q_bench_${TAG}_$wl.log 2>/dev/null | head -3
done
