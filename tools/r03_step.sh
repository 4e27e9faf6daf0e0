#!/bin/bash
# round-3 iteration: targeted GPU tests, then bench lines of the named workloads (fast legs)
# usage: tools/r03_step.sh TAG "pytest -k expr" "wl1 wl2 ..." [extra bench args]
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; K=$2; WLS=${3:-}; shift 3; EXTRA="$*"
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" \
      > gpurun_out/r03_t_$TAG.log 2>&1
  rc=$?; tail -3 gpurun_out/r03_t_$TAG.log
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/r03_t_$TAG.log | head -30; exit $rc; }
fi
for wl in $WLS; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --init random --no-cpu-baseline --no-ref-torch \
      --no-other-exchange $EXTRA > gpurun_out/r03_b_${TAG}_$wl.log 2>&1 || { tail gpurun_out/r03_b_${TAG}_$wl.log; exit 1; }
  python tools/bsum.py gpurun_out/r03_b_${TAG}_$wl.log
done
