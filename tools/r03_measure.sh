#!/bin/bash
# round-3 measurement pass: one bench line per workload (fast legs only) + PMC passes on the named workloads
# usage: tools/r03_measure.sh TAG "wl1 wl2 ..." "pmc_wl1 ..."
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; WLS=$2; PMCS=${3:-}
for wl in $WLS; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --init random --no-cpu-baseline --no-ref-torch \
      --no-other-exchange > gpurun_out/r03_m_${TAG}_$wl.log 2>&1 || { tail gpurun_out/r03_m_${TAG}_$wl.log; exit 1; }
  python tools/bsum.py gpurun_out/r03_m_${TAG}_$wl.log
done
for wl in $PMCS; do
  bash tools/pmc_bench.sh ${TAG}_$wl --workload $wl || exit 1
  python tools/pmc_bench_summary.py gpurun_out/pmc_bench_${TAG}_$wl gpurun_out/pmc_${TAG}_$wl.json || exit 1
done
