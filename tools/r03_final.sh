#!/bin/bash
# round-3 final evidence for the named workloads: PMC passes (FETCH / WRITE / MFMA busy) over the bench
# command -> profiles/r03_pmc_bench_<wl>.json (the bench's roofline `traffic` source on these kernel
# sources), then the bench line and a rocprofv3 --kernel-trace --stats summary of the same command.
# usage: tools/r03_final.sh TAG "wl ..." [tests]     (tests: also the whole GPU suite and smoke first)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; WLS=$2; T=${3:-}
if [ "$T" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r03_gpu_tests_$TAG.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/r03_gpu_tests_$TAG.log
  [ $rc -ne 0 ] && { grep -E "^FAILED|Error" gpurun_out/r03_gpu_tests_$TAG.log | head -20; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_smoke_$TAG.log 2>&1 || { tail gpurun_out/r03_smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/r03_smoke_$TAG.log
fi
for wl in $WLS; do
  bash tools/pmc_bench.sh ${TAG}_$wl --workload $wl > gpurun_out/pmc_log_${TAG}_$wl.txt 2>&1 || { tail gpurun_out/pmc_log_${TAG}_$wl.txt; exit 1; }
  python tools/pmc_bench_summary.py gpurun_out/pmc_bench_${TAG}_$wl gpurun_out/r03_pmc_bench_$wl.json > /dev/null || exit 1
  cp gpurun_out/r03_pmc_bench_$wl.json profiles/r03_pmc_bench_$wl.json
  if [ "$wl" = "llama2-7b" ]; then EXTRA="--steps 20 --warmup 5"; else EXTRA="--steps 10 --warmup 3 --no-cpu-baseline"; fi
  timeout -k 10 600 python bench.py --workload $wl $EXTRA > gpurun_out/r03_bench_${TAG}_$wl.log 2>&1 || { tail gpurun_out/r03_bench_${TAG}_$wl.log; exit 1; }
  python tools/bsum.py gpurun_out/r03_bench_${TAG}_$wl.log 2>/dev/null | head -3
  rm -rf /tmp/rp_$wl
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rp_$wl -o run -- python3 bench.py --workload $wl \
      --steps 10 --warmup 3 --init random --no-cpu-baseline --no-ref-torch --no-other-exchange > gpurun_out/r03_rp_${TAG}_$wl.log 2>&1 || exit 1
  f=$(find /tmp/rp_$wl -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/r03_rocprof_stats_${TAG}_$wl.csv
done
