#!/bin/bash
# Round-end evidence on one GPU box: full GPU tests, the default bench, the bench under
# rocprofv3 --kernel-trace --stats, and the bench-command PMC passes.  Each step has its own
# time limit; the script stops at the first fault / timeout.
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/final_steps.txt
  if [ $rc -ne 0 ] && [ "$name" != "tests" ]; then exit $rc; fi
  if [ $rc -ge 124 ]; then exit $rc; fi
  return 0
}
: > gpurun_out/final_steps.txt
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    bench) step bench 600 python bench.py ;;
    prof) rm -rf /tmp/prof_bench; step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o run -- python3 bench.py --no-ref-torch --no-cpu-baseline
          find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_kernel_stats.csv \; ;;
    pmc) step pmc 1200 bash tools/pmc_bench.sh && python tools/pmc_bench_summary.py gpurun_out/pmc_bench gpurun_out/pmc_bench/summary.json > /dev/null ;;
  esac
done
