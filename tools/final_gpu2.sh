#!/bin/bash
# Round-2 evidence: GPU tests, default bench, bench under rocprofv3 --kernel-trace --stats, and bench
# lines of the other BASELINE workloads (each step time-limited; stops at the first failure)
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
: > gpurun_out/final_steps.txt
step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/final_steps.txt
  [ $rc -ne 0 ] && exit $rc
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    prof) rm -rf /tmp/prof_bench; step prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_bench -o run -- python3 bench.py --no-ref-torch --no-cpu-baseline
          find /tmp/prof_bench -name "*kernel_stats.csv" -exec cp {} gpurun_out/prof_kernel_stats.csv \; ;;
    wl) for w in qwen2.5-0.5b mistral-7b llama2-13b qproj; do step "bench_$w" 600 python bench.py --workload $w --no-cpu-baseline --emulate-wn 1; done ;;
  esac
done
