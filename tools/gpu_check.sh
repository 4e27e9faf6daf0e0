#!/bin/bash
# GPU-box check script: each GPU step under its own time limit; stop at the first step that
# faults, aborts or times out (exit 124/134/137/139 or >128).  Plain test failures (pytest rc 1)
# do not stop the script.  Usage: bash tools/gpu_check.sh [tests] [smoke] [ktime] [bench ARGS...]
set -u
mkdir -p gpurun_out
run_step() {  # name limit cmd...
  local name=$1 limit=$2; shift 2
  timeout -k 10 "$limit" "$@" >> "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc" | tee -a gpurun_out/steps.txt
  if [ $rc -ge 124 ] || [ $rc -gt 1 -a $rc -ne 0 -a "$name" != "tests" ]; then
    echo "stopping after $name (rc=$rc)" | tee -a gpurun_out/steps.txt
    exit $rc
  fi
  if [ "$name" = "tests" ] && [ $rc -gt 1 ]; then
    echo "stopping after tests (rc=$rc)" | tee -a gpurun_out/steps.txt
    exit $rc
  fi
  return 0
}
: > gpurun_out/steps.txt; rm -f gpurun_out/*.log
for step in "$@"; do
  case $step in
    tests) run_step tests 600 python -m pytest tests -m gpu -q -x ;;
    kern) HDP_SYNC_DEBUG=1 run_step tests 400 python -m pytest tests/test_gpu_kernels.py -m gpu -q -x -k "not svd" ;;
    svd) HDP_SYNC_DEBUG=1 run_step tests 300 python -m pytest tests/test_gpu_kernels.py -m gpu -q -k svd ;;
    layer) run_step tests 300 python -m pytest tests/test_gpu_layer.py -m gpu -q ;;
    comm) run_step tests 300 python -m pytest tests/test_gpu_comm.py -m gpu -q ;;
    alltests) run_step tests 900 python -m pytest tests -m gpu -q ;;
    cfg) run_step tests 600 python -m pytest tests/test_gpu_configs.py -m gpu -q -x ;;
    smoke) run_step smoke 180 python __graft_entry__.py smoke ;;
    bench8) run_step bench8 300 python bench.py --layers 8 --steps 5 --warmup 2 --no-cpu-baseline --no-ref-torch --emulate-wn 1 ;;
    ktime) run_step ktime 400 python tools/kernel_timing.py ;;
    ktimeq) run_step ktime 300 python tools/kernel_timing.py --quick ;;
    bench) run_step bench 900 python bench.py ;;
  esac
done
