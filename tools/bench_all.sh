#!/bin/bash
# every BASELINE workload's bench line on one box (each run under its own limit; stop at the first fault)
# usage: bash tools/bench_all.sh TAG [workload ...]
set -u
TAG=$1; shift
mkdir -p gpurun_out
for w in "$@"; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --warmup 3 > gpurun_out/bench_${TAG}_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc"
  [ $rc -ne 0 ] && exit $rc
  grep '^{' gpurun_out/bench_${TAG}_$w.log > gpurun_out/bench_${TAG}_$w.jsonl
done
exit 0
