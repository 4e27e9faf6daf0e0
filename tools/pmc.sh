#!/bin/bash
# two PMC passes (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950) over the hot-path kernels
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc
for c in FETCH_SIZE WRITE_SIZE; do
  rm -rf /tmp/pmc_$c
  HOTPATH_TIMING_OUT=gpurun_out/pmc/hotpath_timing.json timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d /tmp/pmc_$c -o run -- python3 tools/hotpath_kernels.py > gpurun_out/pmc/$c.log 2>&1 || exit $?
  find /tmp/pmc_$c -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc/$c.csv \;
  find /tmp/pmc_$c -name "*kernel_trace.csv" -exec cp {} gpurun_out/pmc/${c}_trace.csv \;
done
