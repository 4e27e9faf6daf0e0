#!/bin/bash
# HBM traffic of the H2 K4 plan at Wn = 8 (tools/delta_bench.py, 4 LLaMA-2-7B layers): FETCH_SIZE
# and WRITE_SIZE in separate passes, plus MFMA busy
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_h2
mkdir -p $OUT
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_MFMA GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/pmch_$i
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmch_$i -o run -- python3 tools/delta_bench.py --layers 4 --wn 8 --pol 3 --reps 1 > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmch_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
done
