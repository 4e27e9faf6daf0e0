#!/bin/bash
# SQ counter passes over the wide x3 K4 plan at Wn = 8 (tools/delta_bench.py, 4 LLaMA-2-7B
# layers): the real kernel and the measurement-only variant without W traffic (HDP_K4_DBG_NOW).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_x3w
mkdir -p $OUT
for var in base now; do
  i=0
  for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS" \
             "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    rm -rf /tmp/pmcx_$var$i
    if [ $var = now ]; then export HDP_K4_DBG_NOW=1; else unset HDP_K4_DBG_NOW; fi
    timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmcx_$var$i -o run -- python3 tools/delta_bench.py --layers 4 --wn 8 --pol 3 --reps 1 > $OUT/${var}_pass$i.log 2>&1 || exit $?
    find /tmp/pmcx_$var$i -name "*counter_collection.csv" -exec cp {} $OUT/${var}_pass$i.csv \;
  done
done
