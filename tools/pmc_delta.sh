#!/bin/bash
# SQ counter passes over K4 at Wn = 8 (tools/delta_bench.py, one LLaMA-2-7B layer, both maths,
# one launch per module): cycle split, instruction mix, MFMA busy, LDS conflicts.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmc_delta${TAG:-}
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  rm -rf /tmp/pmcd_$i
  timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmcd_$i -o run -- python3 tools/delta_bench.py --layers 1 --wn 8 --math ${MATHS:-f32 x3} ${SINGLE:-} --reps 1 > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmcd_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
done
