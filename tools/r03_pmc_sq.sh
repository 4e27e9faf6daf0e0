#!/bin/bash
# SQ counter passes over the bench command (measurement tool): usage tools/r03_pmc_sq.sh TAG [bench args]
# env of the caller (HDP_* knobs) passes through; summary: python tools/pmc_sq_summary.py gpurun_out/pmc_sq_TAG
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_sq_$TAG
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_LDS" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/pmcsq_$i
  timeout -s KILL 300 rocprofv3 --pmc $set --kernel-include-regex "hdp::" --output-format csv -d /tmp/pmcsq_$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange "$@" \
      > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmcsq_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
  echo "pass $i done ($TAG)"
done
python3 tools/pmc_sq_summary.py $OUT
