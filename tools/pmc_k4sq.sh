#!/bin/bash
# SQ / TCC counter passes over one K4 plan configuration (tools/delta_bench.py args), e.g.
#   bash tools/pmc_k4sq.sh TAG --shapes mistral-7b --dtype bf16 --round --r 64 --layers 8 --wn 8
# summary: python tools/pmc_sq_summary.py gpurun_out/pmc_k4sq_TAG
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_k4sq_$TAG
mkdir -p $OUT
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM" \
           "SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_WAVES GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  rm -rf /tmp/pmck4_$i
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmck4_$i -o run -- \
      python3 tools/delta_bench.py --reps 2 "$@" > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmck4_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
  echo "pass $i done"
done
