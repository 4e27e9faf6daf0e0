#!/bin/bash
# SQ counter passes over the probe kernels (tools/probe_sweep.py at LLaMA-2-7B shapes):
# cycles split (active / wait / issue-stall), instruction mix, LDS and MFMA busy.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_sq
i=0
for set in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_INSTS_SMEM" \
           "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM"; do
  i=$((i+1))
  rm -rf /tmp/pmcsq_$i
  timeout -k 10 300 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmcsq_$i -o run -- python3 tools/probe_sweep.py > gpurun_out/pmc_sq/pass$i.log 2>&1 || exit $?
  find /tmp/pmcsq_$i -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_sq/pass$i.csv \;
done
