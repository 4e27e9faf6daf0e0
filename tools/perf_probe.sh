#!/bin/bash
# Probe path comparison at LLaMA-2-7B shapes: sweep path at several group budgets vs the split
# path.  Appends to gpurun_out/ps.log; stops at the first failing step.
set -u
mkdir -p gpurun_out
for b in ${BUDGETS:-160 384 768 1536}; do
  HDP_PROBE_BUDGET_MB=$b timeout -k 10 120 python tools/probe_sweep.py >> gpurun_out/ps.log 2>&1 || exit $?
done
HDP_PROBE_PATH=split HDP_PROBE_BUDGET_MB=160 timeout -k 10 120 python tools/probe_sweep.py >> gpurun_out/ps.log 2>&1 || exit $?
