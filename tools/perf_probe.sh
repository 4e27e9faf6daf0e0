#!/bin/bash
# Probe path comparison at LLaMA-2-7B shapes (PROBE_T rows): sweep and split paths at several
# group budgets.  Appends to gpurun_out/ps.log; stops at the first failing step.
set -u
mkdir -p gpurun_out
for path in ${PATHS:-sweep split}; do
  for b in ${BUDGETS:-96 160 256 768}; do
    HDP_PROBE_PATH=$path HDP_PROBE_BUDGET_MB=$b timeout -k 10 120 python tools/probe_sweep.py >> gpurun_out/ps.log 2>&1 || exit $?
  done
done
