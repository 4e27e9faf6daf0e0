#!/bin/bash
mkdir -p gpurun_out
for cols in 128 256 512; do for u in 1 2 3; do
  HDP_P1_COLS=$cols HDP_P1_U=$u timeout -k 10 120 python tools/probe_sweep.py >> gpurun_out/sweep.log 2>&1 || exit $?
done; done
