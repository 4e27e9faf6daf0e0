#!/bin/bash
# K4 float32 (LLaMA-2-7B shapes, Wn=1) ablation timings: base library vs tools/abl variants
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base f16b}; do
  if [ $v = base ]; then L=hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so; else L=tools/abl/libhdpissa_$v.so; fi
  HDPISSA_LIB=$L timeout -k 10 120 python tools/delta_bench.py --shapes llama2-7b --r 16 --dtype f32 --layers 8 --wn 1 --reps 7 > gpurun_out/abl32_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abl32_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/abl32_$v.log)"
done
