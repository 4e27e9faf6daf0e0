#!/bin/bash
# K4 bf16 ablation timings (tools/k4_ablate.py builds): base library vs variants
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in ${VARIANTS:-base nomfma nodma now}; do
  if [ $v = base ]; then L=hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so; else L=tools/abl/libhdpissa_$v.so; fi
  for s in "mistral-7b 64" "llama2-13b 128"; do
    set -- $s
    HDPISSA_LIB=$L timeout -k 10 120 python tools/delta_bench.py --shapes $1 --r $2 --dtype bf16 --layers 8 --wn 1 --reps 5 --math h2 > gpurun_out/abl_${v}_$1.log 2>&1 || { echo "$v $1 failed"; tail -3 gpurun_out/abl_${v}_$1.log; exit 1; }
    echo "$v $1: $(tail -1 gpurun_out/abl_${v}_$1.log)"
  done
done
