#!/bin/bash
# K4 at Wn = 8 with parts of the H2 kernel removed (HDP_H2_ABL measurement builds from
# tools/k4abl_build.sh, loaded through HDPISSA_LIB; results wrong by construction, timing only).
# usage: bash tools/k4_wn8_abl.sh [variant ...]   (variant "0" = the library build)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/k4_wn8_abl.jsonl
: > $out
for v in "$@"; do
  if [ "$v" = "0" ]; then lib=hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so; else lib=scratch/abl/libhdpissa_h2abl$v.so; fi
  for cfg in "--shapes llama2-7b --dtype f32 --r 16 --layers 8" \
             "--shapes mistral-7b --dtype bf16 --round --r 64 --layers 8" \
             "--shapes llama2-13b --dtype bf16 --round --r 128 --layers 2"; do
    echo "abl=$v $cfg" | tee -a $out
    HDPISSA_LIB=$lib timeout -k 10 120 python tools/delta_bench.py --wn 8 --reps 5 $cfg >> $out 2>&1 || exit $?
  done
done
cat $out
