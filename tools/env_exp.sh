#!/bin/bash
# A/B one environment knob over the 8-layer bench (measurement tool):
#   bash tools/env_exp.sh VAR v1 v2 ...   -> gpurun_out/exp_VAR_v.json
set -u
mkdir -p gpurun_out
var=$1; shift
for v in "$@"; do
  env "$var=$v" timeout -k 10 240 python bench.py --layers 8 --steps 5 --warmup 2 --no-cpu-baseline --no-ref-torch \
      --emulate-wn 1 --no-other-exchange > gpurun_out/exp_${var}_$v.json 2> gpurun_out/exp_${var}_$v.err || exit $?
  echo "$var=$v done"
done
