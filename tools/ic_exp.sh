#!/bin/bash
# Infinity-Cache residency experiment for the K2 sweep: phase C re-reads S1; with small probe
# groups the S1 + S2 bytes streamed between phases A and C fit the 256 MiB Infinity Cache.
set -u
mkdir -p gpurun_out
for g in "$@"; do
  HDP_PROBE_GROUP=$g timeout -k 10 240 python bench.py --layers 8 --steps 5 --warmup 2 --no-cpu-baseline \
      --no-ref-torch --emulate-wn 1 > gpurun_out/ic_g$g.json 2> gpurun_out/ic_g$g.err || exit $?
  echo "group $g done"
done
