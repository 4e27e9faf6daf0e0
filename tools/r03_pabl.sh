#!/bin/bash
# K2 ablation timing (tools/probe_ablate.py builds): the bench's probe phases with the product library, then
# with each variant swapped in for libhdpissa.so in this (scratch) copy of the tree
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
B="--steps 10 --warmup 3 --no-cpu-baseline --no-ref-torch --no-other-exchange"
timeout -k 10 300 python bench.py $B > gpurun_out/pabl_base.log 2>&1 || { tail gpurun_out/pabl_base.log; exit 1; }
python tools/bsum.py gpurun_out/pabl_base.log | head -3
for v in ${VARIANTS:-halfmfma}; do
  cp tools/abl/libhdpissa_$v.so hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so
  timeout -k 10 300 python bench.py $B > gpurun_out/pabl_$v.log 2>&1 || { tail gpurun_out/pabl_$v.log; exit 1; }
  python tools/bsum.py gpurun_out/pabl_$v.log | head -3
done
