#!/bin/bash
# L2 / fabric counters of K4 at Wn = 8 (x3 plan): one PMC pass per (counter set, x3 stage) over
# tools/delta_bench.py (LAYERS layers, default 2).  Output: gpurun_out/pmc_l2/<stage>_<i>.csv
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_l2
for stage in ${STAGES:-g w}; do
  i=0
  for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum" "WRITE_SIZE"; do
    i=$((i+1))
    rm -rf /tmp/pmcl2
    HDP_K4_X3_STAGE=$stage timeout -k 10 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d /tmp/pmcl2 -o run -- python3 tools/delta_bench.py --layers ${LAYERS:-2} --wn 8 --math x3 --pol 3 --reps 1 > gpurun_out/pmc_l2/${stage}_$i.log 2>&1 || exit $?
    find /tmp/pmcl2 -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_l2/${stage}_$i.csv \;
  done
done
