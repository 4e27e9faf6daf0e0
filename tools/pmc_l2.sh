#!/bin/bash
# L2 hit/miss of K4 at Wn = 8 (x3 plan): one PMC pass over tools/delta_bench.py (one layer).
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/pmc_l2
rm -rf /tmp/pmcl2
timeout -k 10 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum --kernel-trace --output-format csv -d /tmp/pmcl2 -o run -- python3 tools/delta_bench.py --layers ${LAYERS:-2} --wn 8 --math x3 --reps 1 > gpurun_out/pmc_l2/pass.log 2>&1 || exit $?
find /tmp/pmcl2 -name "*counter_collection.csv" -exec cp {} gpurun_out/pmc_l2/pass.csv \;
