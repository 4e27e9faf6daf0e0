#!/bin/bash
# L2 / fetch counters of the probe phases (tools/probe_phase.py at a workload's shapes): where phase C's
# bytes come from.  usage: bash tools/pmc_probe_c.sh TAG [probe_phase args]
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_probe_$TAG
mkdir -p $OUT
i=0
for set in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum TCC_READ_sum TCC_EA0_RDREQ_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum SQ_INSTS_VMEM_RD SQ_WAVES"; do
  i=$((i+1))
  rm -rf /tmp/pmcp_$i
  timeout -s KILL 200 rocprofv3 --pmc $set --kernel-include-regex "probe" --output-format csv -d /tmp/pmcp_$i -o run -- \
      python3 tools/probe_phase.py --reps 2 "$@" > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmcp_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
  echo "pass $i done"
done
