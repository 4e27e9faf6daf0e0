#!/bin/bash
# rocprofv3 PMC passes over THE BENCH COMMAND (python bench.py, default llama2-7b workload unless
# overridden by extra args, e.g. --workload mistral-7b; --init random so the thousands of rocSOLVER
# init launches stay out, and --kernel-include-regex hdp:: so only the library's kernels count):
#   pass 1 FETCH_SIZE, pass 2 WRITE_SIZE (separate passes on gfx950), pass 3 MFMA busy cycles.
# usage: tools/pmc_bench.sh OUT_TAG [bench args...]   (output gpurun_out/pmc_bench_OUT_TAG)
# Summary: python tools/pmc_bench_summary.py gpurun_out/pmc_bench_<tag> profiles/r04_pmc_bench_<workload>.json
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
OUT=gpurun_out/pmc_bench_$TAG
mkdir -p $OUT
echo "$@" > $OUT/args.txt
i=0
for set in "FETCH_SIZE" "WRITE_SIZE" "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/pmcb_$i
  timeout -s KILL 400 rocprofv3 --pmc $set --kernel-include-regex "hdp::" --output-format csv -d /tmp/pmcb_$i -o run -- \
      python3 bench.py --steps 2 --warmup 1 --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 \
      --no-other-exchange --timing-out $OUT/timing.json "$@" > $OUT/pass$i.log 2>&1 || exit $?
  find /tmp/pmcb_$i -name "*counter_collection.csv" -exec cp {} $OUT/pass$i.csv \;
  echo "pass $i done ($TAG)"
done
