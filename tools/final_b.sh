#!/bin/bash
# round-end evidence, part B: rocprofv3 kernel stats of the headline bench command (both exchanges) and the
# bench-command PMC passes of every workload (tools/pmc_bench.sh)
set -u
bash tools/prof_bench.sh final7b --steps 10 --warmup 3 || exit $?
bash tools/prof_bench.sh final7b_ar --steps 10 --warmup 3 --exchange allreduce || exit $?
for w in llama2-7b mistral-7b llama2-13b qproj qwen2.5-0.5b; do
  bash tools/pmc_bench.sh $w --workload $w || exit $?
done
bash tools/pmc_bench.sh llama2-7b_allreduce --workload llama2-7b --exchange allreduce || exit $?
bash tools/pmc_bench.sh mistral-7b_allreduce --workload mistral-7b --exchange allreduce || exit $?
