#!/bin/bash
# round-end PMC passes of every workload's bench command (tools/pmc_bench.sh), both exchange legs where measured
set -u
for w in llama2-7b mistral-7b llama2-13b qproj qwen2.5-0.5b; do
  bash tools/pmc_bench.sh $w --workload $w || exit $?
done
bash tools/pmc_bench.sh llama2-7b_allreduce --workload llama2-7b --exchange allreduce || exit $?
bash tools/pmc_bench.sh mistral-7b_allreduce --workload mistral-7b --exchange allreduce || exit $?
