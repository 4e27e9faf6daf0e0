#!/bin/bash
# rocprofv3 kernel-trace + stats of bench.py; keeps only the summary CSVs (gpurun_out <= 64 MiB)
# usage: bash tools/prof_bench.sh NAME [bench args...]
set -u
name=$1; shift
cd /tmp && export TMPDIR=/tmp
out=/tmp/prof_$name
rm -rf "$out"
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$out" -o run --output-format csv -- python3 bench.py "$@" \
  > "gpurun_out/prof_${name}_bench.log" 2>&1
rc=$?
mkdir -p "gpurun_out/prof_$name"
find "$out" -name "*stats*.csv" -exec cp {} "gpurun_out/prof_$name/" \;
exit $rc
