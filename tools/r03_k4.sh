#!/bin/bash
# round-3 K4 experiments: bf16 single-segment merges (Mistral r64, LLaMA-2-13B r128) under rocprofv3 stats,
# MERGE vs STORE (loads of W vs none), so the pack / scale passes and the main kernel are timed apart
set -u
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-a}
i=0
for cfg in "--shapes mistral-7b --r 64 --dtype bf16 --layers 8" \
           "--shapes llama2-13b --r 128 --dtype bf16 --layers 8" "--shapes llama2-7b --r 16 --dtype f32 --layers 8 --wn 8"; do
  i=$((i+1))
  rm -rf /tmp/k4p_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k4p_$i -o run -- python3 tools/delta_bench.py --wn 1 $cfg --reps 5 \
      > gpurun_out/k4_${TAG}_$i.log 2>&1 || { tail gpurun_out/k4_${TAG}_$i.log; exit 1; }
  grep '^{' gpurun_out/k4_${TAG}_$i.log
  f=$(find /tmp/k4p_$i -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/k4_${TAG}_${i}_stats.csv
  python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'hdp' in r['Name'] or 'delta' in r['Name'] or 'k4_' in r['Name']:
        print(f"  {r['Name'][:90]:90s} calls {r['Calls']:>5s} avg_us {float(r['AverageNs'])/1e3:10.1f}")
PY
done
if [ -x tools/bin/lds_stream ]; then timeout -k 10 120 tools/bin/lds_stream > gpurun_out/lds_stream_$TAG.log 2>&1; cat gpurun_out/lds_stream_$TAG.log; fi
