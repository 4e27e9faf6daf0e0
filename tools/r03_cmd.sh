set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python tools/delta_bench.py --shapes mistral-7b --r 64 --dtype bf16 --layers 8 --wn 1 --reps 5 --math x3 | tail -1
timeout -k 10 120 python tools/delta_bench.py --shapes llama2-13b --r 128 --dtype bf16 --layers 8 --wn 1 --reps 5 --math x3 | tail -1
rm -rf /tmp/k4x
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k4x -o run -- python3 tools/delta_bench.py --shapes mistral-7b --r 64 --dtype bf16 --layers 8 --wn 1 --reps 5 --math x3 > /dev/null 2>&1
f=$(find /tmp/k4x -name "*kernel_stats.csv" | head -1); python3 - "$f" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'delta' in r['Name'] or 'k4_' in r['Name']:
        print(f"  {r['Name'][:80]:80s} calls {r['Calls']:>4s} avg_us {float(r['AverageNs'])/1e3:9.1f}")
PY
