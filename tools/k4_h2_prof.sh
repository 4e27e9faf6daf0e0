# per-kernel time of the K4 Wn=8 plan run: H2 vs bf16x3 (rocprofv3 kernel stats)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in auto x3; do
  rm -rf /tmp/k4p_$m
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/k4p_$m -o run -- python3 tools/delta_bench.py --layers 32 --wn 8 --pol 3 --reps 3 --math $m > gpurun_out/k4p_$m.log 2>&1 || exit 1
  f=$(find /tmp/k4p_$m -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/k4p_${m}_stats.csv
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(r["Name"][:90], r["Calls"], round(float(r["AverageNs"]) / 1e6, 3), "ms avg")
PY
  grep plan gpurun_out/k4p_$m.log
done
