set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "merge or adam or probe_grads or large_group" > gpurun_out/t4.log 2>&1; rc=$?; tail -2 gpurun_out/t4.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/t4.log | head; exit 1; }
for wl in mistral-7b llama2-7b; do for nt in 0 1; do
  HDP_PROBE_NTZ=$nt timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --init random --no-cpu-baseline --no-ref-torch > gpurun_out/r03_b_nt${nt}_$wl.log 2>&1 || { tail gpurun_out/r03_b_nt${nt}_$wl.log; exit 1; }
  echo "NTZ=$nt"; python tools/bsum.py gpurun_out/r03_b_nt${nt}_$wl.log | head -3
  python - gpurun_out/r03_b_nt${nt}_$wl.log <<'PY'
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
lg=d.get('exchange_legs',{}).get('allreduce',{})
print('  allreduce leg dw ms', lg.get('dw_ms_per_step'), 'merge', (lg.get('merge') or {}).get('frac'), 'k5 alone', (lg.get('k5_merge_alone') or {}).get('frac'))
PY
done; done
HDP_PROBE_NTZ=1 bash tools/pmc_bench.sh nt1_mistral --workload mistral-7b > /dev/null 2>&1 && python tools/pmc_bench_summary.py gpurun_out/pmc_bench_nt1_mistral gpurun_out/pmc_nt1_mistral.json | head -30
