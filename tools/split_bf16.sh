#!/bin/bash
# split path (r > 32) with bf16 activations: parity tests, then the r64 / r128 workloads
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "probe" > gpurun_out/t_split.log 2>&1 || { tail -40 gpurun_out/t_split.log; exit 1; }
tail -1 gpurun_out/t_split.log
for w in mistral-7b llama2-13b; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange --init random > gpurun_out/bs_$w.log 2>&1 || exit 1
  python - $w <<'PY'
import json,sys
w=sys.argv[1]
d=json.loads([l for l in open(f'gpurun_out/bs_{w}.log') if l.startswith('{')][-1])
r=d['roofline']
print(w, d['value'], d['ms_per_step'], r['component_ms_per_step'], {k: (v['per_launch']['avg_us'], v['achieved'], v['unit']) for k, v in r['others'].items()})
PY
done
