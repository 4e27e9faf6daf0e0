#!/bin/bash
# single-segment stripes write their gradient directly: parity, then llama2-7b and mistral-7b
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py tests/test_gpu_layer.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_fold.log 2>&1 || { tail -40 gpurun_out/t_fold.log; exit 1; }
tail -1 gpurun_out/t_fold.log
for w in llama2-7b mistral-7b; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange --init random > gpurun_out/bf_$w.log 2>&1 || exit 1
  python - $w <<'PY'
import json,sys
d=json.loads([l for l in open(f'gpurun_out/bf_{sys.argv[1]}.log') if l.startswith('{')][-1])
r=d['roofline']
print(sys.argv[1], d['value'], d['ms_per_step'], 'host', d['host_ms_per_step'], r['component_ms_per_step'], r.get('per_launch',{}).get('phases_us'))
PY
done
