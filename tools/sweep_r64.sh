#!/bin/bash
# r = 64 on the sweep path: parity, then Mistral-7B (bf16, r 64) sweep vs split
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_configs.py -x -q --timeout 300 --timeout-method thread -k "probe" > gpurun_out/t_r64.log 2>&1 || { tail -40 gpurun_out/t_r64.log; exit 1; }
tail -1 gpurun_out/t_r64.log
for path in sweep; do
  if [ $path = sweep ]; then unset HDP_PROBE_PATH; else export HDP_PROBE_PATH=split; fi
  timeout -k 10 600 python bench.py --workload mistral-7b --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange --init random > gpurun_out/b64_$path.log 2>&1 || exit 1
  python - $path <<'PY'
import json,sys
d=json.loads([l for l in open(f'gpurun_out/b64_{sys.argv[1]}.log') if l.startswith('{')][-1])
r=d['roofline']
print(sys.argv[1], d['value'], d['ms_per_step'], r['component_ms_per_step'], r.get('per_launch',{}).get('phases_us'))
PY
done
