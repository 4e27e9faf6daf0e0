#!/bin/bash
# bf16 single-segment K4 merges on the wide x3 kernel: delta / layer / config parity, then Mistral-7B
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_layer.py tests/test_gpu_configs.py tests/test_trajectory.py -m gpu -x -q --timeout 300 --timeout-method thread -k "delta or step or layer or config or trajectory or merge or residual" > gpurun_out/t_k4b.log 2>&1 || { tail -40 gpurun_out/t_k4b.log; exit 1; }
tail -1 gpurun_out/t_k4b.log
for w in mistral-7b llama2-13b; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange --init random > gpurun_out/bk_$w.log 2>&1 || exit 1
  python - $w <<'PY'
import json,sys
d=json.loads([l for l in open(f'gpurun_out/bk_{sys.argv[1]}.log') if l.startswith('{')][-1])
print(sys.argv[1], d['value'], d['ms_per_step'], 'dw', d['dw_ms_per_step'], d['roofline']['component_ms_per_step'])
PY
done
