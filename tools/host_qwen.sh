#!/bin/bash
# host-path changes: layer / trajectory / step GPU tests, then the host-bound Qwen2.5-0.5B bench and LLaMA-2-7B
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_layer.py tests/test_trajectory.py tests/test_gpu_comm.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t_host.log 2>&1 || { tail -40 gpurun_out/t_host.log; exit 1; }
tail -1 gpurun_out/t_host.log
for w in qwen2.5-0.5b llama2-7b; do
  timeout -k 10 600 python bench.py --workload $w --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange > gpurun_out/bh_$w.log 2>&1 || exit 1
  python - $w <<'PY'
import json,sys
d=json.loads([l for l in open(f'gpurun_out/bh_{sys.argv[1]}.log') if l.startswith('{')][-1])
print(sys.argv[1], d['value'], d['ms_per_step'], 'host', d['host_ms_per_step'], d['roofline']['component_ms_per_step'])
PY
done
