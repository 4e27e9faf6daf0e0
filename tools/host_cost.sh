set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 200 python tools/host_probe_cost.py > gpurun_out/hostcost.log 2>&1; grep -v amdgpu.ids gpurun_out/hostcost.log | head -24
timeout -k 10 300 python bench.py --init random --no-cpu-baseline --no-ref-torch --emulate-wn 1 --no-other-exchange > gpurun_out/b.log 2>&1 || exit 1
python -c "
import json; d=json.loads([l for l in open('gpurun_out/b.log') if l.startswith('{')][-1]); print({k:d[k] for k in ('value','ms_per_step','host_ms_per_step','dw_ms_per_step')})"
