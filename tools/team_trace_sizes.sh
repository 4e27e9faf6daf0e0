set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
HDP_TM_L=12 timeout -k 10 200 python tools/team_trace.py 4096 8 > gpurun_out/trace4096.log 2>&1; cat gpurun_out/trace4096.log | grep -v amdgpu.ids
HDP_TM_L=12 timeout -k 10 200 python tools/team_trace.py 672 32 > gpurun_out/trace672.log 2>&1; cat gpurun_out/trace672.log | grep -v amdgpu.ids
