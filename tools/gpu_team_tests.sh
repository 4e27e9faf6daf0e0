set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 120 --timeout-method thread -k "team" > gpurun_out/t_team.log 2>&1
rc=$?; echo "team rc=$rc"; tail -5 gpurun_out/t_team.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -k "probe" > gpurun_out/t_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -5 gpurun_out/t_probe.log
exit $rc
