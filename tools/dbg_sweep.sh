set -u
for d in 0 1 2 3; do HDP_SW_DBG=$d HDP_PROBE_BUDGET_MB=768 timeout -k 10 120 python tools/probe_sweep.py >> gpurun_out/dbg.log 2>&1 || exit $?; done
timeout -k 10 120 ./tools/bin/stream_bw > gpurun_out/stream_bw.log 2>&1
