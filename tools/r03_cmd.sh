set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "probe or config or layer or plumbing" > gpurun_out/t5.log 2>&1; rc=$?; tail -2 gpurun_out/t5.log; [ $rc -ne 0 ] && { grep -E "^FAILED|Error|assert" gpurun_out/t5.log | head; exit 1; }
for wl in mistral-7b llama2-13b; do
  timeout -k 10 400 python bench.py --workload $wl --steps 10 --warmup 3 --init random --no-cpu-baseline --no-ref-torch --no-other-exchange > gpurun_out/r03_b_s5_$wl.log 2>&1 || { tail gpurun_out/r03_b_s5_$wl.log; exit 1; }
  python tools/bsum.py gpurun_out/r03_b_s5_$wl.log | head -4
done
