set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "h2_bf16 or dma" > gpurun_out/t2.log 2>&1; tail -2 gpurun_out/t2.log
for d in 0 3; do HDP_K4_DEFER=$d timeout -k 10 120 python tools/delta_bench.py --shapes mistral-7b --r 64 --dtype bf16 --layers 8 --wn 1 --reps 5 | tail -1; done
HDP_K4_DEFER=3 bash tools/r03_pmc_sq.sh k4d3 --workload mistral-7b > gpurun_out/pmc_k4d3.txt 2>&1 || exit 1
HDP_K4_DEFER=0 bash tools/r03_pmc_sq.sh k4d0 --workload mistral-7b > gpurun_out/pmc_k4d0.txt 2>&1 || exit 1
HDP_PROBE_DMA=1 bash tools/r03_pmc_sq.sh dma1 > gpurun_out/pmc_dma1.txt 2>&1 || exit 1
HDP_PROBE_DMA=0 bash tools/r03_pmc_sq.sh dma0 > gpurun_out/pmc_dma0.txt 2>&1 || exit 1
