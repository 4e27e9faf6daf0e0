#!/bin/bash
# round-end evidence, part A: the GPU suite, smoke, every workload's bench line
set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/final_tests.log 2>&1
rc=$?; tail -n 2 gpurun_out/final_tests.log; [ $rc -ge 2 ] && exit $rc
timeout -k 10 240 python __graft_entry__.py smoke > gpurun_out/final_smoke.log 2>&1 || exit $?
tail -n 2 gpurun_out/final_smoke.log
bash tools/bench_all.sh final llama2-7b qwen2.5-0.5b mistral-7b llama2-13b qproj
