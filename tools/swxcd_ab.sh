#!/bin/bash
# A/B of the probe sweep's workgroup order: probe tests on the default build, then probe_phase timings
# alternating the default (XCD-contiguous) and the blockIdx-order build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_probe_layers.py \
  tests/test_gpu_kernels.py -k "probe" > gpurun_out/swxcd_tests.log 2>&1 || { tail -30 gpurun_out/swxcd_tests.log; exit 1; }
tail -n 1 gpurun_out/swxcd_tests.log
out=gpurun_out/swxcd_ab.jsonl; : > $out
for rep in 1 2; do
  for lib in default scratch/abl/libhdpissa_swxcd0.so; do
    for cfg in "--workload llama2-7b --layers 8" "--workload mistral-7b --layers 8" "--workload llama2-13b --layers 4"; do
      if [ $lib = default ]; then L=hd-pissa_amd/hdpissa_amd/_lib/libhdpissa.so; else L=$lib; fi
      echo "lib=$lib $cfg" >> $out
      HDPISSA_LIB=$L timeout -k 10 120 python tools/probe_phase.py $cfg 2>/dev/null | grep '^{' >> $out || exit 1
    done
  done
done
cat $out
