#!/bin/bash
set -e
cd "$(dirname "$0")/../hd-pissa_amd"
mkdir -p ../scratch/abl
F="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -mcode-object-version=5 -I../include -I/opt/rocm/include -munsafe-fp-atomics"
for b in $@; do
  /opt/rocm/bin/hipcc $F -DHDP_H2_ABL=$b -c csrc/hdp_delta.hip -o ../scratch/abl/hdp_delta_h2abl$b.o &
done
wait
for b in $@; do
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lrocsolver -lrocblas ../scratch/abl/hdp_delta_h2abl$b.o build/hdp_probe.o build/hdp_elementwise.o build/hdp_svd.o build/hdp_api.o build/hdp_comm.o -o ../scratch/abl/libhdpissa_h2abl$b.so
done
ls -la ../scratch/abl/
