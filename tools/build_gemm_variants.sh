#!/bin/bash
# dev: tools/gv_<name>/{libsmg_hip.so,ubench_gemm} with gemm.hip built under
# extra defines; usage: build_gemm_variants.sh name "-DX=1 -DY=2" ...
set -e
cd "$(dirname "$0")/.."
OBJS=$(ls math_amd/lib/obj/*.o | grep -v "/gemm.o")
while [ $# -ge 2 ]; do
  name=$1; defs=$2; shift 2
  mkdir -p tools/gv_$name
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -mllvm -pragma-unroll-threshold=500000 \
    -mllvm -amdgpu-mfma-vgpr-form -Iinclude $defs -c -o /tmp/gemm_$name.o math_amd/csrc/gemm.hip
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS /tmp/gemm_$name.o -o tools/gv_$name/libsmg_hip.so \
    -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
  /opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 -Iinclude tools/ubench_gemm.cpp -o tools/gv_$name/ubench_gemm \
    -Ltools/gv_$name -lsmg_hip -Wl,-rpath,'$ORIGIN'
done
