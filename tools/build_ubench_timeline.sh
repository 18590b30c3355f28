#!/bin/bash
# builds tools/ubench_timeline: the GP bench step against a library whose
# cholesky.hip is compiled with SMG_PANEL_TIMELINE (tools/tl/libsmg_hip.so)
set -e
cd "$(dirname "$0")/.."
mkdir -p tools/tl
OBJS=$(ls math_amd/lib/obj/*.o | grep -v "/cholesky.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -w -mllvm -pragma-unroll-threshold=500000 \
  -mllvm -amdgpu-mfma-vgpr-form -Iinclude -DSMG_PANEL_TIMELINE -c -o /tmp/cholesky_tl.o math_amd/csrc/cholesky.hip
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS /tmp/cholesky_tl.o -o tools/tl/libsmg_hip.so \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
g++ -std=c++17 -O2 -DSTAN_MATH_AMD_TLS_INITIAL_EXEC -Imath_amd/include -Iinclude -isystem /root/reference/lib/eigen_3.3.3 \
  tools/ubench_timeline.cpp -o tools/ubench_timeline -Ltools/tl -lsmg_hip -Wl,-rpath,'$ORIGIN/tl'
