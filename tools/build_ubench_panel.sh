#!/bin/bash
# builds tools/ubench_panel (includes cholesky.hip with SMG_PANEL_TRACE) with the library's flags
set -e
cd "$(dirname "$0")/.."
OBJS=$(ls math_amd/lib/obj/*.o | grep -v "/cholesky.o")
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -w -mllvm -pragma-unroll-threshold=500000 \
  -mllvm -amdgpu-mfma-vgpr-form -Iinclude $UB_FLAGS -c -o /tmp/ubench_panel.o tools/ubench_panel.hip
/opt/rocm/bin/hipcc --offload-arch=gfx950 -o ${UB_OUT:-tools/ubench_panel} /tmp/ubench_panel.o $OBJS \
  -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib
