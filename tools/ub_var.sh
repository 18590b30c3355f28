#!/bin/bash
# ubench_gemm against variant builds of libsmg_hip.so (var/<name>/, dev only)
set -o pipefail
for v in base ${VARS}; do
  for t in ${TILES:-0}; do
    echo "== $v tile $t"
    if [ $v = base ]; then SMG_GEMM_TILE=$t timeout -k 10 120 tools/ubench_gemm || exit 1
    else LD_LIBRARY_PATH=$GRAFT_REPO_ROOT/var/$v SMG_GEMM_TILE=$t timeout -k 10 120 tools/ubench_gemm || exit 1; fi
  done
done
