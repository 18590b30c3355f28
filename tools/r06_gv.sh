#!/bin/bash
# dev: ubench_gemm of each tools/gv_* variant over the HVP shapes, twice, interleaved
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${1:-gv}; shift
SH=${SH:-17 24 25 26 27 28 29 30 31}
for r in 1 2; do
for v in "$@"; do
  for s in $SH; do timeout -k 10 60 $GRAFT_REPO_ROOT/tools/gv_$v/ubench_gemm $s | tail -1 | sed "s/^/$v /" || exit 1; done
done
done > $O/${TAG}.txt 2>&1 || { cat $O/${TAG}.txt; exit 1; }
cat $O/${TAG}.txt
