#!/bin/bash
# GEMM microbench over the listed ub_shapes indices (default: the big NN and
# the HVP tangent products), then FETCH_SIZE / WRITE_SIZE passes on $PMC shapes
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${1:-ubg}; shift
SH=${@:-17 24 25 26 27 28 29 30 31}
for s in $SH; do timeout -k 10 60 $GRAFT_REPO_ROOT/tools/ubench_gemm $s | tail -1 || exit 1; done > $O/${TAG}.txt 2>&1 || { cat $O/${TAG}.txt; exit 1; }
cat $O/${TAG}.txt
cd /tmp && export TMPDIR=/tmp
for s in ${PMC:-}; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $O/${TAG}_pmc$s/f -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $s > $O/${TAG}_pmc$s.log 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES -d $O/${TAG}_pmc$s/w -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $s >> $O/${TAG}_pmc$s.log 2>&1 || exit 1
done
echo ubg done
