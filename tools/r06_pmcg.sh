#!/bin/bash
# ubench_gemm shapes: time + PMC passes (MFMA busy / waits / LDS, fetch, write)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${1:-pmcg}; shift
for s in ${@:-2 18 19}; do timeout -k 10 60 $GRAFT_REPO_ROOT/tools/ubench_gemm $s | tail -1 || exit 1; done > $O/${TAG}.txt 2>&1 || { cat $O/${TAG}.txt; exit 1; }
cat $O/${TAG}.txt
cd /tmp && export TMPDIR=/tmp
for s in ${@:-2 18 19}; do
  D=$O/${TAG}_s$s; mkdir -p $D
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $D/p1 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $s > $D/p1.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $D/p2 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $s > $D/p2.log 2>&1 || exit 1
  timeout -s KILL 60 rocprofv3 --kernel-trace --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_F64 -d $D/p3 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $s > $D/p3.log 2>&1 || exit 1
done
echo pmcg done
