#!/bin/bash
# PMC passes (separate runs, kernel-trace only) for one ubench_gemm shape
set -o pipefail
SHAPE=${1:-3}
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc_gemm_$SHAPE
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES -d $OUT/p1 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $SHAPE > $OUT/p1.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc FETCH_SIZE GRBM_GUI_ACTIVE -d $OUT/p2 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $SHAPE > $OUT/p2.log 2>&1 || exit 1
timeout -k 10 120 rocprofv3 --kernel-trace --stats --pmc WRITE_SIZE SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d $OUT/p3 -o run -- $GRAFT_REPO_ROOT/tools/ubench_gemm $SHAPE > $OUT/p3.log 2>&1 || exit 1
echo done
