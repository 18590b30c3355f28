#!/bin/bash
# HBM traffic from PMC counters, one counter group per pass (kernel-trace only),
# for the calibration kernel and the GP / GLM benches.  Output DBs under
# gpurun_out/pmc_<tag>_{calib,gp,glm}_{fetch,write}/.
set -o pipefail
TAG=${1:-r01}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
run() {  # name counter cmd...
  local name=$1 ctr=$2; shift 2
  timeout -k 10 600 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${TAG}_${name} -o run -- "$@" > $O/pmc_${TAG}_${name}.log 2>&1
}
run calib_fetch FETCH_SIZE $GRAFT_REPO_ROOT/tools/calib_fetch || exit 1
run calib_write WRITE_SIZE $GRAFT_REPO_ROOT/tools/calib_fetch || exit 1
run glm_fetch FETCH_SIZE python3 $GRAFT_REPO_ROOT/bench.py --workload glm --steps 2 --warmup 1 --no-cpu-baseline || exit 1
run glm_write WRITE_SIZE python3 $GRAFT_REPO_ROOT/bench.py --workload glm --steps 2 --warmup 1 --no-cpu-baseline || exit 1
run gp_fetch FETCH_SIZE python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-glm-strong || exit 1
run gp_write WRITE_SIZE python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-glm-strong || exit 1
echo done
