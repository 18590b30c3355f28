#!/bin/bash
# PMC HBM traffic of the GP bench with the panel kernel's register-resident
# below-panel tiles off (tag ${1}0) and on (tag ${1}1): calibration + FETCH_SIZE
# and WRITE_SIZE passes each (kernel-trace only), as tools/pmc_traffic.sh
set -o pipefail
TAG=${1:-r05p}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
for r in 0 1; do
  T=${TAG}$r
  run() {  # name counter cmd...
    local name=$1 ctr=$2; shift 2
    SMG_PANEL_RESIDENT=$r timeout -k 10 300 rocprofv3 --kernel-trace --pmc $ctr -d $O/pmc_${T}_${name} -o run -- "$@" > $O/pmc_${T}_${name}.log 2>&1
  }
  run calib_fetch FETCH_SIZE $GRAFT_REPO_ROOT/tools/calib_fetch || exit 1
  run calib_write WRITE_SIZE $GRAFT_REPO_ROOT/tools/calib_fetch || exit 1
  run gp_fetch FETCH_SIZE python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-glm-strong || exit 1
  run gp_write WRITE_SIZE python3 $GRAFT_REPO_ROOT/bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-glm-strong || exit 1
done
echo pmc done
