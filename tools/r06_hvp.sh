#!/bin/bash
# HVP: parity tests, same-box A/B against a control build, a kernel-trace summary
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-hvp}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 600 --timeout-method thread -k "${KX:-hessian}" > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
tail -2 $O/${TAG}_pytest.log
WL=hvp TAG=$TAG bash tools/r06_multi_ab.sh ${R:-2} ${CTL:-base} || exit 1
if [ "${PROF:-1}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload hvp --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_prof.log 2>&1 || exit 1
fi
echo hvp done
