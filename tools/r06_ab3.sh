#!/bin/bash
# targeted GPU tests, then same-box A/Bs (GP, then HVP) against _bisect/$CTL
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:?tag}
K=${KX:-gp or hessian or cholesky or handoff or mvn or progressive}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "$K" > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
tail -2 $O/${TAG}_pytest.log
WL=gp TAG=${TAG}g bash tools/r06_multi_ab.sh ${RG:-3} ${CTL:-head} || exit 1
[ "${RH:-0}" -gt 0 ] && { WL=hvp TAG=${TAG}h bash tools/r06_multi_ab.sh $RH ${CTL:-head} || exit 1; }
echo ab3 done
