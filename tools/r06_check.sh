#!/bin/bash
# round-6: targeted GPU tests, smoke, then the baseline measurements (tools/r06_base.sh)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-r06b}
K=${KEXPR:-two_inverse or N1024 or progressive_inverses or intermediate or closed_form}
timeout -k 10 ${TT:-600} python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread -k "$K" > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
tail -3 $O/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail $O/${TAG}_smoke.log; exit 1; }
cat $O/${TAG}_smoke.log
if [ "${BASE:-1}" = 1 ]; then bash tools/r06_base.sh $TAG; fi
