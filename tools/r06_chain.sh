#!/bin/bash
# panel-kernel change: the panel / Cholesky / GP GPU tests, the panel trace, a same-box GP A/B against _bisect/head
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-ch}
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread -k "${KX:-cholesky or panel or gp_ or handoff or progressive or smoke}" > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
tail -2 $O/${TAG}_pytest.log
timeout -k 10 120 ./tools/ubench_panel > $O/${TAG}_ubp.txt 2>&1 || { tail $O/${TAG}_ubp.txt; exit 1; }
grep -E "panel kernel" $O/${TAG}_ubp.txt
grep -E "^WG 0:" $O/${TAG}_ubp.txt | head -c 1500; echo
TAG=$TAG bash tools/r06_multi_ab.sh ${R:-3} ${CTL:-head} || exit 1
echo chain done
