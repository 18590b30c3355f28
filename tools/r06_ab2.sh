#!/bin/bash
# same-box: panel ubench of control + tree, then GP A/B rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${2:-ab}
for v in _bisect/$1 .; do
  n=$(basename $v); [ "$v" = . ] && n=tree
  (cd $GRAFT_REPO_ROOT/$v && timeout -k 10 120 ./tools/ubench_panel) > $O/${TAG}_ubp_$n.txt 2>&1 || { tail $O/${TAG}_ubp_$n.txt; exit 1; }
  echo $n; grep "panel kernel" $O/${TAG}_ubp_$n.txt
done
bash $GRAFT_REPO_ROOT/tools/r06_ab.sh $1 ${3:-3} $TAG
