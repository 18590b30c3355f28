#!/bin/bash
# rocprofv3 kernel-trace summaries of the GP bench for the control build (_bisect/$1) and the tree
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out
TAG=${2:-st}
cd /tmp && export TMPDIR=/tmp
for v in _bisect/$1 .; do
  n=$(basename $v); [ "$v" = . ] && n=tree
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_${n} -o run -- python3 $GRAFT_REPO_ROOT/$v/bench.py --workload gp --steps 10 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_${n}.log 2>&1 || { tail $O/${TAG}_${n}.log; exit 1; }
done
echo stats done
