#!/bin/bash
# one GPU call: every bench workload (with its CPU baseline), the rocprofv3
# kernel-trace summary of the default (GP) bench, and the PMC traffic passes.
# Each step is time-limited; the first failure ends the call.
set -o pipefail
TAG=${1:-m}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
for w in gp glm mulchol hvp; do
  timeout -k 10 400 python bench.py --workload $w > $O/${TAG}_bench_$w.json 2> $O/${TAG}_bench_$w.err || { tail $O/${TAG}_bench_$w.err; exit 1; }
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_prof.log 2>&1 || exit 1
bash $GRAFT_REPO_ROOT/tools/pmc_traffic.sh $TAG || exit 1
echo done
