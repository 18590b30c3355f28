#!/bin/bash
# rocprofv3 kernel trace of one bench workload (few steps): $1 = tag, $2 = workload
set -o pipefail
TAG=${1:-p}; W=${2:-gp}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 3 --warmup 2 --no-cpu-baseline > $O/${TAG}_prof.log 2>&1
echo "rc=$?" >> $O/${TAG}_prof.log
