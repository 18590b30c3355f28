#!/bin/bash
# rocprofv3 kernel-trace summary of the GP bench (tag $1): per-kernel counts and
# average durations -> gpurun_out/<tag>_stats/
set -o pipefail
TAG=${1:-r05s}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_stats.log 2>&1 || { tail $O/${TAG}_stats.log; exit 1; }
echo stats done
