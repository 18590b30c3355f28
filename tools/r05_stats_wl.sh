#!/bin/bash
# rocprofv3 kernel-trace summary of one bench workload ($2, tag $1) -> gpurun_out/<tag>_stats/
set -o pipefail
TAG=${1:-r05w}
W=${2:-hvp}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_stats -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload $W --steps 4 --warmup 1 --no-cpu-baseline > $O/${TAG}_stats.log 2>&1 || { tail $O/${TAG}_stats.log; exit 1; }
echo stats done
