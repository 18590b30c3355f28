#!/bin/bash
# rocprofv3 kernel + memory-copy trace of a short gp_eigen bench ($1 tag) -> gpurun_out/<tag>_eig/
set -o pipefail
TAG=${1:-r05t}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace -d $O/${TAG}_eig -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload gp_eigen --steps 4 --warmup 2 --no-cpu-baseline > $O/${TAG}_eig.log 2>&1 || { tail $O/${TAG}_eig.log; exit 1; }
echo trace done
