#!/bin/bash
# rocprofv3 HIP-API + kernel trace of a short GP bench (tag $1): when the host
# issued each launch against when the kernel ran -> gpurun_out/<tag>_hip/
set -o pipefail
TAG=${1:-r05h}
O=$GRAFT_REPO_ROOT/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --hip-trace -d $O/${TAG}_hip -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 4 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_hip.log 2>&1 || { tail $O/${TAG}_hip.log; exit 1; }
echo hiptrace done
