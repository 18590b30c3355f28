#!/bin/bash
# round-6 final build: smoke, then the HVP bench's kernel-trace summary
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-r06f}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/${TAG}_smoke.log 2>&1 || { tail $O/${TAG}_smoke.log; exit 1; }
cat $O/${TAG}_smoke.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_hvpprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload hvp --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_hvpprof.log 2>&1 || exit 1
echo final done
