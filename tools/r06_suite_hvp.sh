#!/bin/bash
# the full GPU suite, then the HVP parity tests / A-B / kernel trace, then the kernel-gap probe
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-r06t}
timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 300 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -30 $O/${TAG}_pytest.log; exit 1; }
tail -2 $O/${TAG}_pytest.log
WL=hvp TAG=${TAG}_hvp bash tools/r06_multi_ab.sh 2 base || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/${TAG}_hvpprof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload hvp --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_hvpprof.log 2>&1 || exit 1
timeout -k 10 60 $GRAFT_REPO_ROOT/tools/ubench_kgap > $O/${TAG}_kgap.txt 2>&1 || exit 1
cat $O/${TAG}_kgap.txt
