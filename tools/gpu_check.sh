#!/bin/bash
# one GPU call: tests, smoke, bench, rocprof summary (each step time-limited)
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-run}
timeout -k 10 900 python -u -m pytest tests -q -m gpu -x --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1; echo "pytest rc=$?" >> gpurun_out/${TAG}_pytest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/${TAG}_smoke.log; exit 1; }
timeout -k 10 600 python bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || { echo "bench failed"; tail gpurun_out/${TAG}_bench.err; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/${TAG}_prof.log 2>&1
echo "prof rc=$?"
