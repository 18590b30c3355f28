#!/bin/bash
# one GPU call: the tests named by $K, the GP bench, and a kernel-trace summary
# of the GP bench.  Each step time-limited; the first failure ends it.
set -o pipefail
TAG=${1:-q}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -q -m gpu -x -k "$K" --timeout 200 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
  tail -2 $O/${TAG}_pytest.log
fi
for w in ${WLS:-gp}; do
  timeout -k 10 400 python bench.py --workload $w --steps 20 --no-cpu-baseline > $O/${TAG}_bench_$w.json 2> $O/${TAG}_bench_$w.err || { tail $O/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
[ "${PROF:-1}" = 1 ] || exit 0
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $O/${TAG}_prof.log 2>&1 || exit 1
echo done
