#!/bin/bash
# one GPU call (round 5): selected GPU tests ($K: pytest -k expression, or
# none), then alternating GP bench runs with an env switch off/on ($V, e.g.
# SMG_MVN_INV), $REP times each, then optional extras.  Each step
# time-limited; the first failure ends it.
set -o pipefail
TAG=${1:-r05ab}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
if [ "${K:-none}" != none ]; then
  timeout -k 10 900 python -u -m pytest tests -q -m gpu -x -k "$K" --timeout 300 --timeout-method thread > $O/${TAG}_pytest.log 2>&1 || { tail -40 $O/${TAG}_pytest.log; exit 1; }
  tail -3 $O/${TAG}_pytest.log
fi
W=${WL:-gp}
for r in $(seq 1 ${REP:-2}); do
  for v in ${VALS:-0 1}; do
    if [ -n "$V" ]; then export $V=$v; fi
    timeout -k 10 300 python bench.py --workload $W --steps 20 --no-cpu-baseline --no-glm-strong > $O/${TAG}_${v}_$r.json 2> $O/${TAG}_${v}_$r.err || { tail $O/${TAG}_${v}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${TAG}_${v}_$r.json'));print('$V=$v', d['value'], d['ms_per_step'])"
  done
done
unset $V
if [ "${UBT:-0}" = 1 ]; then
  timeout -k 10 120 ./tools/ubench_timeline > $O/${TAG}_ubt.txt 2>&1 || { tail $O/${TAG}_ubt.txt; exit 1; }
  head -8 $O/${TAG}_ubt.txt
fi
if [ "${PROF:-0}" = 1 ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/${TAG}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-glm-strong > $O/${TAG}_prof.log 2>&1 || { tail $O/${TAG}_prof.log; exit 1; }
  echo prof ok
fi
