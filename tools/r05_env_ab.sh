#!/bin/bash
# one GPU call (round 5): alternating GP bench runs under env settings given
# as $CFGS (';'-separated, each a space-separated list of VAR=VALUE, "-" for
# none), $REP times; each run time-limited, the first failure ends it
set -o pipefail
TAG=${1:-r05env}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
W=${WL:-gp}
IFS=';' read -ra CS <<< "$CFGS"
for r in $(seq 1 ${REP:-2}); do
  i=0
  for c in "${CS[@]}"; do
    i=$((i+1))
    E=""; [ "$c" != "-" ] && E="$c"
    env $E timeout -k 10 300 python bench.py --workload $W --steps 20 --no-cpu-baseline --no-glm-strong > $O/${TAG}_${i}_$r.json 2> $O/${TAG}_${i}_$r.err || { tail $O/${TAG}_${i}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${TAG}_${i}_$r.json'));print('[$c]', d['value'], d['ms_per_step'])"
  done
done
