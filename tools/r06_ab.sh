#!/bin/bash
# same-box A/B: the GP bench of the control build (_bisect/$1) and the tree, $2 rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${3:-ab}
for r in $(seq 1 ${2:-3}); do
  for v in _bisect/$1 .; do
    n=$(basename $v); [ "$v" = . ] && n=tree
    (cd $GRAFT_REPO_ROOT/$v && timeout -k 10 300 python bench.py --workload ${WL:-gp} --steps 20 --no-cpu-baseline --no-glm-strong) > $O/${TAG}_${n}_$r.json 2> $O/${TAG}_${n}_$r.err || { tail $O/${TAG}_${n}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${TAG}_${n}_$r.json'));print('$n', d['value'], d['ms_per_step'])"
  done
done
