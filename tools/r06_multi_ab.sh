#!/bin/bash
# same-box GP A/B of several control builds against the tree: $1 = rounds, rest = _bisect dirs
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
TAG=${TAG:-mab}
R=$1; shift
for r in $(seq 1 $R); do
  for v in "$@" .; do
    n=$(basename $v); [ "$v" = . ] && n=tree
    d=$GRAFT_REPO_ROOT/$v; [ "$v" != . ] && d=$GRAFT_REPO_ROOT/_bisect/$v
    (cd $d && timeout -k 10 300 python bench.py --workload ${WL:-gp} --steps 20 --no-cpu-baseline --no-glm-strong) > $O/${TAG}_${n}_$r.json 2> $O/${TAG}_${n}_$r.err || { tail $O/${TAG}_${n}_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/${TAG}_${n}_$r.json'));print('$n', round(d['value'],1), round(d['ms_per_step'],4))"
  done
done
