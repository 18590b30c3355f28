#!/bin/bash
# GP bench of a control build (_bisect/<commit>, $1) beside the current tree, $2 rounds
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
for r in $(seq 1 ${2:-2}); do
  for v in _bisect/$1 .; do
    (cd $GRAFT_REPO_ROOT/$v && timeout -k 10 300 python bench.py --workload gp --steps 20 --no-cpu-baseline --no-glm-strong) > $O/ctl_$(basename $v)_$r.json 2> $O/ctl_$(basename $v)_$r.err || { tail $O/ctl_$(basename $v)_$r.err; exit 1; }
    python -c "import json;d=json.load(open('$O/ctl_$(basename $v)_$r.json'));print('$v', d['value'], d['ms_per_step'])"
  done
done
