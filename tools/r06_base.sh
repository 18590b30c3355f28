#!/bin/bash
# round-6 baseline: panel trace, factor phases, two GP bench lines
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-r06a}
timeout -k 10 120 ./tools/ubench_panel > $O/${TAG}_ubp.txt 2>&1 || { tail $O/${TAG}_ubp.txt; exit 1; }
grep "panel kernel" $O/${TAG}_ubp.txt
timeout -k 10 120 ./tools/ubench_phase > $O/${TAG}_phase.txt 2>&1 || { tail $O/${TAG}_phase.txt; exit 1; }
cat $O/${TAG}_phase.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --workload gp --steps 20 --no-cpu-baseline --no-glm-strong > $O/${TAG}_gp$r.json 2> $O/${TAG}_gp$r.err || { tail $O/${TAG}_gp$r.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_gp$r.json'));print('gp', d['value'], d['ms_per_step'])"
done
