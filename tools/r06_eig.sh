#!/bin/bash
# gp_eigen: host THP mode, and the line at two warmups (the ramp within a process)
set -o pipefail
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O
cd $GRAFT_REPO_ROOT
TAG=${1:-eig}
{ cat /sys/kernel/mm/transparent_hugepage/enabled /sys/kernel/mm/transparent_hugepage/defrag; nproc; free -g | head -2; } > $O/${TAG}_host.txt 2>&1
cat $O/${TAG}_host.txt
for wu in ${WUS:-3 40}; do
  timeout -k 10 300 python bench.py --workload gp_eigen --warmup $wu --steps ${ST:-20} --no-cpu-baseline > $O/${TAG}_w$wu.json 2> $O/${TAG}_w$wu.err || { tail $O/${TAG}_w$wu.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${TAG}_w$wu.json'));print('warmup $wu', d['value'], d['ms_per_step'], d['eval_phases_ms']['gradient_call'])"
done
