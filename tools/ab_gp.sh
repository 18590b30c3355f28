#!/bin/bash
# A/B of an env switch on the GP bench on one box: alternating runs
# usage: tools/ab_gp.sh VAR [workload]
set -o pipefail
V=$1; W=${2:-gp}
mkdir -p gpurun_out
for r in 1 2 3; do
  for x in 0 1; do
    env $V=$x timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --steps 40 > gpurun_out/ab_$x.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_$x.json'));print('$V=$x', round(d['value'],2), round(d['ms_per_step'],4))"
  done
done
