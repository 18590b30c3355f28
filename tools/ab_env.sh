#!/bin/bash
# same-box A/B of dev environment switches on one bench workload:
#   VAR=SMG_GEMM_TRI VALS="0 12864 6402" tools/ab_env.sh hvp
set -o pipefail
W=${1:-gp}
mkdir -p gpurun_out
for r in 1 2; do
  for v in ${VALS}; do
    env $VAR=$v timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --steps ${STEPS:-10} > gpurun_out/ab_env.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/ab_env.json'));print('$VAR=$v', round(d['value'],3), round(d['ms_per_step'],4))"
  done
done
