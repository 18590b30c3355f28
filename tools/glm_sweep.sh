#!/bin/bash
# GLM streaming-kernel variant sweep on one box (SMG_GLM_REG x SMG_GLM_NB)
set -o pipefail
mkdir -p gpurun_out
for v in ${VARIANTS:-0 1 2 3}; do
  for nb in ${NBS:-256 512}; do
    SMG_GLM_REG=$v SMG_GLM_NB=$nb timeout -k 10 200 python bench.py --workload glm --no-cpu-baseline --steps 30 > gpurun_out/sw.json || exit 1
    python -c "import json;d=json.load(open('gpurun_out/sw.json'));print('REG=$v NB=$nb', round(d['value'],2), round(d['roofline']['achieved'],1))"
  done
done
