#!/bin/bash
# one GPU call: a pytest subset (-k expr in $2), the GP kernel trace summary,
# and $3 (default 2) GP bench lines.  $1 = tag.
set -o pipefail
TAG=${1:-ab}; K=${2:-gemm}; NB=${3:-2}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -q -m gpu -k "$K" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_t.log 2>&1; rc=$?
tail -2 gpurun_out/${TAG}_t.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_bench.sh ${TAG} gp || exit 1
python3 tools/rocpd_summary.py gpurun_out/${TAG}_prof/run_results.db 12
for i in $(seq $NB); do
  timeout -k 10 300 python bench.py --workload ${W:-gp} --no-cpu-baseline > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err || { tail gpurun_out/${TAG}_b$i.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_b$i.json')); print('bench', d['value'], d['ms_per_step'])"
done
