#!/bin/bash
# one GPU call: the GPU test suite, then one bench line per workload named in
# $2.. (default gp), no CPU baseline.  Each step time-limited; first failure ends it.
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-t}
shift
WLS=${@:-gp}
timeout -k 10 800 python -u -m pytest tests -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -3 gpurun_out/${TAG}_pytest.log
for w in $WLS; do
  timeout -k 10 300 python bench.py --workload $w --no-cpu-baseline > gpurun_out/${TAG}_bench_$w.json 2> gpurun_out/${TAG}_bench_$w.err || { tail gpurun_out/${TAG}_bench_$w.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_bench_$w.json'));print('$w', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
