set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -k "gemm or hessian or hvp or tangent or tri or chol or gp or mvn or boundary or spd" --timeout 800 --timeout-method thread > gpurun_out/r03s_t.log 2>&1; rc=$?
tail -2 gpurun_out/r03s_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do for W in hvp gp mulchol; do
  timeout -k 10 300 python bench.py --workload $W --steps 10 --no-cpu-baseline > gpurun_out/r03s.json 2> gpurun_out/r03s.err || { tail gpurun_out/r03s.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03s.json')); print('$W', d['value'], d['ms_per_step'])"
done; done
