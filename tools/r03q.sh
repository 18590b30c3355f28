set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu -k "hessian or hvp or tangent or mdivide or tri or mvn or gp_marginal or boundary" --timeout 800 --timeout-method thread > gpurun_out/r03q_t.log 2>&1; rc=$?
tail -5 gpurun_out/r03q_t.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --workload hvp --steps 10 --no-cpu-baseline > gpurun_out/r03q.json 2> gpurun_out/r03q.err || { tail gpurun_out/r03q.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03q.json')); print('hvp', d['value'], d['ms_per_step'])"
done
bash tools/prof_bench.sh r03q hvp || exit 1
python3 tools/rocpd_summary.py gpurun_out/r03q_prof/run_results.db 16
