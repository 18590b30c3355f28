set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cpp_functors.py tests/test_boundary.py -q -m gpu --timeout 300 --timeout-method thread -k "multi_block or full_size or boundary or bridge or nan_poisoned or gp_nd" > gpurun_out/r03c_pytest.log 2>&1; rc=$?; tail -15 gpurun_out/r03c_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload gp --no-cpu-baseline > gpurun_out/r03c_gp.json 2> gpurun_out/r03c_gp.err || { tail gpurun_out/r03c_gp.err; exit 1; }
timeout -k 10 300 python bench.py --workload gp_eigen --steps 10 --no-cpu-baseline > gpurun_out/r03c_gpe.json 2> gpurun_out/r03c_gpe.err || { tail gpurun_out/r03c_gpe.err; exit 1; }
SMG_BENCH_MALLOC_TUNING=0 timeout -k 10 300 python bench.py --workload gp_eigen --steps 10 --no-cpu-baseline > gpurun_out/r03c_gpe0.json 2> gpurun_out/r03c_gpe0.err || { tail gpurun_out/r03c_gpe0.err; exit 1; }
python -c "
import json
for f in ['gp','gpe','gpe0']:
    d=json.load(open('gpurun_out/r03c_%s.json'%f)); print(f, d['value'], d['ms_per_step'], d.get('bridge_cost_ms'))
"
