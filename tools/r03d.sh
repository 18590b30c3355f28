set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_boundary.py tests/test_cpp_layer.py -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03d_pytest.log 2>&1; rc=$?; tail -5 gpurun_out/r03d_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload gp_eigen --steps 10 --no-cpu-baseline > gpurun_out/r03d_gpe.json 2> gpurun_out/r03d_gpe.err || { tail gpurun_out/r03d_gpe.err; exit 1; }
python -c "
import json
d=json.load(open('gpurun_out/r03d_gpe.json')); print(d['value'], d['ms_per_step'], d.get('bridge_cost_ms'))
"
