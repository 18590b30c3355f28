set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -q -m gpu --maxfail=10 --timeout 300 --timeout-method thread > gpurun_out/r03e_pytest.log 2>&1; rc=$?; tail -15 gpurun_out/r03e_pytest.log; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do timeout -k 10 300 python bench.py --workload gp --no-cpu-baseline > gpurun_out/r03e_gp$i.json 2> gpurun_out/r03e_gp$i.err || { tail gpurun_out/r03e_gp$i.err; exit 1; }; done
timeout -k 10 300 python bench.py --workload mulchol --no-cpu-baseline > gpurun_out/r03e_mc.json 2> gpurun_out/r03e_mc.err || { tail gpurun_out/r03e_mc.err; exit 1; }
timeout -k 10 300 python bench.py --workload hvp --no-cpu-baseline > gpurun_out/r03e_hvp.json 2> gpurun_out/r03e_hvp.err || { tail gpurun_out/r03e_hvp.err; exit 1; }
python -c "
import json
for f in ['gp1','gp2','mc','hvp']:
    d=json.load(open('gpurun_out/r03e_%s.json'%f)); print(f, d['value'], d['ms_per_step'])
"
