set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_cpp_layer.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r03w_t.log 2>&1; rc=$?
tail -15 gpurun_out/r03w_t.log; [ $rc -eq 0 ] || exit $rc
for V in 1 0 1 0; do
  SMG_CHOL_MVN_CLOSED_FORM=$V timeout -k 10 300 python bench.py --workload gp --steps 20 --no-cpu-baseline > gpurun_out/r03w.json 2> gpurun_out/r03w.err || { tail gpurun_out/r03w.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03w.json')); print('closed=$V', round(d['value'],2), round(d['ms_per_step'],3))"
done
