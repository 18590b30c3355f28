set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -q -m gpu -k "glm or sharding or map_rect" --timeout 300 --timeout-method thread > gpurun_out/r03h_t.log 2>&1; rc=$?; tail -3 gpurun_out/r03h_t.log; [ $rc -eq 0 ] || exit $rc
for R in 1e7 1.25e6; do
 timeout -k 10 300 python bench.py --workload glm --rows $R --steps 50 --no-cpu-baseline > gpurun_out/r03h_glm_$R.json 2> gpurun_out/r03h_glm_$R.err || { tail gpurun_out/r03h_glm_$R.err; exit 1; }
 python3 -c "import json; d=json.load(open('gpurun_out/r03h_glm_$R.json')); r=d['roofline']; print('$R', d['value'], d['ms_per_step'], r['frac'], r['avg_launch_ms'], r['step_minus_glm_kernels_us'])"
done
