set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for V in 0 1; do
  SMG_HOST_STREAM=$V timeout -k 10 300 python bench.py --workload gp_eigen --steps 10 --no-cpu-baseline > gpurun_out/r03u.json 2> gpurun_out/r03u.err || { tail gpurun_out/r03u.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03u.json')); print('stream=$V', round(d['value'],2), round(d['ms_per_step'],2), {k: round(v,2) for k, v in d['bridge_cost_ms'].items() if k != 'note'}, round(d['eval_phases_ms']['forward'],2))"
done; done
