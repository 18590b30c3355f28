set -o pipefail
mkdir -p gpurun_out
for W in gp gp_eigen; do
  timeout -k 10 300 python bench.py --workload $W --steps 20 --no-cpu-baseline > gpurun_out/r03v_$W.json 2> gpurun_out/r03v_$W.err || { tail gpurun_out/r03v_$W.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/r03v_$W.json')); print('$W', round(d['value'],2), round(d['ms_per_step'],3), d.get('eval_phases_ms'), d.get('bridge_cost_ms'))"
done
