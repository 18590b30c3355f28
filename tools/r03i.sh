set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do for IO in 1 0; do for R in 1.25e6 1e7; do
 SMG_GLM_IO=$IO timeout -k 10 300 python bench.py --workload glm --rows $R --steps 100 --no-cpu-baseline > gpurun_out/r03i.json 2> gpurun_out/r03i.err || { tail gpurun_out/r03i.err; exit 1; }
 python3 -c "import json; d=json.load(open('gpurun_out/r03i.json')); r=d['roofline']; print('io=$IO', '$R', round(d['ms_per_step'],4), round(r['frac'],3), round(r['avg_launch_ms'],4), round(r['step_minus_glm_kernels_us'],1))"
done; done; done
