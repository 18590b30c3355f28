set -o pipefail
mkdir -p gpurun_out
STEPS=30 bash tools/ab_lib.sh casync gp || exit 1
cp var/casync/libsmg_hip.so math_amd/lib/libsmg_hip.so
bash tools/prof_bench.sh ca gp
tail -2 gpurun_out/ca_prof.log
