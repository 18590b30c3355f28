#!/bin/bash
# gp_eigen under host-thread / CPU-placement variants ($1 tag), alternating, 2 rounds
set -o pipefail
TAG=${1:-r05e}
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
echo "visible: HIP=$HIP_VISIBLE_DEVICES ROCR=$ROCR_VISIBLE_DEVICES"
python3 -c "import ctypes;h=ctypes.CDLL('libamdhip64.so');b=ctypes.create_string_buffer(64);h.hipDeviceGetPCIBusId(b,64,0);print('gpu bus', b.value)" 2>&1 | tail -1
run() {  # name prefix...
  local name=$1; shift
  "$@" timeout -k 10 300 python bench.py --workload gp_eigen --steps 20 --no-cpu-baseline --no-glm-strong > $O/${TAG}_$name.json 2> $O/${TAG}_$name.err || { tail $O/${TAG}_$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${TAG}_$name.json'));p=d['eval_phases_ms'];print('$name', round(d['value'],1), round(p['forward_K'],2), round(p['forward_Kd'],2), round(p['forward_L'],2))"
}
for r in 1 2; do
  run t16_$r env || exit 1
  run t8_$r env SMG_HOST_THREADS=8 || exit 1
  run t15_$r env SMG_HOST_THREADS=15 || exit 1
  run n0_$r taskset -c 0-63,128-191 || exit 1
  run n1_$r taskset -c 64-127,192-255 || exit 1
done
