#!/bin/bash
# gp_eigen: the NUMA-pinned host pool against unpinned / the old 16 threads ($1 tag), alternating, 3 rounds
set -o pipefail
TAG=${1:-r05f}
O=$GRAFT_REPO_ROOT/gpurun_out; mkdir -p $O; cd $GRAFT_REPO_ROOT
python3 -c "
import ctypes;l=ctypes.CDLL('math_amd/lib/libsmg_hip.so');print('device numa node', l.smg_device_numa_node(0))"
run() {  # name env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --workload gp_eigen --steps 20 --no-cpu-baseline --no-glm-strong > $O/${TAG}_$name.json 2> $O/${TAG}_$name.err || { tail $O/${TAG}_$name.err; return 1; }
  python3 -c "import json;d=json.load(open('$O/${TAG}_$name.json'));p=d['eval_phases_ms'];print('$name', round(d['value'],1), round(p['forward_K'],2), round(p['forward_Kd'],2), round(p['forward_L'],2))"
}
for r in 1 2 3; do
  run pin_$r SMG_X=1 || exit 1
  run nopin_$r SMG_HOST_PIN=0 || exit 1
  run old_$r SMG_HOST_PIN=0 SMG_HOST_THREADS=16 || exit 1
done
