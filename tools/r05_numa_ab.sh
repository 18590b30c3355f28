#!/bin/bash
# one GPU call: gp_eigen (and gp) bench with the process unbound, bound to the
# GPU's NUMA node's CPUs, and bound to the other node's ($REP rounds)
set -o pipefail
TAG=${1:-r05numa}
O=$GRAFT_REPO_ROOT/gpurun_out
mkdir -p $O
cd $GRAFT_REPO_ROOT
node=$(rocm-smi --showtoponuma 2>/dev/null | grep -m1 "Numa Node:" | awk '{print $NF}')
local_cpus=$(cat /sys/devices/system/node/node${node:-0}/cpulist)
other=$((1 - ${node:-0}))
remote_cpus=$(cat /sys/devices/system/node/node$other/cpulist 2>/dev/null || echo "$local_cpus")
echo "gpu numa node $node local $local_cpus remote $remote_cpus"
for r in $(seq 1 ${REP:-2}); do
  for v in none local remote; do
    case $v in
      none) PRE="" ;;
      local) PRE="taskset -c $local_cpus" ;;
      remote) PRE="taskset -c $remote_cpus" ;;
    esac
    for w in ${WLS:-gp_eigen}; do
      timeout -k 10 300 $PRE python bench.py --workload $w --steps 10 --no-cpu-baseline --no-glm-strong > $O/${TAG}_${w}_${v}_$r.json 2> $O/${TAG}_${w}_${v}_$r.err || { tail $O/${TAG}_${w}_${v}_$r.err; exit 1; }
      python -c "import json;d=json.load(open('$O/${TAG}_${w}_${v}_$r.json'));p=d.get('eval_phases_ms',{});print('$w $v', round(d['value'],1), round(d['ms_per_step'],2), p.get('forward_K'), p.get('forward_L'))"
    done
  done
done
