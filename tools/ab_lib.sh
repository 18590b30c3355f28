#!/bin/bash
# A/B of a variant libsmg_hip.so (var/<name>/, dev builds) against the
# in-tree one on a bench workload, alternating runs on the same box; the
# variant is swapped into math_amd/lib of the box's copy of the tree (the
# Python binding loads the library by path) and swapped back at the end
# usage: tools/ab_lib.sh <name> [workload]
set -o pipefail
V=$1; W=${2:-gp}
LIB=$GRAFT_REPO_ROOT/math_amd/lib/libsmg_hip.so
mkdir -p gpurun_out
cp $LIB /tmp/ab_base.so || exit 1
rc=0
for r in 1 2 3; do
  cp /tmp/ab_base.so $LIB
  timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --steps ${STEPS:-40} > gpurun_out/ab_base.json || { rc=1; break; }
  python -c "import json;d=json.load(open('gpurun_out/ab_base.json'));print('base', round(d['value'],2), round(d['ms_per_step'],4))"
  cp $GRAFT_REPO_ROOT/var/$V/libsmg_hip.so $LIB
  timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --steps ${STEPS:-40} > gpurun_out/ab_var.json || { rc=1; break; }
  python -c "import json;d=json.load(open('gpurun_out/ab_var.json'));print('$V', round(d['value'],2), round(d['ms_per_step'],4))"
done
cp /tmp/ab_base.so $LIB
exit $rc
