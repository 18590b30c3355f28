#!/bin/bash
# one GPU call: the GPU test suite (optionally a subset: extra pytest args),
# time-limited, log under gpurun_out/
set -o pipefail
mkdir -p gpurun_out
TAG=${1:-t}
shift
timeout -k 10 900 python -u -m pytest tests -q -m gpu --maxfail=15 --timeout 200 --timeout-method thread "$@" > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -40 gpurun_out/${TAG}_pytest.log
exit $rc
