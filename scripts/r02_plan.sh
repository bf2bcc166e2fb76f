#!/bin/bash
# planner iteration: planner/rsp/C4/Divide parity, then the C4 bench line + phase split + kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-pl}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "planner or rsp or c4 or divide or fuzz or plan_rows or scratch or c5" > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r02_c4.sh "$tag"
