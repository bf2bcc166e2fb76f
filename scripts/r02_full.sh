#!/bin/bash
# Full GPU suite, then rocprofv3 passes (kernel trace + SQ + HBM) of the two bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-f}
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest_gpu.log 2>&1
rc=$?; tail -5 gpurun_out/${tag}_pytest_gpu.log; echo "== pytest rc=$rc"
[ $rc -ne 0 ] && exit $rc
UNITS=1000000 bash scripts/profile.sh c3 ${tag} || exit $?
bash scripts/profile.sh c2 ${tag}
