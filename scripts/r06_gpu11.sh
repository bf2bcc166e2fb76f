#!/bin/bash
# full GPU suite, then round-5 head vs the tree on every config
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -v --timeout 300 --timeout-method thread -m gpu > gpurun_out/r06s_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06s_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/r06_gpu10.sh
