#!/bin/bash
# zero-request instantiation: parity (zero-request / relaxed / c3p / c3 full), then the C3 / c3p A/B vs 1a24a29
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py -k "zero_request or relaxed or golden" tests/test_gpu_c3_full.py > gpurun_out/r06zr_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06zr_pytest.log; [ $rc -ne 0 ] && exit $rc
bash scripts/ab_stats.sh r06zr3 c3 1000000 "c4u new" 10 > gpurun_out/r06zr.txt 2>&1 || { cat gpurun_out/r06zr.txt; exit 1; }
bash scripts/ab_stats.sh r06zrp c3p 1000000 "c4u new" 10 >> gpurun_out/r06zr.txt 2>&1 || { cat gpurun_out/r06zr.txt; exit 1; }
cat gpurun_out/r06zr.txt
