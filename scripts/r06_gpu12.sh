#!/bin/bash
# word-coalesced req_row_kernel: parity (requirement rows, label-free ops, C5 subsets, fuzz), then C5 / C3 A/B
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "requirement or label_free or c5 or fuzz or golden_filter" > gpurun_out/r06rc_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06rc_pytest.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_full_configs.py \
  -k c5 > gpurun_out/r06rc_pytest2.log 2>&1
rc=$?; tail -3 gpurun_out/r06rc_pytest2.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/r06rc.txt
for r in 1 2; do bash scripts/ab_stats.sh r06rc${r} c5 100000 "rc0 new" 10 >> gpurun_out/r06rc.txt 2>&1 || { cat gpurun_out/r06rc.txt; exit 1; }; done
cat gpurun_out/r06rc.txt
