#!/bin/bash
# Round 6, first GPU call: the new GPU tests (routed units at the 125k shard, relaxed snapshots, c3p full
# size, group member / concurrency), the C4 wide-kernel bisect (kernel stats per revision), the GPU suite.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_rows_inline.py tests/test_gpu_group.py \
  "tests/test_gpu_parity.py::test_fuzz_relaxed_snapshot_gpu_equals_c_oracle" \
  "tests/test_gpu_c3_full.py::test_c3p_full_equals_c_oracle" > gpurun_out/r06a_new.log 2>&1 \
  || { echo "new tests failed"; tail -30 gpurun_out/r06a_new.log; exit 1; }
tail -3 gpurun_out/r06a_new.log
bash scripts/ab_stats.sh r06bis c4 1000000 "r4 b1 b2 b3 b4 new" 10 > gpurun_out/r06bis_c4.txt 2>&1 \
  || { echo "bisect failed"; tail -20 gpurun_out/r06bis_c4.txt; exit 1; }
cat gpurun_out/r06bis_c4.txt
timeout -k 10 900 $T -m gpu tests > gpurun_out/r06a_suite.log 2>&1 || { echo "suite failed"; tail -30 gpurun_out/r06a_suite.log; exit 1; }
tail -3 gpurun_out/r06a_suite.log
