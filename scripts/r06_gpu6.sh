#!/bin/bash
# Round 6, GPU call 6: zero-request score column (wide kernel) — parity (relaxed fuzz, c3p / c3 / c3r full size,
# rows inline, planner), A/B c3p and c3 (new vs nozs), kernel stats of C4 and C5 on the current build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 1000 $T -k "relaxed or clean or c3 or planner or plan_rows or rows or c4" tests/test_gpu_parity.py \
  tests/test_gpu_c3_full.py tests/test_gpu_rows_inline.py tests/test_gpu_full_configs.py > gpurun_out/r06zs_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r06zs_tests.log | head; tail -30 gpurun_out/r06zs_tests.log; exit 1; }
tail -3 gpurun_out/r06zs_tests.log
bash scripts/ab_stats.sh r06zsp c3p 1000000 "nozs new nozs new" 10 > gpurun_out/r06zs_c3p.txt 2>&1 \
  || { echo "zs A/B failed"; tail -20 gpurun_out/r06zs_c3p.txt; exit 1; }
cat gpurun_out/r06zs_c3p.txt
bash scripts/ab_stats.sh r06zs3 c3 1000000 "nozs new" 10 > gpurun_out/r06zs_c3.txt 2>&1 \
  || { echo "zs3 A/B failed"; tail -20 gpurun_out/r06zs_c3.txt; exit 1; }
cat gpurun_out/r06zs_c3.txt
bash scripts/ab_stats.sh r06k4 c4 1000000 "new" 10 > gpurun_out/r06k_c4.txt 2>&1 && cat gpurun_out/r06k_c4.txt
bash scripts/ab_stats.sh r06k5 c5 100000 "new" 10 > gpurun_out/r06k_c5.txt 2>&1 && cat gpurun_out/r06k_c5.txt
