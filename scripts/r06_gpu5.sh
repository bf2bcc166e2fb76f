#!/bin/bash
# Round 6, GPU call 5: class-sorted planner rows + persistent prep — parity (planner / C4 / group incl. the
# 8-member full C3 split, full-size C3 / C4 / C5), then A/B: planner occupancy and classes on C4, persistent
# prep on C3 and C5 (kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 1000 $T -k "c4 or c1 or c5 or rsp or fuzz or group or planner or prep" tests/test_gpu_parity.py \
  tests/test_gpu_full_configs.py tests/test_gpu_group.py tests/test_gpu_prep_wave.py tests/test_gpu_c3_full.py \
  > gpurun_out/r06cl_tests.log 2>&1 \
  || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/r06cl_tests.log | head; tail -30 gpurun_out/r06cl_tests.log; exit 1; }
tail -3 gpurun_out/r06cl_tests.log
bash scripts/ab_stats.sh r06pw c4 1000000 "base pw6 new cl6" 10 > gpurun_out/r06pw_c4.txt 2>&1 \
  || { echo "pw A/B failed"; tail -20 gpurun_out/r06pw_c4.txt; exit 1; }
cat gpurun_out/r06pw_c4.txt
bash scripts/ab_stats.sh r06prep c3 1000000 "prep0 new" 10 > gpurun_out/r06prep_c3.txt 2>&1 \
  || { echo "prep A/B failed"; tail -20 gpurun_out/r06prep_c3.txt; exit 1; }
cat gpurun_out/r06prep_c3.txt
bash scripts/ab_stats.sh r06prep5 c5 100000 "prep0 new" 10 > gpurun_out/r06prep_c5.txt 2>&1 \
  || { echo "prep5 A/B failed"; tail -20 gpurun_out/r06prep_c5.txt; exit 1; }
cat gpurun_out/r06prep_c5.txt
