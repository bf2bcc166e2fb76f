#!/bin/bash
# Round 6, GPU call 3: the half-wave pair planner — planner parity (golden x 3 paths, random rows, C4 full
# size, fuzz / C1 Divide units), then the C4 kernel-stat A/B (base = the round's previous commit, new, pw6).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 900 $T -k "planner or plan_rows or c4 or c1 or fuzz or rsp or group" tests/test_gpu_parity.py \
  tests/test_gpu_full_configs.py tests/test_gpu_group.py > gpurun_out/r06p_tests.log 2>&1 \
  || { echo "planner tests failed"; grep -E "FAIL|Error|assert" gpurun_out/r06p_tests.log | head -20; tail -30 gpurun_out/r06p_tests.log; exit 1; }
tail -3 gpurun_out/r06p_tests.log
bash scripts/ab_stats.sh r06pair c4 1000000 "base new pw6 new" 10 > gpurun_out/r06pair_c4.txt 2>&1 \
  || { echo "pair A/B failed"; tail -20 gpurun_out/r06pair_c4.txt; exit 1; }
cat gpurun_out/r06pair_c4.txt
bash scripts/ab_stats.sh r06ff c3 1000000 "new ff1k new" 10 > gpurun_out/r06ff_c3.txt 2>&1 \
  || { echo "fence A/B failed"; tail -20 gpurun_out/r06ff_c3.txt; exit 1; }
cat gpurun_out/r06ff_c3.txt
