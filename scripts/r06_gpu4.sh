#!/bin/bash
# Round 6, GPU call 4: group tests after the conftest HIP-init fix; A/B: pair planner (C4), prep fences and the
# compaction's dummy stride (C3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 300 --timeout-method thread"
timeout -k 10 600 $T -m gpu tests/test_gpu_abi.py tests/test_gpu_group.py > gpurun_out/r06g_tests.log 2>&1 \
  || { echo "group tests failed"; tail -30 gpurun_out/r06g_tests.log; exit 1; }
tail -3 gpurun_out/r06g_tests.log
bash scripts/ab_stats.sh r06pair c4 1000000 "base new pw6 new" 10 > gpurun_out/r06pair_c4.txt 2>&1 \
  || { echo "pair A/B failed"; tail -20 gpurun_out/r06pair_c4.txt; exit 1; }
cat gpurun_out/r06pair_c4.txt
bash scripts/ab_stats.sh r06ff c3 1000000 "new ff1k pad new" 10 > gpurun_out/r06ff_c3.txt 2>&1 \
  || { echo "fence A/B failed"; tail -20 gpurun_out/r06ff_c3.txt; exit 1; }
cat gpurun_out/r06ff_c3.txt
