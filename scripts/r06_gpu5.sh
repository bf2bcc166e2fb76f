#!/bin/bash
# Round 6, GPU call 5: pair planner occupancy A/B on C4 (kernel stats).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_stats.sh r06pw c4 1000000 "base pw4 pw5 pw6 pw7 new" 10 > gpurun_out/r06pw_c4.txt 2>&1 \
  || { echo "pw A/B failed"; tail -20 gpurun_out/r06pw_c4.txt; exit 1; }
cat gpurun_out/r06pw_c4.txt
