#!/bin/bash
# round-5 head (72348d9) vs the working tree on every bench config, kernel stats per library (same box)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/r06reg.txt
for cu in "c2 100000" "c3 1000000" "c3 125000" "c4 1000000" "c5 100000"; do
  set -- $cu
  echo "## $1 $2 units" >> gpurun_out/r06reg.txt
  bash scripts/ab_stats.sh r06reg_$1_$2 $1 $2 "${LIBS:-r5 new}" 10 >> gpurun_out/r06reg.txt 2>&1 || { cat gpurun_out/r06reg.txt; exit 1; }
done
cat gpurun_out/r06reg.txt
