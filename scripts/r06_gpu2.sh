#!/bin/bash
# Round 6, GPU call 2: C4 wide-kernel A/B of the compaction variants (kernel stats), the default bench
# (C3 + extras incl. c3p), group-mode bench tests.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_stats.sh r06c8 c4 1000000 "b2 new c8p c16 new" 10 > gpurun_out/r06c8_c4.txt 2>&1 \
  || { echo "c8 A/B failed"; tail -20 gpurun_out/r06c8_c4.txt; exit 1; }
cat gpurun_out/r06c8_c4.txt
timeout -k 10 600 python bench.py > gpurun_out/r06_bench1.out 2> gpurun_out/r06_bench1.err \
  || { echo "bench failed"; tail -20 gpurun_out/r06_bench1.err; exit 1; }
tail -c 2500 gpurun_out/r06_bench1.out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_dist.py > gpurun_out/r06_benchdist.log 2>&1 \
  || { echo "bench dist tests failed"; tail -30 gpurun_out/r06_benchdist.log; exit 1; }
tail -3 gpurun_out/r06_benchdist.log
