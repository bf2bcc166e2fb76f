#!/bin/bash
# round-end: smoke, then the default bench line (planner stage now counts plan_pair_kernel)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06h_smoke.log 2>&1
rc=$?; tail -3 gpurun_out/r06h_smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/r06h_bench.json 2> gpurun_out/r06h_bench.log
rc=$?; tail -3 gpurun_out/r06h_bench.log; [ $rc -ne 0 ] && exit $rc
tail -c 600 gpurun_out/r06h_bench.json
