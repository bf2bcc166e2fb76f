#!/bin/bash
# Round 6, GPU call 7: interim round measurement — the GPU suite, the default bench line (C3 + extras + sweep),
# and a group-mode C3 line with 8 members on the box's GPU.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06i_suite.log 2>&1 \
  || { echo "suite failed"; tail -30 gpurun_out/r06i_suite.log; exit 1; }
tail -2 gpurun_out/r06i_suite.log
timeout -k 10 600 python bench.py > gpurun_out/r06i_bench.out 2> gpurun_out/r06i_bench.err \
  || { echo "bench failed"; tail -20 gpurun_out/r06i_bench.err; exit 1; }
tail -c 3000 gpurun_out/r06i_bench.out
timeout -k 10 300 python bench.py --gpus 8 --group-devices 0,0,0,0,0,0,0,0 --steps 10 > gpurun_out/r06i_group8.out 2> gpurun_out/r06i_group8.err \
  || { echo "group bench failed"; tail -20 gpurun_out/r06i_group8.err; exit 1; }
tail -c 1500 gpurun_out/r06i_group8.out
