#!/bin/bash
# One GPU-box session: smoke → parity tests → short bench → rocprofv3 kernel trace.
# Stops at the first crash / timeout (exit code other than 0 or 1); never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 8 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && { [ $rc -ne 1 ] || [ "$name" = smoke ] || grep -q "illegal memory\|HSA_STATUS_ERROR\|hipError" "gpurun_out/$name.log"; }; then
    echo "aborting after $name (rc=$rc)"; exit $rc; fi
  return 0
}
what=${1:-all}
if [ "$what" = all ] || [ "$what" = test ]; then
  step smoke 300 python __graft_entry__.py
  step pytest_gpu 900 python -m pytest tests -m gpu -x -q --timeout 300 -rf
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench 600 python bench.py --steps 20 --warmup 3
fi
if [ "$what" = all ] || [ "$what" = prof ]; then
  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
      python bench.py --steps 10 --warmup 2 --no-cpu-baseline
  find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | head -20
fi
