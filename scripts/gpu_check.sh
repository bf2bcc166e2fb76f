#!/bin/bash
# One GPU-box session: smoke → parity tests → short bench. Stops at the first
# crash / timeout (exit code other than 0 or 1), never retries a GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "aborting after $name (rc=$rc)"; exit $rc; fi
  return 0
}
step smoke 300 python __graft_entry__.py
step pytest_gpu 1500 python -m pytest tests -m gpu -q -p pytest_timeout --timeout 600 -rf
step bench 600 python bench.py --steps 10 --warmup 2
