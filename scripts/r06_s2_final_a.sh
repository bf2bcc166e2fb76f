#!/bin/bash
# Round 6 (session 2) final records, part 1: GPU suite, then PMC profiles of c4 c3 c3p (scripts/profile.sh)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s2f_pytest_gpu.log 2>&1
rc=$?; tail -1 gpurun_out/s2f_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for cfg in ${CFGS:-c4 c3 c3p}; do
  timeout -k 10 500 bash scripts/profile.sh "$cfg" s2f > "gpurun_out/s2f_prof_$cfg.log" 2>&1
  rc=$?; echo "== prof $cfg rc=$rc"; tail -n 2 "gpurun_out/s2f_prof_$cfg.log"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
