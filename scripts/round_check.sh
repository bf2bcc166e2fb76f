#!/bin/bash
# One GPU-box session: smoke -> GPU parity suite -> default bench line (C3 + C2/C4/C5 extras + shard sweep)
# -> rocprofv3 kernel trace + PMC passes per config (scripts/profile.sh).
# Every GPU step runs under its own time limit; the first crash / timeout ends the session (no retries).
#   scripts/round_check.sh [test] [bench] [prof:c3,c2,...] [tag=NAME]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=run
for a in "$@"; do case $a in tag=*) tag=${a#tag=};; esac; done
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ]; then echo "aborting after $name (rc=$rc)"; exit $rc; fi
}
for a in "$@"; do
  case $a in
    test)
      step smoke 300 python __graft_entry__.py
      step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf ;;
    bench)
      timeout -k 10 900 python bench.py --steps 20 --warmup 3 > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.log"
      rc=$?; echo "== bench rc=$rc"; tail -n 3 "gpurun_out/${tag}_bench.log"
      [ $rc -ne 0 ] && exit $rc ;;
    prof:*)
      for cfg in $(echo "${a#prof:}" | tr , ' '); do
        timeout -k 10 1000 bash scripts/profile.sh "$cfg" "$tag" > "gpurun_out/${tag}_prof_$cfg.log" 2>&1
        rc=$?; echo "== prof $cfg rc=$rc"; tail -n 3 "gpurun_out/${tag}_prof_$cfg.log"
        [ $rc -ne 0 ] && exit $rc
      done ;;
  esac
done
exit 0
