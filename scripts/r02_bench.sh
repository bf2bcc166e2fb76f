#!/bin/bash
# Bench iteration on the GPU box: default bench line (C3 1M x 1k + embedded C2), a 2-rank gloo rehearsal of
# the multi-GPU path on one GPU, then the C3 PMC profile that bench.py's roofline reads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-b}
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_$name.json" 2> "gpurun_out/${tag}_$name.log"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 1500 "gpurun_out/${tag}_$name.json"; echo
  if [ $rc -ne 0 ]; then tail -n 15 "gpurun_out/${tag}_$name.log"; exit $rc; fi
}
step bench 600 python bench.py --steps 20 --warmup 5
step rehearse2 600 python bench.py --gpus 2 --backend gloo --share-gpu --units 200000 --steps 10 --warmup 2 --no-cpu-baseline
if [ -n "$PROFILE" ]; then
  UNITS=1000000 bash scripts/profile.sh c3 "$tag" > gpurun_out/${tag}_profile.log 2>&1 || { tail -20 gpurun_out/${tag}_profile.log; exit 1; }
  tail -30 gpurun_out/${tag}_profile.log
fi
