#!/bin/bash
# Round-end measurement: GPU suite, default bench line (C3 + C2), C4 / C5 / C1 lines, two-rank rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fin}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_pytest.log; echo "== pytest rc=$rc"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_pytest.log | head -30; exit $rc; }
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_$name.json" 2> "gpurun_out/${tag}_$name.log"
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 15 "gpurun_out/${tag}_$name.log"; exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/${tag}_$name.json').read().strip().splitlines()[-1]); print(d['config']['workload'][:40], d['value'], d['ms_per_step'], d['config']['stage_ms'])"
}
step bench 600 python bench.py --steps 20 --warmup 5
step c4 600 python bench.py --config c4 --steps 10 --warmup 2 --cpu-seconds 10
step c5 600 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10
step c1 300 python bench.py --config c1 --steps 20 --warmup 5 --cpu-seconds 5
step rehearse2 600 python bench.py --gpus 2 --backend gloo --share-gpu --units 200000 --steps 10 --warmup 2 --no-cpu-baseline
