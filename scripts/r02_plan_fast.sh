#!/bin/bash
# planner parity + the C4 bench line only
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-pf}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "planner or rsp or c4 or divide or plan_rows or fuzz" > gpurun_out/${tag}_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_tests.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/${tag}_bench.out 2> gpurun_out/${tag}_bench.log || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
python - gpurun_out/${tag}_bench.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C4", d["value"], d["ms_per_step"], d["config"]["stage_ms"])
PY
