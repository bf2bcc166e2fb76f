#!/bin/bash
# C2 A/B: lean kernel (default) vs the wide kernel (KAD_WIDE_MIN_NCH=1)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-ab}
for v in default wide; do
  if [ $v = wide ]; then export KAD_WIDE_MIN_NCH=1; fi
  timeout -k 10 300 python bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline --no-extra > gpurun_out/${tag}_$v.out 2> gpurun_out/${tag}_$v.log || exit $?
  python - gpurun_out/${tag}_$v.out $v <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], d["value"], d["ms_per_step"], d["config"]["stage_ms"])
PY
done
