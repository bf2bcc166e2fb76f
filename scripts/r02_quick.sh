#!/bin/bash
# Quick GPU iteration: parity of the kernel variants (forced wide kernel + full suite), the default bench
# line, phase split of the C3 wide kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-q}
run() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_$name.out" 2> "gpurun_out/${tag}_$name.log"
  local rc=$?
  echo "== $name rc=$rc"; tail -c 600 "gpurun_out/${tag}_$name.out"; echo
  if [ $rc -ne 0 ]; then tail -n 20 "gpurun_out/${tag}_$name.log"; exit $rc; fi
}
run wide_tests 600 env KAD_WIDE_MIN_NCH=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -m gpu -x -q --timeout 300 -k "clean or c3 or c2_full or c5_clusters or config_shaped or abi or fuzz"
[ -n "$FULL" ] && run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300
run bench 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
python - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}_bench.out").read().strip().splitlines()[-1])
print("C3", d["value"], d["ms_per_step"], d["config"]["stage_ms"])
print("C2", d["extra"]["c2"]["value"], d["extra"]["c2"]["ms_per_step"], d["extra"]["c2"]["config"]["stage_ms"])
PY
run phase 300 python scripts/phase_prof.py --config c3 --units 100000 --out gpurun_out/${tag}_phase_c3.json
grep -h "lean_[ABDE]\|straddle_cy\|replay_" gpurun_out/${tag}_phase_c3.json
