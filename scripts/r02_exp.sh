#!/bin/bash
# Attribution runs for the C3 wide kernel: bench stage times and SQ instruction / issue counters with the
# measurement-only KAD_WIDE_EXPERIMENT variants (bit 0: no pdqsort replay) against the product kernel.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-e}
out=gpurun_out/${tag}
mkdir -p "$out"
B="python bench.py --config c3 --steps 5 --warmup 1 --no-cpu-baseline --no-extra"
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$out/$name.out" 2> "$out/$name.log"
  local rc=$?
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$out/$name.log"; exit $rc; fi
}
step avail 120 rocprofv3 --list-avail
for e in 0 1; do
  export KAD_WIDE_EXPERIMENT=$e
  step bench_e$e 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline --no-extra
  python - "$out/bench_e$e.out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("exp", sys.argv[1], d["value"], d["ms_per_step"], d["config"]["stage_ms"])
PY
  step sq_e$e 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d "$out/sq_e$e" -o sq -- $B
done
unset KAD_WIDE_EXPERIMENT
python - "$out" <<'PY'
import csv, glob, sys
from collections import defaultdict
for e in (0, 1):
    acc = defaultdict(list)
    for f in glob.glob(f"{sys.argv[1]}/sq_e{e}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "schedule_wide_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print("exp", e, {k: round(sum(v) / len(v) / 1e6, 2) for k, v in sorted(acc.items())}, "(1e6 per dispatch)")
PY
