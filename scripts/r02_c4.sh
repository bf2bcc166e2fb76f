#!/bin/bash
# C4 (1M x 512, Divide + ClusterCapacityWeight planner): bench line, phase split, kernel stats
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-c4}
timeout -k 10 600 python bench.py --config c4 --steps 5 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/${tag}_bench.out 2> gpurun_out/${tag}_bench.log || { tail -20 gpurun_out/${tag}_bench.log; exit 1; }
python - gpurun_out/${tag}_bench.out <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C4", d["value"], d["ms_per_step"], d["config"]["stage_ms"])
PY
timeout -k 10 300 python scripts/phase_prof.py --config c4 --units 100000 --out gpurun_out/${tag}_phase_c4.json > /dev/null 2> gpurun_out/${tag}_phase.log || { tail -5 gpurun_out/${tag}_phase.log; exit 1; }
grep -h "lean_\|plan_" gpurun_out/${tag}_phase_c4.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -o t -- python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/${tag}_trace.log 2>&1 || { tail -5 gpurun_out/${tag}_trace.log; exit 1; }
find gpurun_out/${tag}_trace -name "*kernel_stats.csv" -exec cut -d, -f1-4 {} \;
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d gpurun_out/${tag}_sq -o sq -- python bench.py --config c4 --steps 3 --warmup 1 --no-cpu-baseline --no-extra > gpurun_out/${tag}_sq.log 2>&1 || { tail -5 gpurun_out/${tag}_sq.log; exit 1; }
python - gpurun_out/${tag}_sq <<'PY'
import csv, glob, sys
from collections import defaultdict
acc = defaultdict(lambda: defaultdict(list))
for f in glob.glob(f"{sys.argv[1]}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in acc.items():
    if "plan" in k or "wide" in k or "prep" in k:
        print(k, {c: round(sum(v) / len(v) / 1e6, 2) for c, v in sorted(d.items())})
PY
