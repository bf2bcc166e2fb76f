#!/bin/bash
# Round-end measurement, second half: PMC passes for the given configs (scripts/profile.sh), their
# pmc_<cfg>.json copied into profiles/ (so the bench line's rooflines use counters of this code: bench.py
# checks src_hash), then the driver's default bench line and a kernel trace of it.
#   scripts/final_bench.sh TAG "c4 c5"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-fin}; cfgs=${2:-}
for cfg in $cfgs; do
  timeout -k 10 1000 bash scripts/profile.sh "$cfg" "$tag" > "gpurun_out/${tag}_prof_$cfg.log" 2>&1
  rc=$?; echo "== prof $cfg rc=$rc"; tail -n 3 "gpurun_out/${tag}_prof_$cfg.log"
  [ $rc -ne 0 ] && exit $rc
  cp "gpurun_out/prof_${cfg}_${tag}/pmc_$cfg.json" "profiles/pmc_$cfg.json" || exit 1
done
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > "gpurun_out/${tag}_bench.json" 2> "gpurun_out/${tag}_bench.log"
rc=$?; echo "== bench rc=$rc"; tail -n 3 "gpurun_out/${tag}_bench.log"
[ $rc -ne 0 ] && exit $rc
python - "$tag" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/{sys.argv[1]}_bench.json").read().strip().splitlines()[-1])
def show(d, n):
    r = d.get("roofline") or {}
    print(n, "%.4g" % d["value"], round(d["ms_per_step"], 4), r.get("bound"), r.get("frac"), r.get("pmc"),
          "parity_mismatches", d.get("parity_mismatches", (d.get("parity") or {}).get("mismatches")))
show(d, "c3")
for k, v in d.get("extra", {}).items():
    show(v, k)
PY
exit 0
