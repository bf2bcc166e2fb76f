#!/bin/bash
# Kernel iteration on the GPU box: parity subset, C3 phase profile at one shard size, bench lines.
#   scripts/iter2.sh TAG "pytest -k expr" "c3:125000 c3:1000000 c2" [phase-units]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-it}; sel=${2:-}; benches=${3:-c3}; punits=${4:-}
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" \
    > gpurun_out/${tag}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
  tail -2 gpurun_out/${tag}_pytest.log
fi
if [ -n "$punits" ]; then
  for pu in $punits; do
    cfg=${pu%%:*}; u=${pu#*:}
    timeout -k 10 300 python scripts/phase_prof.py --config $cfg --units $u --out gpurun_out/${tag}_phase_${cfg}_$u.json \
      > gpurun_out/${tag}_phase_${cfg}_$u.log 2>&1 || { echo "phase failed"; tail -20 gpurun_out/${tag}_phase_${cfg}_$u.log; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/${tag}_phase_${cfg}_$u.json')); print('$pu', {k:v for k,v in d.items() if v and not isinstance(v,list)})"
  done
fi
for cu in $benches; do
  cfg=${cu%%:*}; u=""; [ "$cu" != "$cfg" ] && u="--units ${cu#*:}"
  timeout -k 10 300 python bench.py --config $cfg $u --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e \
    > gpurun_out/${tag}_bench_$cfg${cu#$cfg}.json 2> gpurun_out/${tag}_bench.log || { echo "bench $cu failed"; tail -20 gpurun_out/${tag}_bench.log; exit 1; }
  python - "gpurun_out/${tag}_bench_$cfg${cu#$cfg}.json" "$cu" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
st = d["config"]["stage_ms"]
print(sys.argv[2], "value %.4g ms %.4f" % (d["value"], d["ms_per_step"]), {k: round(v, 4) for k, v in st.items()})
PY
done
exit 0
