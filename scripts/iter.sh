#!/bin/bash
# One kernel-iteration session on the GPU box: parity tests of the touched paths, phase profiles, a short
# bench line per config. Every step has its own time limit; the first failure ends the session.
#   scripts/iter.sh TAG "pytest -k expr" "configs for phase_prof" "configs for bench"
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-it}; sel=${2:-}; phases=${3:-c3}; benches=${4:-c3}; trace=${5:-}
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$sel" \
    > gpurun_out/${tag}_pytest.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
  tail -2 gpurun_out/${tag}_pytest.log
fi
for cfg in $phases; do
  u=""; [ "$cfg" = c3 ] && u="--units 200000"
  timeout -k 10 300 python scripts/phase_prof.py --config $cfg $u --out gpurun_out/${tag}_phase_$cfg.json \
    > gpurun_out/${tag}_phase_$cfg.log 2>&1 || { echo "phase $cfg failed"; tail -20 gpurun_out/${tag}_phase_$cfg.log; exit 1; }
done
for cfg in $benches; do
  timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep \
    > gpurun_out/${tag}_bench_$cfg.json 2> gpurun_out/${tag}_bench_$cfg.log || { echo "bench $cfg failed"; tail -20 gpurun_out/${tag}_bench_$cfg.log; exit 1; }
  python - "$tag" "$cfg" <<'PY'
import json, sys
t, c = sys.argv[1:3]
d = json.loads(open(f"gpurun_out/{t}_bench_{c}.json").read().strip().splitlines()[-1])
st = d["config"]["stage_ms"]
print(c, "value %.4g ms %.4f" % (d["value"], d["ms_per_step"]), {k: round(v, 4) for k, v in st.items()},
      "e2e %.3g" % d["end_to_end"]["decisions_per_s"] if d.get("end_to_end") else "")
PY
done
# kernel trace of one config at a unit count ("c3:125000")
if [ -n "$trace" ]; then
  cfg=${trace%%:*}; units=${trace#*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_trace -o run -- \
    python bench.py --config $cfg --units $units --steps 10 --warmup 2 --no-cpu-baseline --no-extra --no-sweep \
    > gpurun_out/${tag}_trace.log 2>&1 || { echo "trace failed"; tail -20 gpurun_out/${tag}_trace.log; exit 1; }
  find gpurun_out/${tag}_trace -name "*kernel_stats.csv" -exec cat {} \; | cut -d, -f1-5 | head -14
fi
exit 0
