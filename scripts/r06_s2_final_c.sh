#!/bin/bash
# Round 6 (session 2) final records after the pair-planner grid cap: GPU suite and smoke, then PMC profiles
# of the configs in CFGS (scripts/profile.sh), their pmc_<cfg>.json into profiles/, then (BENCH=1) the bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$SUITE" ]; then
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/s2g_smoke.log 2>&1 || { tail -5 gpurun_out/s2g_smoke.log; exit 1; }
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/s2g_pytest_gpu.log 2>&1
  rc=$?; tail -1 gpurun_out/s2g_pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for cfg in $CFGS; do
  timeout -k 10 500 bash scripts/profile.sh "$cfg" s2g > "gpurun_out/s2g_prof_$cfg.log" 2>&1
  rc=$?; echo "== prof $cfg rc=$rc"; [ $rc -ne 0 ] && { tail -5 "gpurun_out/s2g_prof_$cfg.log"; exit $rc; }
  cp "gpurun_out/prof_${cfg}_s2g/pmc_$cfg.json" "profiles/pmc_$cfg.json"
done
if [ -n "$BENCH" ]; then
  timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/s2g_bench.json 2> gpurun_out/s2g_bench.log
  rc=$?; echo "== bench rc=$rc"; tail -n 2 gpurun_out/s2g_bench.log; exit $rc
fi
exit 0
