#!/bin/bash
# Round 6 (session 2) final records, part 2: PMC profiles of c2 c3r c5, every profiled config's pmc_<cfg>.json
# into profiles/ (bench.py checks their src_hash), then the default bench line
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for cfg in ${CFGS:-c2 c3r c5}; do
  timeout -k 10 500 bash scripts/profile.sh "$cfg" s2f > "gpurun_out/s2f_prof_$cfg.log" 2>&1
  rc=$?; echo "== prof $cfg rc=$rc"; tail -n 2 "gpurun_out/s2f_prof_$cfg.log"
  [ $rc -ne 0 ] && exit $rc
done
for cfg in c2 c3 c3r c3p c4 c5; do
  [ -f "gpurun_out/prof_${cfg}_s2f/pmc_$cfg.json" ] && cp "gpurun_out/prof_${cfg}_s2f/pmc_$cfg.json" "profiles/pmc_$cfg.json"
done
timeout -k 10 900 python bench.py --steps 20 --warmup 3 > gpurun_out/s2f_bench.json 2> gpurun_out/s2f_bench.log
rc=$?; echo "== bench rc=$rc"; tail -n 2 gpurun_out/s2f_bench.log
exit $rc
