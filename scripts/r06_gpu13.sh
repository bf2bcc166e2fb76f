#!/bin/bash
# prep program-word padding: parity (prep paths), then C3 / C3p / C4 / C2 kernel A/B vs the unpadded build
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "fuzz or golden_filter or requirement or label_free or c3_clusters or c4_subset or zero_request" > gpurun_out/r06pp_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r06pp_pytest.log; [ $rc -ne 0 ] && exit $rc
: > gpurun_out/r06pp.txt
for o in "pp0 new" "new pp0"; do
  for cu in "c3 1000000" "c4 1000000" "c2 100000"; do
    set -- $cu
    bash scripts/ab_stats.sh r06pp_$1_${o// /_} $1 $2 "$o" 10 >> gpurun_out/r06pp.txt 2>&1 || { cat gpurun_out/r06pp.txt; exit 1; }
  done
done
grep -o '^[a-z0-9]* .*prep_kernel=[0-9.]*' gpurun_out/r06pp.txt | sed 's/schedule.*prep_kernel/prep_kernel/;s/plan_pair.*prep_kernel/prep_kernel/'
