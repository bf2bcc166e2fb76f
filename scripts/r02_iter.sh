#!/bin/bash
# One iteration on the GPU box: parity (forced wide kernel + full suite), kernel traces, phase split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-it}
bash scripts/ab_check.sh "$tag" || exit $?
timeout -k 10 300 python scripts/phase_prof.py --config c3 --units 100000 --out gpurun_out/${tag}_phase_c3.json > gpurun_out/${tag}_phase.log 2>&1 || exit $?
KAD_WIDE_MIN_NCH=1 timeout -k 10 300 python scripts/phase_prof.py --config c2 --out gpurun_out/${tag}_phase_c2_wide.json >> gpurun_out/${tag}_phase.log 2>&1 || exit $?
timeout -k 10 300 python scripts/phase_prof.py --config c2 --out gpurun_out/${tag}_phase_c2_lean.json >> gpurun_out/${tag}_phase.log 2>&1 || exit $?
grep -h "lean_[ABDE]\|straddle_cy" gpurun_out/${tag}_phase_*.json
