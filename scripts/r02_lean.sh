#!/bin/bash
# lean kernel iteration: kernel-variant parity, bench lines, C2 SQ counters (wave lifetime)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=${1:-ln}
bash scripts/r02_quick.sh "$tag" || exit $?
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 -k "c2_full or c1_full or c4_subset or fuzz" > gpurun_out/${tag}_lean_tests.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_lean_tests.log; [ $rc -ne 0 ] && exit $rc
bash scripts/profile.sh c2 "$tag" > /dev/null || exit $?
python - gpurun_out/prof_c2_${tag}/pmc_c2.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["main_kernel"]
life = d["SQ_WAVE_CYCLES"] * 4 / d["SQ_WAVES"]
print(d["name"], "avg_ns", d["avg_ns"], "wave lifetime frac", life / (d["avg_ns"] * 2.4))
PY
