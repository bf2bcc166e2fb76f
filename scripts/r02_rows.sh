#!/bin/bash
# Row-kernel iteration: parity on the paths it serves, its phase split (profiling build) and the C5 bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-rw}
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -m gpu -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${tag}_pytest.log; echo "== pytest rc=$rc"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_pytest.log | head -30; exit $rc; }
timeout -k 10 300 python scripts/phase_prof.py --config c5 --units 100000 --out gpurun_out/${tag}_phase_c5.json \
  > /dev/null 2> gpurun_out/${tag}_phase.log || { tail gpurun_out/${tag}_phase.log; exit 1; }
grep row_ gpurun_out/${tag}_phase_c5.json
timeout -k 10 300 python bench.py --config c5 --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/${tag}_c5.json \
  2> gpurun_out/${tag}_c5.log || { tail gpurun_out/${tag}_c5.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_c5.json')); print(d['value'], d['ms_per_step'], d['config']['stage_ms'])"
