#!/bin/bash
# C5 iteration: parity tests touching the changed paths, then the C5 full-size bench under a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-c5i}
K=${PYTEST_K:-"taint or c5 or fuzz or large or c3 or c2_full or extreme or tie"}
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -m gpu -x -q --timeout 300 \
  --timeout-method thread -k "$K" > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -4 gpurun_out/${tag}_pytest.log; echo "== pytest rc=$rc"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_pytest.log | head -30; exit $rc; }
out=gpurun_out/prof_c5_${tag}
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- \
  python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/trace.log
rc=$?; echo "== trace rc=$rc"
[ $rc -ne 0 ] && { tail -20 $out/trace.log; exit $rc; }
python -c "import json,sys; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['config']['stage_ms'])"
find $out -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \; | head -12
