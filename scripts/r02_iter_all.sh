#!/bin/bash
# Iteration: full GPU suite, C5 full-size bench under a kernel trace, default bench line (C3 + C2) w/o CPU baseline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-it}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/${tag}_pytest.log; echo "== pytest rc=$rc"
[ $rc -ne 0 ] && { grep -E "Error|assert|FAIL" gpurun_out/${tag}_pytest.log | head -30; exit $rc; }
out=gpurun_out/prof_c5_${tag}
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- \
  python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $out/bench.json 2> $out/trace.log
rc=$?; echo "== c5 trace rc=$rc"
[ $rc -ne 0 ] && { tail -20 $out/trace.log; exit $rc; }
python -c "import json,sys; d=json.load(open('$out/bench.json')); print(d['value'], d['ms_per_step'], d['config']['stage_ms'])"
find $out -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \; | head -12
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log
rc=$?; echo "== bench rc=$rc"
[ $rc -ne 0 ] && { tail -20 gpurun_out/${tag}_bench.log; exit $rc; }
python -c "import json; d=json.load(open('gpurun_out/${tag}_bench.json')); print('c3', d['value'], d['ms_per_step'], d['config']['stage_ms']); e=d['extra']['c2']; print('c2', e['value'], e['ms_per_step'], e['config']['stage_ms'])"
