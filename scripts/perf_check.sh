#!/bin/bash
# GPU parity suite, then short bench lines for C2 (default) and C5 (subset); stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests -m gpu -x -q --timeout 300 > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for cfg in ${PERF_CONFIGS:-c2 c5}; do
  extra=""
  [ "$cfg" = c5 ] && extra="--units 10000"
  [ "$cfg" = c3 ] && extra="--units 250000"
  [ "$cfg" = c4 ] && extra="--units 200000"
  timeout -k 10 300 python bench.py --config $cfg $extra --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/perf_$cfg.json 2> gpurun_out/perf_$cfg.log || { tail -5 gpurun_out/perf_$cfg.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/perf_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', 'value=%.4g' % d['value'], 'ms=%.4f' % d['ms_per_step'], 'frac=%.3f' % d['roofline']['frac'], d['config']['kernel_ms'])"
done
