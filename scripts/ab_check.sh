#!/bin/bash
# Parity of the kernel variants on the GPU, then A/B timings with rocprofv3 kernel stats.
# Usage: scripts/ab_check.sh <tag> [test-selection]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-ab}
sel=${2:-"clean or c3 or c2_full or c5_clusters or config_shaped or abi"}
step() {  # name, timeout, cmd...
  local name=$1 t=$2; shift 2
  echo "== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/${tag}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "gpurun_out/${tag}_$name.log"
  if [ $rc -ne 0 ]; then echo "aborting after $name (rc=$rc)"; exit $rc; fi
}
step wide_tests 600 env KAD_WIDE_MIN_NCH=1 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_abi.py -m gpu -x -q --timeout 300 -k "$sel"
step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300
for cfg in ${CONFIGS:-c3 c2}; do
  units=""; [ "$cfg" = c3 ] && units="--units ${C3_UNITS:-250000}"
  step trace_$cfg 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof_$cfg -o run -- \
      python bench.py --config $cfg $units --steps 10 --warmup 2 --no-cpu-baseline
  if [ "$cfg" = c2 ]; then
    step trace_c2_wide 600 env KAD_WIDE_MIN_NCH=1 rocprofv3 --kernel-trace --stats --output-format csv \
        -d gpurun_out/${tag}_prof_c2_wide -o run -- python bench.py --config c2 --steps 10 --warmup 2 --no-cpu-baseline
  fi
done
for f in gpurun_out/${tag}_prof_*/run_kernel_stats.csv; do echo "== $f"; cut -d, -f1-4 "$f" | head -8; done
