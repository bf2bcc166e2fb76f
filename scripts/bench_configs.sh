#!/bin/bash
# One bench line per BASELINE.json config on one GPU (bounded unit counts for the big configs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name, timeout, args...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" python bench.py "$@" > "gpurun_out/bench_$name.json" 2> "gpurun_out/bench_$name.log"
  local rc=$?; echo "== $name rc=$rc"; tail -c 600 "gpurun_out/bench_$name.json"; echo
  if [ $rc -ne 0 ]; then tail -5 "gpurun_out/bench_$name.log"; exit $rc; fi
}
run c1 300 --config c1 --steps 20 --warmup 3 --cpu-seconds 5
run c3 600 --config c3 --units 250000 --steps 10 --warmup 2 --no-cpu-baseline
run c4 600 --config c4 --units 200000 --steps 10 --warmup 2 --no-cpu-baseline
run c5 600 --config c5 --units 10000 --steps 5 --warmup 1 --no-cpu-baseline
