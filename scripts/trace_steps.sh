#!/bin/bash
# Kernel-trace timelines of C3 pipeline passes at the 8-GPU shard (125k units) and at 1M (scripts/timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=${1:-r05}
for W in 125000 1000000; do
  out=gpurun_out/trace_${tag}_$W
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$out" -o run -- \
    python bench.py --config ${CFG:-c3} --units $W --steps 30 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e \
    > "$out.log" 2>&1 || { echo "trace $W failed"; tail -5 "$out.log"; exit 1; }
  python scripts/timeline.py "$out" --last 25 --skip-last 10 --json "$out.json" | head -60
done
