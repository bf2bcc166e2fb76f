#!/bin/bash
# C5 (100k x 10k) at full size: bench line, then a rocprofv3 kernel trace of the same workload.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
tag=${1:-c5}
timeout -k 10 600 python bench.py --config c5 --steps 10 --warmup 2 --cpu-seconds 10 \
  > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log
rc=$?; echo "== bench rc=$rc"; tail -c 3000 gpurun_out/${tag}_bench.json; echo; tail -5 gpurun_out/${tag}_bench.log
[ $rc -ne 0 ] && exit $rc
out=gpurun_out/prof_c5_${tag}
mkdir -p $out
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o trace -- \
  python bench.py --config c5 --steps 5 --warmup 1 --no-cpu-baseline > $out/trace.log 2>&1
rc=$?; echo "== trace rc=$rc"
[ $rc -ne 0 ] && { tail -20 $out/trace.log; exit $rc; }
find $out -name '*kernel_stats.csv' -exec cut -d, -f1-5 {} \; | head -20
