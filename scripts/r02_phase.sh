#!/bin/bash
# phase splits (profiling build) of the C2 lean kernel and the C3 wide kernel
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-ph}
for c in c2 c3; do
  u=100000
  timeout -k 10 300 python scripts/phase_prof.py --config $c --units $u --out gpurun_out/${tag}_phase_$c.json > /dev/null 2> gpurun_out/${tag}_phase_$c.log || { tail -5 gpurun_out/${tag}_phase_$c.log; exit 1; }
  echo "== $c"; grep -h "lean_\|replay_\|plan_rows" gpurun_out/${tag}_phase_$c.json
done
