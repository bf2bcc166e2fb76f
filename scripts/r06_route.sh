#!/bin/bash
# Round 6 (session 2): early routing threshold (KAD_ROUTE_MIN of a -DKAD_TUNING build: units with more feasible
# (KAD_ROUTE_MIN exists only with profiles/r06/route_min.patch applied; the sources do not keep it)
# clusters than this go to the row body in the wide kernel's opening phase) on C3's 125k shard and 1M.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for u in 125000 1000000; do
  timeout -k 10 300 python -u scripts/step_ab.py --config c3 --units $u --rounds ${ROUNDS:-3} \
    --variants "base;KAD_ROUTE_MIN=448;KAD_ROUTE_MIN=384;KAD_ROUTE_MIN=320;KAD_ROUTE_MIN=256" > gpurun_out/route_$u.json 2> gpurun_out/route_$u.err \
    || { echo "step_ab $u failed"; tail -20 gpurun_out/route_$u.err; exit 1; }
  cat gpurun_out/route_$u.json
done
