#!/bin/bash
# Round 6 (session 2): replay issue priority (replay_prio) on vs off (the KAD_*_EXPERIMENT bit 4 of a -DKAD_TUNING
# (the knobs exist only with profiles/r06/replay_priority.patch applied; the sources do not keep it)
# build turns it off), alternating in one process per config; results asserted equal by step_ab.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # tag config units variants
  timeout -k 10 300 python -u scripts/step_ab.py --config $2 --units $3 --rounds ${ROUNDS:-4} --variants "$4" \
    > gpurun_out/prio2_$1.json 2> gpurun_out/prio2_$1.err || { echo "step_ab $1 failed"; tail -20 gpurun_out/prio2_$1.err; exit 1; }
  cat gpurun_out/prio2_$1.json
}
run c3_125k c3 125000 "base;KAD_WIDE_EXPERIMENT=16" &&
run c3 c3 0 "base;KAD_WIDE_EXPERIMENT=16" &&
run c2 c2 0 "base;KAD_LEAN_EXPERIMENT=16" &&
run c5 c5 0 "base;KAD_ROW_EXPERIMENT=16;KAD_LEAN_EXPERIMENT=16;KAD_ROW_EXPERIMENT=16,KAD_LEAN_EXPERIMENT=16" &&
run c4 c4 0 "base;KAD_WIDE_EXPERIMENT=16"
