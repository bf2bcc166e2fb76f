#!/bin/bash
# Round 6 (session 2): where C3's prep_kernel time goes — KAD_PREP_EXPERIMENT bits of a -DKAD_TUNING build
# (results differ: 1 no ClusterAffinity, 2 no fit rows, 4 no placement / current clusters, 8 no folded taint / API)
# (KAD_PREP_EXPERIMENT existed only for this measurement; the sources do not keep it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/step_ab.py --config ${CFG:-c3} --units ${UNITS:-0} --rounds 2 --stages \
  --variants "${VARIANTS:-base;EXP=1,KAD_PREP_EXPERIMENT=1;EXP=1,KAD_PREP_EXPERIMENT=2;EXP=1,KAD_PREP_EXPERIMENT=4;EXP=1,KAD_PREP_EXPERIMENT=8;EXP=1,KAD_PREP_EXPERIMENT=15}" \
  > gpurun_out/prepexp_${CFG:-c3}.json 2> gpurun_out/prepexp_${CFG:-c3}.err || { tail -20 gpurun_out/prepexp_${CFG:-c3}.err; exit 1; }
cat gpurun_out/prepexp_${CFG:-c3}.json
