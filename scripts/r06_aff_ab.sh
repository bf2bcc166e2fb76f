#!/bin/bash
# Round 6 (session 2): requirement rows ANDed KAD_AFF_UNROLL at a time in affinity_words (prep_kernel,
# prep_wave_kernel): u1 / u2 / u4 variant libraries of one source and the product library (new), kernel averages
# per config (scripts/ab_stats.sh) and result digests.
# (KAD_AFF_UNROLL exists only with profiles/r06/aff_unroll.patch applied; the sources do not keep it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in ${CFGS:-c5 c3}; do
  bash scripts/ab_stats.sh aff_$c $c 0 "${LIBS:-new u1 u2 u4}" 10 > gpurun_out/aff_$c.txt 2>&1 || { cat gpurun_out/aff_$c.txt; exit 1; }
  echo "== $c"; cat gpurun_out/aff_$c.txt; grep -ho '"digest": "[0-9a-f]*"' gpurun_out/aff_${c}_*.log | sort | uniq -c
done
