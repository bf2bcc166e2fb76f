#!/bin/bash
# Round 6 (session 2): prep_kernel's branch-free taint-table lookups (new = libkad.so) against the previous code
# (ablibs/libkad_b256.so = HEAD 42ae01d's kernels), kernel averages per config, result digests.
# (the branch-free variant is described in profiles/r06/ab_prep_taint_branchfree.txt; the sources do not keep it)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for c in c3 c4 c2; do
  bash scripts/ab_stats.sh tt_$c $c 0 "b256 new" 10 > gpurun_out/tt_$c.txt 2>&1 || { cat gpurun_out/tt_$c.txt; exit 1; }
  echo "== $c"; cat gpurun_out/tt_$c.txt; grep -ho '"digest": "[0-9a-f]*"' gpurun_out/tt_${c}_*.log
done
