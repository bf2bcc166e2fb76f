#!/bin/bash
# Same-box A/B/... of several builds of libkad.so (ablibs/libkad_<name>.so, "new" = the product
# library) on one config: scripts/step_ab.py per (round, lib) in its own process, alternating.
#   scripts/ab_libs.sh TAG "old B C" UNITS [rounds] [cfg]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-ab}; libs=${2:-"old new"}; u=${3:-1000000}; rounds=${4:-3}; cfg=${5:-c3}
for r in $(seq 1 $rounds); do
  for lib in $libs; do
    L=ablibs/libkad_$lib.so; [ $lib = new ] && L=kubeadmiral_amd/libkad.so
    timeout -k 10 300 python scripts/step_ab.py --config $cfg --units $u --lib $L --rounds 1 --steps 30 > gpurun_out/${tag}_${lib}_$r.json 2>> gpurun_out/${tag}.log || exit 1
    echo "$cfg $lib $u $r $(python -c "import json; d=json.load(open('gpurun_out/${tag}_${lib}_$r.json')); print(d['mean']['base'])")"
  done
done
