#!/bin/bash
# Same-box A/B of ablibs/libkad_old.so vs the product library on one config at given unit counts:
# scripts/step_ab.py per (round, lib, units) in its own process, alternating.   scripts/ab_units.sh TAG "125000 1000000" [rounds] [cfg]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-ab}; units=${2:-1000000}; rounds=${3:-3}; cfg=${4:-c3}
for r in $(seq 1 $rounds); do
  for u in $units; do
    for lib in old new; do
      L=kubeadmiral_amd/libkad.so; [ $lib = old ] && L=ablibs/libkad_old.so
      timeout -k 10 300 python scripts/step_ab.py --config $cfg --units $u --lib $L --rounds 1 --steps 30 > gpurun_out/${tag}_${lib}_${u}_$r.json 2>> gpurun_out/${tag}.log || exit 1
      echo "$lib $u $r $(python -c "import json,sys; d=json.load(open('gpurun_out/${tag}_${lib}_${u}_$r.json')); print(d['mean']['base'])")"
    done
  done
done
