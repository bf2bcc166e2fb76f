#!/bin/bash
# libkad_old.so from a git revision's sources (default HEAD), for same-box A/B runs against the working tree's
# libkad.so (scripts/ab_units.sh, scripts/ab_libs.sh).   scripts/build_old.sh [REV] [NAME]
set -e
rev=${1:-HEAD}; name=${2:-old}
repo=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d); mkdir -p "$repo/ablibs"
git -C "$repo" archive "$rev" kubeadmiral_amd/csrc include | tar x -C "$d"
cd "$d/kubeadmiral_amd/csrc"
for f in kad_kernels.hip kad_trigger.hip kad_delta.hip kad_diff.hip kad_api.hip kad_pack.cpp kad_objects.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -pthread -c $f -o "$d/$f.o" &
done
for j in $(jobs -p); do wait $j || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "$repo/ablibs/libkad_$name.so" "$d"/*.o
rm -rf "$d"
echo "$repo/ablibs/libkad_$name.so ($rev)"
