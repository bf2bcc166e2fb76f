#!/bin/bash
# libkad_NAME.so from the working tree's sources with extra compile flags (tuning macros), for same-box A/B
# runs against libkad.so / libkad_old.so.   scripts/build_variant.sh NAME "-DKAD_PREP_AFFW=2 ..."
set -e
name=$1; flags=$2
repo=$(cd "$(dirname "$0")/.." && pwd)
d=$(mktemp -d); mkdir -p "$repo/ablibs"
cd "$repo/kubeadmiral_amd/csrc"
for f in kad_kernels.hip kad_trigger.hip kad_delta.hip kad_diff.hip kad_api.hip kad_pack.cpp kad_objects.cpp; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -w -pthread $flags \
    -I"$repo/include" -c $f -o "$d/$f.o" &
done
for j in $(jobs -p); do wait $j || { echo "compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -pthread -o "$repo/ablibs/libkad_$name.so" "$d"/*.o
rm -rf "$d"
echo "$repo/ablibs/libkad_$name.so ($flags)"
