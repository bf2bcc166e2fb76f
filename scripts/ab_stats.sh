#!/bin/bash
# Same-box kernel-time A/B of several builds (ablibs/libkad_<name>.so, "new" = libkad.so): one
# rocprofv3 --kernel-trace --stats run of scripts/step_ab.py per lib, then each kernel's average duration.
#   scripts/ab_stats.sh TAG CFG UNITS "old new px1" [steps]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; cfg=$2; units=$3; libs=$4; steps=${5:-10}
mkdir -p gpurun_out
for lib in $libs; do
  L=ablibs/libkad_$lib.so; [ $lib = new ] && L=kubeadmiral_amd/libkad.so
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_$lib -o run -- python \
    scripts/step_ab.py --config $cfg --units $units --lib $L --rounds 1 --steps $steps > gpurun_out/${tag}_$lib.log 2>&1 \
    || { echo "stats run $lib failed"; tail -5 gpurun_out/${tag}_$lib.log; exit 1; }
done
python - "$tag" $libs <<'PY'
import csv, glob, sys
tag, libs = sys.argv[1], sys.argv[2:]
for lib in libs:
    for f in glob.glob(f"gpurun_out/{tag}_{lib}/**/*kernel_stats.csv", recursive=True):
        rows = [r for r in csv.DictReader(open(f)) if int(r["Calls"]) > 2]
        print(lib, " ".join(f"{r['Name'].split('(')[0].replace('void ', '').replace('kad::', '')}={float(r['AverageNs'])/1e3:.1f}" for r in rows))
PY
