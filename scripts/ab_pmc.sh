#!/bin/bash
# Same-box counter A/B of ablibs/libkad_old.so vs the product library: one rocprofv3 --pmc pass per
# (lib, counter set) over scripts/step_ab.py, then the per-dispatch average of each counter for the kernels
# matching REGEX.   scripts/ab_pmc.sh TAG CFG UNITS REGEX "FETCH_SIZE" ["WRITE_SIZE" ...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag=$1; cfg=$2; units=$3; rx=$4; shift 4
mkdir -p gpurun_out
for lib in old new; do
  L=kubeadmiral_amd/libkad.so; [ $lib = old ] && L=ablibs/libkad_old.so
  i=0
  for set in "$@"; do
    i=$((i + 1))
    d=gpurun_out/${tag}_${lib}_$i
    timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d $d -o run -- python scripts/step_ab.py --config $cfg \
      --units $units --lib $L --rounds 1 --steps 5 > $d.log 2>&1 || { echo "pmc pass $lib $set failed"; tail -5 $d.log; exit 1; }
  done
done
python - "$tag" "$rx" <<'EOF'
import csv, glob, re, sys
from collections import defaultdict
tag, rx = sys.argv[1], re.compile(sys.argv[2])
for lib in ("old", "new"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(f"gpurun_out/{tag}_{lib}_*/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if rx.search(r["Kernel_Name"]):
                acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, d in acc.items():
        print(lib, k, {c: round(sum(v) / len(v), 1) for c, v in d.items()})
EOF
