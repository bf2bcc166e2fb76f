#!/bin/bash
# Wide-kernel phase costs on the GPU box: per KAD_WIDE_EXPERIMENT variant, the stage times and one SQ
# instruction-count pass (rocprofv3 --pmc, counters only). Needs ablibs/libkad_tune.so
# (python scripts/wide_exp.py --build, on the CPU side).   scripts/wide_exp.sh [cfg] [units] [bits...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=${1:-c3}; units=${2:-0}; shift 2
bits=${*:-0 1 2 4 8}
out=gpurun_out/wide_exp_$cfg
mkdir -p "$out"
for b in $bits; do
  KAD_WIDE_EXPERIMENT=$b timeout -k 10 240 python scripts/wide_exp.py --config "$cfg" --units "$units" > "$out/time_$b.json" 2> "$out/time_$b.log"
  rc=$?; echo "== exp $b time rc=$rc $(cat $out/time_$b.json)"; [ $rc -ne 0 ] && exit $rc
  KAD_WIDE_EXPERIMENT=$b timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY --output-format csv -d "$out/pmc_$b" -o pmc -- python scripts/wide_exp.py --config "$cfg" --units "$units" --reps 3 > "$out/pmc_$b.log" 2>&1
  rc=$?; echo "== exp $b pmc rc=$rc"; [ $rc -ne 0 ] && { tail -5 "$out/pmc_$b.log"; exit $rc; }
done
python - "$out" $bits <<'PY'
import csv, glob, json, sys, collections
out, bits = sys.argv[1], sys.argv[2:]
for b in bits:
    f = glob.glob(f"{out}/pmc_{b}/**/*counter_collection.csv", recursive=True)
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(f[0])):
        if "schedule_wide_kernel" in row["Kernel_Name"]:
            acc[(row["Dispatch_Id"], row["Counter_Name"])].append(float(row["Counter_Value"]))
    per = collections.defaultdict(list)
    for (d, c), v in acc.items():
        per[c].append(sum(v))
    t = json.load(open(f"{out}/time_{b}.json"))
    W = t["units"]
    print(b, f"main_ms={t['stage_ms']['main']:.3f}", " ".join(f"{c}/unit={sum(v)/len(v)/W:.1f}" for c, v in sorted(per.items())))
PY
