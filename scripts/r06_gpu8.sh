#!/bin/bash
# LDS bank-conflict lead: score gathers at lane order (timing only) vs libkad.so on C3
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/ab_stats.sh r06nc ${CFG:-c3} 1000000 "${LIBS:-new nc1}" 10 > gpurun_out/r06nc_c3.txt 2>&1 || { cat gpurun_out/r06nc_c3.txt; exit 1; }
cat gpurun_out/r06nc_c3.txt
for lib in ${LIBS:-new nc1}; do
  L=ablibs/libkad_$lib.so; [ $lib = new ] && L=kubeadmiral_amd/libkad.so
  timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_ANY SQ_WAVE_CYCLES --output-format csv -d gpurun_out/r06nc_pmc_$lib -o run -- python \
    scripts/step_ab.py --config ${CFG:-c3} --units 1000000 --lib $L --rounds 1 --steps 5 > gpurun_out/r06nc_pmc_$lib.log 2>&1 || { echo "pmc $lib failed"; tail -5 gpurun_out/r06nc_pmc_$lib.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
import os
for lib in os.environ.get("LIBS", "new nc1").split():
    acc = collections.defaultdict(list)
    for f in glob.glob(f"gpurun_out/r06nc_pmc_{lib}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "schedule_wide_kernel" in r["Kernel_Name"]:
                acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(lib, {k: "%.4g" % (sum(v) / max(1, len(set(range(len(v)))))) for k, v in acc.items()})
PY
