#!/bin/bash
# A/B of two builds of libkad.so on the same box: bench lines alternating between the product library and
# ablibs/libkad_old.so (runtime.LIB_PATH patched before the first load).
#   scripts/ab_lib.sh TAG "c3 c2" [rounds]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
tag=${1:-ab}; cfgs=${2:-c3}; rounds=${3:-2}
for r in $(seq 1 $rounds); do
  for lib in old new; do
    for cfg in $cfgs; do
      timeout -k 10 300 python - "$lib" "$cfg" > gpurun_out/${tag}_${lib}_${cfg}_$r.json 2>> gpurun_out/${tag}.log <<'PY' || exit 1
import os, runpy, sys
lib, cfg = sys.argv[1], sys.argv[2]
from kubeadmiral_amd import runtime
if lib == "old":
    runtime.LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(runtime.__file__)), "ablibs", "libkad_old.so")
sys.argv = ["bench.py", "--config", cfg, "--steps", "20", "--warmup", "3", "--no-cpu-baseline", "--no-extra",
            "--no-sweep", "--no-e2e"]
runpy.run_path("bench.py", run_name="__main__")
PY
      python - gpurun_out/${tag}_${lib}_${cfg}_$r.json "$lib $cfg $r" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], "ms %.4f" % d["ms_per_step"], {k: round(v, 4) for k, v in d["config"]["stage_ms"].items()})
PY
    done
  done
done
