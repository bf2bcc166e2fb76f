#!/bin/bash
# rocprofv3 passes for one bench config: kernel trace+stats, SQ instruction mix, HBM bytes.
# Counters are collected in their own passes (no sys/runtime trace alongside --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cfg=${1:-c2}; tag=${2:-run}
out=gpurun_out/prof_${cfg}_${tag}
mkdir -p "$out"
B="python bench.py --config $cfg --steps 5 --warmup 1 --no-cpu-baseline --no-extra --no-sweep --no-e2e ${UNITS:+--units $UNITS}"
run() {  # name, rocprof args...
  local name=$1; shift
  timeout -k 10 600 rocprofv3 "$@" --output-format csv -d "$out/$name" -o "$name" -- $B > "$out/$name.log" 2>&1
  local rc=$?; echo "== $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$out/$name.log"; exit $rc; fi
}
run trace --kernel-trace --stats
run sq --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_WAIT_ANY SQ_WAVE_CYCLES
run sq2 --pmc SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run fetch --pmc FETCH_SIZE
run write --pmc WRITE_SIZE
read W C < <(python -c "from kubeadmiral_amd import synth; print(*synth.SIZES['$cfg'])")
W=${UNITS:-$W}
python scripts/pmc_summary.py "$out" "$cfg" --units "$W" --clusters "$C" --json "$out/pmc_$cfg.json" > "$out/summary.txt"
cat "$out/summary.txt" | tail -30
