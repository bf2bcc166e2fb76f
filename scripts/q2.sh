cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for t in 0 2; do
  KAD_WQ_TAIL=$t timeout -k 10 300 python scripts/phase_prof.py --config c3 --units 125000 --out gpurun_out/q2_phase_t$t.json > gpurun_out/q2_phase_t$t.log 2>&1 || { tail -20 gpurun_out/q2_phase_t$t.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q2_phase_t$t.json')); print('tail $t', {k:v for k,v in d.items() if k.startswith(('lean_span','lean_wave_lifetime_frac','lean_end_p','wide_'))})"
done
bash scripts/iter2.sh q2 "row or c5" "c5" ""
timeout -k 10 300 python scripts/phase_prof.py --config c5 --out gpurun_out/q2_phase_c5.json > gpurun_out/q2_phase_c5.log 2>&1 || { tail -20 gpurun_out/q2_phase_c5.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q2_phase_c5.json')); print('c5', {k:v for k,v in d.items() if k.startswith('row_')})"
