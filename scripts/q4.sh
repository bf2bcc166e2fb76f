cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q4_pytest.log 2>&1 || { tail -30 gpurun_out/q4_pytest.log; exit 1; }
tail -1 gpurun_out/q4_pytest.log
timeout -k 10 300 python scripts/phase_prof.py --config c5 --out gpurun_out/q4_phase_c5.json > gpurun_out/q4_phase_c5.log 2>&1 || { tail -20 gpurun_out/q4_phase_c5.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q4_phase_c5.json')); print('c5', {k:v for k,v in d.items() if k.startswith('row_')})"
for cfg in c5 c3 c2; do
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep > gpurun_out/q4_bench_$cfg.json 2> gpurun_out/q4_bench.log || { tail -20 gpurun_out/q4_bench.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/q4_bench_$cfg.json').read().strip().splitlines()[-1]); e=d['end_to_end']
print('$cfg', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()}, 'e2e %.3g' % e['decisions_per_s'], {k: round(v, 2) for k, v in e['sequential'].items() if k.endswith('ms')}, round(e['pipelined']['total_ms'],1))"
done
for tn in "0 0" "0 1" "2 1"; do
  set -- $tn
  KAD_WQ_TAIL=$1 KAD_WQ_NEAR=$2 timeout -k 10 300 python scripts/phase_prof.py --config c3 --units 125000 --reps 5 --out gpurun_out/q4_c3_$1$2.json > gpurun_out/q4.log 2>&1 || { tail -20 gpurun_out/q4.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q4_c3_$1$2.json')); print('c3 125k tail $1 near $2', {k:v for k,v in d.items() if k in ('lean_span_us','lean_wave_lifetime_frac','wide_late_end_frac_mean','wide_rest_end_frac_mean')})"
done
