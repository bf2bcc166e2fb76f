cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q8_pytest.log 2>&1 || { tail -30 gpurun_out/q8_pytest.log; exit 1; }
tail -1 gpurun_out/q8_pytest.log
for v in "KAD_NO_ORDER=1" "KAD_NO_ORDER=0"; do
  env $v timeout -k 10 300 python scripts/phase_prof.py --config c3 --units 125000 --reps 5 --out gpurun_out/q8_c3_$v.json > gpurun_out/q8.log 2>&1 || { tail -20 gpurun_out/q8.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q8_c3_$v.json')); print('$v', {k:v for k,v in d.items() if k.startswith(('lean_span','lean_wave_lifetime_frac','wide_cu_last','wide_late_units','wide_late_maxunit'))})"
done
for cu in c3:125000 c3 c4; do
  cfg=${cu%%:*}; u=""; [ "$cu" != "$cfg" ] && u="--units ${cu#*:}"
  timeout -k 10 300 python bench.py --config $cfg $u --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e > gpurun_out/q8_bench.json 2> gpurun_out/q8_bench.log || { tail -20 gpurun_out/q8_bench.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/q8_bench.json').read().strip().splitlines()[-1])
print('$cu', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
done
