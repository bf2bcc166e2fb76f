cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in "default" "KAD_ROWS_AFTER=1" "KAD_NO_ROWS=1"; do
  env_arg=""; [ "$v" != default ] && env_arg="$v"
  env $env_arg timeout -k 10 300 python scripts/phase_prof.py --config c3 --units 125000 --reps 5 --out gpurun_out/q5_c3_$v.json > gpurun_out/q5.log 2>&1 || { tail -20 gpurun_out/q5.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q5_c3_$v.json')); print('$v', {k:v for k,v in d.items() if k.startswith(('lean_span','lean_wave_lifetime_frac','wide_cu','wide_xcc'))})"
done
for cfg in c2 c5; do
timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e > gpurun_out/q5_bench_$cfg.json 2> gpurun_out/q5_bench.log || { tail -20 gpurun_out/q5_bench.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/q5_bench_$cfg.json').read().strip().splitlines()[-1])
print('$cfg', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
done
