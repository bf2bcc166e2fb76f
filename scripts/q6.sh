cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for ru in 2 3 4; do
  KAD_PROF_LIB=kubeadmiral_amd/libkad_prof_ru$ru.so timeout -k 10 300 python scripts/phase_prof.py --config c5 --out gpurun_out/q6_c5_ru$ru.json > gpurun_out/q6.log 2>&1 || { tail -20 gpurun_out/q6.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q6_c5_ru$ru.json')); print('ru $ru', {k:v for k,v in d.items() if k.startswith('row_')})"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "row or c5 or affinity or taint" > gpurun_out/q6_pytest.log 2>&1 || { tail -30 gpurun_out/q6_pytest.log; exit 1; }
tail -1 gpurun_out/q6_pytest.log
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e > gpurun_out/q6_bench_c5.json 2> gpurun_out/q6_bench.log || { tail -20 gpurun_out/q6_bench.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/q6_bench_c5.json').read().strip().splitlines()[-1])
print('c5', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
timeout -k 10 300 python scripts/phase_prof.py --config c4 --units 250000 --out gpurun_out/q6_c4.json > gpurun_out/q6.log 2>&1 || { tail -20 gpurun_out/q6.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q6_c4.json')); print('c4', {k:v for k,v in d.items() if k.startswith('plan') or k.startswith('lean_')})"
