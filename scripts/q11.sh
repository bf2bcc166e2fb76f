cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/q11_pytest.log 2>&1 || { tail -30 gpurun_out/q11_pytest.log; exit 1; }
tail -1 gpurun_out/q11_pytest.log
timeout -k 10 300 python scripts/phase_prof.py --config c4 --units 250000 --out gpurun_out/q11_c4.json > gpurun_out/q11.log 2>&1 || { tail -20 gpurun_out/q11.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q11_c4.json')); print('c4', {k:v for k,v in d.items() if k.startswith('plan')})"
cp kubeadmiral_amd/libkad.so /tmp/libkad_pf1.so
for rep in 1 2; do for v in pf1 pf0; do
  if [ $v = pf0 ]; then cp kubeadmiral_amd/libkad_pf0.so kubeadmiral_amd/libkad.so; else cp /tmp/libkad_pf1.so kubeadmiral_amd/libkad.so; fi
  timeout -k 10 300 python bench.py --config c4 --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e > gpurun_out/q11_bench.json 2> gpurun_out/q11_bench.log || { tail -20 gpurun_out/q11_bench.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/q11_bench.json').read().strip().splitlines()[-1])
print('c4 $v', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
done; done
cp /tmp/libkad_pf1.so kubeadmiral_amd/libkad.so
