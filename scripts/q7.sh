cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
cp kubeadmiral_amd/libkad.so /tmp/libkad_orig.so
for rep in 1 2; do
for ru in 2 3; do
  cp kubeadmiral_amd/libkad_ru$ru.so kubeadmiral_amd/libkad.so
  timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 3 --no-cpu-baseline --no-extra --no-sweep --no-e2e > gpurun_out/q7_bench_c5_$ru.json 2> gpurun_out/q7_bench.log || { tail -20 gpurun_out/q7_bench.log; exit 1; }
  python -c "
import json; d=json.loads(open('gpurun_out/q7_bench_c5_$ru.json').read().strip().splitlines()[-1])
print('ru $ru', round(d['ms_per_step'],4), {k: round(v, 4) for k, v in d['config']['stage_ms'].items()})"
done; done
cp /tmp/libkad_orig.so kubeadmiral_amd/libkad.so
