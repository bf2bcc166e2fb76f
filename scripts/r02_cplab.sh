cd "${GRAFT_REPO_ROOT}"
cp kubeadmiral_amd/libkad.so gpurun_out/libkad_base.so
for v in base cpl8 cpl2; do
  if [ $v != base ]; then cp kubeadmiral_amd/libkad_$v.so kubeadmiral_amd/libkad.so; fi
  for cfg in c3 c5; do
    timeout -k 10 300 python bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline --no-extra > gpurun_out/cpl_${v}_$cfg.json 2> gpurun_out/cpl_${v}_$cfg.log || exit 1
    python -c "import json; d=json.load(open('gpurun_out/cpl_${v}_$cfg.json')); print('$v $cfg', d['ms_per_step'], d['config']['stage_ms']['prep'])"
  done
  cp gpurun_out/libkad_base.so kubeadmiral_amd/libkad.so
done
rm -f gpurun_out/libkad_base.so
