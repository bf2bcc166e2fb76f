cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for x in 0 1 2 4 7; do
  KAD_ROW_EXPERIMENT=$x timeout -k 10 300 python scripts/phase_prof.py --config c5 --units 30000 --out gpurun_out/q3_c5_x$x.json > gpurun_out/q3_c5_x$x.log 2>&1 || { tail -20 gpurun_out/q3_c5_x$x.log; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/q3_c5_x$x.json')); print('exp $x', {k:v for k,v in d.items() if k.startswith('row_')})"
done
