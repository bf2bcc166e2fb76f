cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python scripts/phase_prof.py --config c5 --out gpurun_out/q10_c5.json > gpurun_out/q10.log 2>&1 || { tail -20 gpurun_out/q10.log; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/q10_c5.json')); print({k:v for k,v in d.items() if k.startswith('row_')})"
