cd $GRAFT_REPO_ROOT
for b in 0 1 2 3 4 5; do
  if [ $b = 0 ]; then unset KAD_LEAN_BLOCKS_PER_CU; else export KAD_LEAN_BLOCKS_PER_CU=$b; fi
  echo "blocks_per_cu=$b"; timeout -k 10 120 python bench.py --steps 10 --warmup 2 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['config']['kernel_ms'], d['value']/1e9)" || exit 1
done
