cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/round_check.sh test tag=${1:-r03g} || exit 1
bash scripts/final_bench.sh ${1:-r03g} "c3 c2 c4 c5"
