cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
bash scripts/q7.sh || exit 1
bash scripts/round_check.sh test prof:c3,c2 tag=r03f
