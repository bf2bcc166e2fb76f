cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_row_patterns.py -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/q9_pytest.log 2>&1; rc=$?
tail -15 gpurun_out/q9_pytest.log; exit $rc
