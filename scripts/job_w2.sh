mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "c3 or row_kernel or rows or c5_subset" > gpurun_out/w2_pytest.log 2>&1 || { echo "pytest rc=$?"; tail -30 gpurun_out/w2_pytest.log; exit 1; }
tail -3 gpurun_out/w2_pytest.log
KAD_PACK_TIMING=1 KAD_UPLOAD_TIMING=1 timeout -k 10 300 python scripts/e2e_prof.py --config c3 --out gpurun_out/e2e2_c3.json > gpurun_out/e2e2_c3.log 2>&1 || exit 2
KAD_PACK_TIMING=1 timeout -k 10 200 python scripts/e2e_prof.py --config c5 --reps 2 --out gpurun_out/e2e2_c5.json > gpurun_out/e2e2_c5.log 2>&1 || exit 3
bash scripts/wide_exp.sh c3 0 0 1 2 4 8 > gpurun_out/wexp1.log 2>&1 || { tail -5 gpurun_out/wexp1.log; exit 4; }
tail -6 gpurun_out/wexp1.log
