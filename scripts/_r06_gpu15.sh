cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_ragged_gpu.py tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ad_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06ad_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=3 bash scripts/gpu_ab.sh
