cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ragged_gpu.py tests/test_parity_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06t_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r06t_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="head=abl/head/lib/libmerklekv_hip.so new=" REPS=3 bash scripts/gpu_ab.sh
