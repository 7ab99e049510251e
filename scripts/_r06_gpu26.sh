cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_update_gpu.py tests/test_antientropy_gpu.py tests/test_reference_ports_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06aj_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06aj_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=3 TAILC=120 CMD="python tools/ab_diff.py" bash scripts/gpu_ab.sh > /dev/null || exit 1
grep -H "vo-diff" gpurun_out/ab/*_[123].log
