cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest tests/test_parity_gpu.py tests/test_update_gpu.py tests/test_shard_gpu.py tests/test_reference_ports_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ae_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06ae_pytest.log; [ $rc -eq 0 ] || exit $rc
MODES=fixed LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=3 bash scripts/gpu_ab.sh || exit 1
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=2 TAILC=300 CMD="python tools/ab_inc.py" bash scripts/gpu_ab.sh > /dev/null || exit 1
grep -H "configs4" gpurun_out/ab/*_[12].log
