cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_update_gpu.py -x -q -m gpu -k "many or batch or topdown or incremental or variants" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06ab_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06ab_pytest.log; [ $rc -eq 0 ] || exit $rc
LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=2 TAILC=300 CMD="python tools/ab_inc.py" bash scripts/gpu_ab.sh > /dev/null || exit 1
grep -H "configs4" gpurun_out/ab/*_[12].log
PROF_DIR=r06ab_inc BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > /dev/null || exit 1
