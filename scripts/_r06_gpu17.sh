cd $GRAFT_REPO_ROOT
R=$(pwd)
timeout -k 10 300 python -u -m pytest tests/test_ragged_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r06af_pytest.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r06af_pytest.log; [ $rc -eq 0 ] || exit $rc
MODES=ragged LIBS="prev=abl/prev/lib/libmerklekv_hip.so new=" REPS=3 bash scripts/gpu_ab.sh || exit 1
P=$R/gpurun_out/r06af_pmc; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
MODES=ragged STEPS=4 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $P -o run --output-format csv -- python3 $R/tools/ab_ragged.py pmc > $P/run.log 2>&1; rc=$?; echo "ragged pmc rc=$rc"; exit $rc
