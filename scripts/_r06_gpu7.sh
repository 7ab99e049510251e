cd $GRAFT_REPO_ROOT
R=$(pwd); P=$R/gpurun_out/r06s_rag; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
MODES=ragged STEPS=10 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $R/tools/ab_ragged.py trace > $P/trace.log 2>&1; rc=$?; echo "rc=$rc"; tail -3 $P/trace.log; exit $rc
