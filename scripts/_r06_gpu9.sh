cd $GRAFT_REPO_ROOT
R=$(pwd); P=$R/gpurun_out/r06y_vo; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $R/tools/ab_diff.py > $P/trace.log 2>&1; rc=$?; echo "rc=$rc"; tail -3 $P/trace.log; exit $rc
