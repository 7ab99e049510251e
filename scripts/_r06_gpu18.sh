cd $GRAFT_REPO_ROOT
R=$(pwd)
MODES=ragged LIBS="cur= wgs2=abl/wgs2/lib/libmerklekv_hip.so" REPS=3 bash scripts/gpu_ab.sh || exit 1
P=$R/gpurun_out/r06ag_rag; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
MODES=ragged STEPS=6 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $R/tools/ab_ragged.py trace > $P/trace.log 2>&1; rc=$?; echo "trace rc=$rc"; exit $rc
