cd $GRAFT_REPO_ROOT
R=$(pwd)
( while true; do date >> gpurun_out/r06_heartbeat.log; sleep 45; done ) &
HB=$!
trap "kill $HB" EXIT
TAG=r06ev PART=lines bash scripts/gpu_evidence.sh || exit 1
bash scripts/pmc_incremental.sh > gpurun_out/r06ev/pmc_inc.log 2>&1 || { tail -5 gpurun_out/r06ev/pmc_inc.log; exit 1; }
tail -3 gpurun_out/r06ev/pmc_inc.log
PROF_DIR=r06ev/prof_inc BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > /dev/null || exit 1
P=$R/gpurun_out/r06ev/pmc_ragged; mkdir -p $P
cd /tmp && export TMPDIR=/tmp
MODES=ragged STEPS=4 timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE SQ_WAVE_CYCLES -d $P -o run --output-format csv -- python3 $R/tools/ab_ragged.py pmc > $P/run.log 2>&1; rc=$?; echo "ragged pmc rc=$rc"; tail -2 $P/run.log; exit $rc
