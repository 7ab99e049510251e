cd $GRAFT_REPO_ROOT
bash scripts/pmc_incremental.sh > gpurun_out/r06zz_pmc_inc.log 2>&1 || { tail -5 gpurun_out/r06zz_pmc_inc.log; exit 1; }
PROF_DIR=r06zz/prof_inc BENCH_ARGS="--workload incremental" bash scripts/gpu_prof.sh > /dev/null || exit 1
PROF_DIR=r06zz/prof_diff BENCH_ARGS="--workload diff" bash scripts/gpu_prof.sh > /dev/null || exit 1
echo done
