cd $GRAFT_REPO_ROOT
LIBS="cur= kclate=abl/kclate/lib/libmerklekv_hip.so" REPS=3 bash scripts/gpu_ab.sh || exit 1
