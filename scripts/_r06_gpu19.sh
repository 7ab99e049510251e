cd $GRAFT_REPO_ROOT
LIBS="cur= st4=abl/st4/lib/libmerklekv_hip.so" REPS=3 bash scripts/gpu_ab.sh || exit 1
