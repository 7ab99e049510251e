cd $GRAFT_REPO_ROOT
MODES=ragged LIBS="cur= wgs2=abl/wgs2/lib/libmerklekv_hip.so" REPS=4 bash scripts/gpu_ab.sh || exit 1
