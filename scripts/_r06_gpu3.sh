cd $GRAFT_REPO_ROOT
MKV_WAIT_TIMEOUT_S=20 timeout -k 10 150 stdbuf -oL ./tests/cpp/test_sharded > gpurun_out/r06c_sharded.log 2>&1; rc=$?; echo "rc=$rc"; tail -40 gpurun_out/r06c_sharded.log
