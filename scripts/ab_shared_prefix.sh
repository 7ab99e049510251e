cd $GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_parity_gpu.py -k "shared_prefix or long_common or tie_runs or prefix_of or duplicates or ragged or synthetic_sizes" > gpurun_out/pt.log 2>&1 || { tail -30 gpurun_out/pt.log; exit 1; }
tail -2 gpurun_out/pt.log
for L in new old; do
  if [ $L = old ]; then export MKV_LIB_PATH=$GRAFT_REPO_ROOT/merklekv_amd/lib/ab_old/libmerklekv_hip.so; fi
  timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --diff-records 1000000 --anchor-records 0 > gpurun_out/sp_$L.json 2> gpurun_out/sp_$L.err || { tail -20 gpurun_out/sp_$L.err; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/sp_$L.json').read().strip().splitlines()[-1]); print('$L', round(d['ms_per_step'],3), d['stage_ms_per_step'], d['shared_prefix_10m'])"
done
