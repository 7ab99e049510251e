#!/bin/bash
# N>1 code paths of every bench workload on a one-GPU box: ranks share device 0, collectives on gloo.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export MKV_BENCH_SAME_GPU=1 MKV_DIST_BACKEND=gloo
NP=${NP:-2}
run() {
  local tag=$1; shift
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $NP --master-addr 127.0.0.1 \
    --master-port $((29500 + RANDOM % 1000)) bench.py --gpus $NP --steps 2 --warmup 1 --no-cpu-baseline "$@" \
    > gpurun_out/mr_$tag.json 2> gpurun_out/mr_$tag.err || { echo "$tag failed"; tail -30 gpurun_out/mr_$tag.err; exit 1; }
  echo "== $tag"; cat gpurun_out/mr_$tag.json
}
run build --records 1000000 --route-records 1000000
run diff --workload diff --records 1000000
run inc --workload incremental --records 1000000 --batch 1000 --replicas 4

# RCCL (nccl backend) with one rank: the device-resident fringe path (mkv_shard_fringe_device -> RCCL
# all_gather -> mkv_shard_combine_device) and the batched recombine, on the one GPU this box has.
unset MKV_BENCH_SAME_GPU MKV_DIST_BACKEND
export MKV_BENCH_FORCE_DIST=1
NP=1
run build_rccl1 --records 1000000 --no-diff --route-records 2000000
run inc_rccl1 --workload incremental --records 1000000 --batch 1000 --replicas 4
