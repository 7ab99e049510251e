#!/bin/bash
# Round-3 A/B of the new paths on one box (interleaved, same process image): build (top reduce), diff
# workload (fused merge-join), incremental (roofline fields). Each run has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
run() { local tag=$1 lim=$2; shift 2; echo "== $tag"; env "$@" > gpurun_out/ab/$tag.json 2> gpurun_out/ab/$tag.err; local rc=$?
  echo "$tag rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/ab/$tag.err; exit $rc; }
  python3 scripts/ab_extract.py gpurun_out/ab/$tag.json; }
B="timeout -k 10 300 python bench.py --no-cpu-baseline"
for rep in 1 2; do
  run build_top1_$rep 300 MKV_TOP_REDUCE=1 $B --steps 20 --warmup 3 --no-diff
  run build_top0_$rep 300 MKV_TOP_REDUCE=0 $B --steps 20 --warmup 3 --no-diff
done
for rep in 1 2; do
  run diff_f1_$rep 300 MKV_DIFF_FUSED=1 $B --workload diff --steps 10 --warmup 2
  run diff_f0_$rep 300 MKV_DIFF_FUSED=0 $B --workload diff --steps 10 --warmup 2
done
run inc 300 $B --workload incremental --steps 5 --warmup 2
exit 0
