#!/bin/bash
# BASELINE configs 3/4/5 + on-the-fly chairs, current build
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --alternate_corr --size 288 960 --iters 24 --steps 5 --warmup 3 > gpurun_out/bench_cfg4_kitti_alt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg4_kitti_alt.log | cut -c1-200
timeout -k 10 300 python bench.py --size 400 720 --steps 5 --warmup 3 > gpurun_out/bench_cfg3_things.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg3_things.log | cut -c1-200
timeout -k 10 300 python bench.py --alternate_corr --steps 10 --warmup 5 > gpurun_out/bench_chairs_alt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_chairs_alt.log | cut -c1-200
for b in 16 64; do
  timeout -k 10 300 python bench_infer.py --batch $b --steps 3 --warmup 1 --graph > gpurun_out/bench_infer_b${b}_graph.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_infer_b${b}_graph.log | cut -c1-200
done
timeout -k 10 300 python bench_infer.py --batch 16 --steps 3 --warmup 1 > gpurun_out/bench_infer_b16_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_infer_b16_eager.log | cut -c1-200
timeout -k 10 300 python bench_infer.py --batch 64 --steps 3 --warmup 1 --graph --alternate_corr > gpurun_out/bench_infer_b64_alt_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_infer_b64_alt_graph.log | cut -c1-200
