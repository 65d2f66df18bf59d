#!/bin/bash
# other BASELINE configs on the current build + a batch-192 run with MIOpen's fast find
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg
timeout -k 10 400 python bench.py --size 400 720 > gpurun_out/cfg/cfg3_things.log 2>&1 || { tail -3 gpurun_out/cfg/cfg3_things.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*' gpurun_out/cfg/cfg3_things.log | tr '\n' ' '; echo " things"
timeout -k 10 400 python bench.py --size 288 960 --iters 24 --corr_mode onthefly > gpurun_out/cfg/cfg4_kitti_otf.log 2>&1 || { tail -3 gpurun_out/cfg/cfg4_kitti_otf.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*' gpurun_out/cfg/cfg4_kitti_otf.log | tr '\n' ' '; echo " kitti otf"
timeout -k 10 400 python bench.py --small > gpurun_out/cfg/small.log 2>&1 || { tail -3 gpurun_out/cfg/small.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' gpurun_out/cfg/small.log | tr '\n' ' '; echo " small"
timeout -k 10 300 python bench_infer.py --graph --batch 64 > gpurun_out/cfg/infer_b64_graph.log 2>&1 || { tail -3 gpurun_out/cfg/infer_b64_graph.log; exit 1; }
grep -o '"value": [0-9.]*\|"ms_per_pair": [0-9.]*' gpurun_out/cfg/infer_b64_graph.log | tr '\n' ' '; echo " infer b64"
date +%T
MIOPEN_FIND_MODE=2 timeout -k 10 600 python -u bench.py --batch 192 --steps 5 --warmup 2 > gpurun_out/cfg/train_b192_fastfind.log 2>&1
echo "b192 rc=$?"; date +%T
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*' gpurun_out/cfg/train_b192_fastfind.log | tr '\n' ' '
