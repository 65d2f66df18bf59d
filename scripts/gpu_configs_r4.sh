#!/bin/bash
# BASELINE configs beyond the headline on the current build: precisions (fp16 GradScaler, fp32),
# the KITTI config-4 shape with BOTH correlation blocks (the all-pairs / on-the-fly crossover),
# FlyingThings3D, RAFT-small, batched hipGraph inference.  -> gpurun_out/cfg4/
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/cfg4/miopen_db
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/cfg4/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/cfg4/miopen_db
run() {  # run <tag> <timeout> <bench args...>
  local tag=$1 to=$2; shift 2
  timeout -k 10 $to python -u bench.py "$@" > gpurun_out/cfg4/$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/cfg4/$tag.log; return 1; }
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*\|"corr": "[a-z-]*"' gpurun_out/cfg4/$tag.log | tr '\n' ' ')"
}
for c in "$@"; do
  case $c in
    fp16) run fp16 500 --precision fp16 ;;
    fp32) run fp32 900 --precision fp32 ;;
    fp32cl) run fp32cl 900 --precision fp32 --channels_last ;;
    b384) MIOPEN_FIND_MODE=2 run train_b384_bn 900 --batch 384 --steps 3 --warmup 2 ;;
    kitti_ap) run kitti_ap 500 --size 288 960 --iters 24 --corr_mode allpairs ;;
    kitti_otf) run kitti_otf 500 --size 288 960 --iters 24 --corr_mode onthefly ;;
    chairs_otf) run chairs_otf 400 --corr_mode onthefly ;;
    things) run things 400 --size 400 720 ;;
    small) run small 400 --small ;;
    infer) timeout -k 10 300 python bench_infer.py --graph --batch 64 > gpurun_out/cfg4/infer_b64_graph.log 2>&1 && grep -o '"value": [0-9.]*\|"ms_per_pair": [0-9.]*' gpurun_out/cfg4/infer_b64_graph.log | tr '\n' ' '; echo " infer b64" ;;
  esac || exit 1
done
