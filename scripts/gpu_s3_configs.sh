#!/bin/bash
# multi-rank DP rehearsal on one GPU (gloo) + the other BASELINE configs at 1 GPU
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
RAFT_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 scripts/dp_rehearsal.py > gpurun_out/dp_rehearsal.log 2>&1
rc=$?; grep -E "dp rehearsal|Error|error" gpurun_out/dp_rehearsal.log | tail -5
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --alternate_corr --size 288 960 --iters 24 --steps 5 --warmup 2 > gpurun_out/bench_cfg4_kitti_alt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg4_kitti_alt.log | cut -c1-400
timeout -k 10 300 python bench.py --size 400 720 --steps 5 --warmup 2 > gpurun_out/bench_cfg3_things.log 2>&1 || exit $?
tail -1 gpurun_out/bench_cfg3_things.log | cut -c1-400
timeout -k 10 300 python bench.py --alternate_corr --steps 10 --warmup 3 > gpurun_out/bench_chairs_alt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_chairs_alt.log | cut -c1-400
timeout -k 10 300 python bench_infer.py --batch 64 --steps 3 --warmup 1 --graph > gpurun_out/bench_infer_b64_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_infer_b64_graph.log
timeout -k 10 300 python bench_infer.py --batch 64 --steps 3 --warmup 1 --graph --alternate_corr > gpurun_out/bench_infer_b64_alt_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_infer_b64_alt_graph.log
