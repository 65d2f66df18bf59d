#!/bin/bash
# 4-rank data-parallel rehearsal on one GPU (gloo): graphed step, fp32 (pins the all-reduce math)
# and bf16; rank-0 tuning shared with every rank.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp MASTER_ADDR=127.0.0.1 RAFT_DIST_BACKEND=gloo
O=gpurun_out/diag; mkdir -p $O
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
MIOPEN_FIND_MODE=FAST timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29611 scripts/dp_rehearsal.py --graph --fp32 > $O/dp4_graph_fp32.log 2>&1 || { tail -20 $O/dp4_graph_fp32.log; exit 1; }
grep "dp rehearsal" $O/dp4_graph_fp32.log
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29612 scripts/dp_rehearsal.py --graph > $O/dp4_graph_bf16.log 2>&1 || { tail -20 $O/dp4_graph_bf16.log; exit 1; }
grep "dp rehearsal" $O/dp4_graph_bf16.log
