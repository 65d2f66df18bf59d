#!/bin/bash
# round-2 re-measure of the other BASELINE configs + RAFT-small + inference with the current build
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
O=gpurun_out/c19
mkdir -p $O
j() { grep -o '"value[^,]*\|"ms_per_step[^,]*\|"peak_hbm[^,]*\|"host_issue_ms[^,]*\|"corr"[^,]*\|"loss_finite[^,]*' $1 | tr '\n' ' '; }
run() { n=$1; shift; timeout -k 10 420 python "$@" > $O/$n.log 2>&1 || { echo "$n failed"; tail -5 $O/$n.log; exit 1; }; echo "$n $(j $O/$n.log)"; }
run bench_rep1 bench.py --steps 20 --warmup 5
run bench_rep2 bench.py --steps 20 --warmup 5
run cfg3_things bench.py --size 400 720 --steps 10 --warmup 3
run cfg4_kitti_alt bench.py --alternate_corr --size 288 960 --iters 24 --steps 5 --warmup 2
run chairs_alt bench.py --alternate_corr --steps 10 --warmup 3
run small bench.py --small --steps 10 --warmup 3
run train_b24 bench.py --batch 24 --steps 10 --warmup 3
run train_b48 bench.py --batch 48 --steps 10 --warmup 3
run infer_b64_graph bench_infer.py --batch 64 --steps 3 --warmup 1 --graph
