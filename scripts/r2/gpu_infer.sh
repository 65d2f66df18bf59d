#!/bin/bash
# config-5 Sintel inference (436x1024, iters 32): batch sweep up to >=50% of HBM, plus on-the-fly
# correlation under +-64 px smooth / discontinuous warm-start coordinates
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/sweep
mkdir -p $O
j() { grep -o '"value[^,]*\|"ms_per_step[^,]*\|"peak_hbm[^,]*\|"finite[^,]*' $1 | tr '\n' ' '; }
run() { n=$1; shift; timeout -k 10 600 python -u bench_infer.py "$@" > $O/infer_$n.log 2>&1 || { echo "infer $n failed"; tail -5 $O/infer_$n.log; exit 1; }; echo "infer $n $(j $O/infer_$n.log)"; }
run otf_b64 --batch 64 --steps 3 --warmup 1 --graph --alternate_corr
run otf_b64_fi64 --batch 64 --steps 3 --warmup 1 --graph --alternate_corr --flow_init_px 64
run otf_b64_fi64d --batch 64 --steps 3 --warmup 1 --graph --alternate_corr --flow_init_px 64 --discontinuous
run ap_b64_fi64d --batch 64 --steps 3 --warmup 1 --graph --flow_init_px 64 --discontinuous
run ap_b256 --batch 256 --steps 2 --warmup 1 --graph
run otf_b256 --batch 256 --steps 2 --warmup 1 --graph --alternate_corr
run ap_b512 --batch 512 --steps 2 --warmup 1
run otf_b512 --batch 512 --steps 2 --warmup 1 --alternate_corr
run otf_b1024 --batch 1024 --steps 2 --warmup 1 --alternate_corr
