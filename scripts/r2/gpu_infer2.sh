#!/bin/bash
# config-5 large-batch Sintel inference: all-pairs at batch 512 (~68 GB pyramid), auto policy at
# batch 1024 (pyramid 135 GB > budget -> on-the-fly)
set -o pipefail
cd "$(dirname "$0")/../.."
O=gpurun_out/sweep
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_model_gpu.py -q -x -k "auto_corr" --timeout 150 > $O/test_auto.log 2>&1; rc=$?; tail -1 $O/test_auto.log; [ $rc -eq 0 ] || exit $rc
j() { grep -o '"value[^,]*\|"ms_per_step[^,]*\|"peak_[a-z_]*gib[^,]*\|"device_used_gib[^,]*\|"corr"[^,]*\|"finite[^,]*' $1 | tr '\n' ' '; }
run() { n=$1; shift; timeout -k 10 900 python -u bench_infer.py "$@" > $O/infer_$n.log 2>&1 || { echo "infer $n failed"; tail -5 $O/infer_$n.log; exit 1; }; echo "infer $n $(j $O/infer_$n.log)"; }
run ap_b512 --batch 512 --steps 2 --warmup 1 --corr_mode allpairs
run auto_b1024 --batch 1024 --steps 2 --warmup 1
