#!/bin/bash
# large-batch training sweep (HBM headroom): per-GPU batch 96 / 192 / 384, all-pairs vs on-the-fly
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/sweep
CFGS=${SWEEP_CFGS:-"96:allpairs 96:onthefly 192:allpairs 192:onthefly 384:onthefly"}
for cfg in $CFGS; do
  set -- ${cfg/:/ }
  # first call of a new batch size: conv autotune + MIOpen find + graph capture (minutes at 192+)
  timeout -k 10 700 python bench.py --batch $1 --corr_mode $2 --steps 5 --warmup 2 > gpurun_out/sweep/train_b$1_$2.log 2>&1 || { tail -3 gpurun_out/sweep/train_b$1_$2.log; exit 1; }
  echo "b$1 $2: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*\|"peak_reserved_gib_rank0": [0-9.]*' gpurun_out/sweep/train_b$1_$2.log | tr '\n' ' ')"
done
