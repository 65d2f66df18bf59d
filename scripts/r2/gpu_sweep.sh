#!/bin/bash
# batch sweep (training pairs/s + peak HBM, all-pairs and on-the-fly), config-5 large-batch Sintel
# inference, on-the-fly under large / discontinuous lookup coordinates
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
O=gpurun_out/sweep
mkdir -p $O
j() { grep -o '"value[^,]*\|"ms_per_step[^,]*\|"peak_hbm[^,]*\|"loss_finite[^,]*\|"finite[^,]*' $1 | tr '\n' ' '; }
for b in 12 24 48 96; do
  for c in "ap:" "otf:--alternate_corr"; do
    n=${c%%:*}; f=${c#*:}
    timeout -k 10 400 python bench.py --batch $b --steps 10 --warmup 3 $f > $O/train_b${b}_$n.log 2>&1 || { echo "train b$b $n failed"; tail -5 $O/train_b${b}_$n.log; exit 1; }
    echo "train b$b $n $(j $O/train_b${b}_$n.log)"
  done
done
