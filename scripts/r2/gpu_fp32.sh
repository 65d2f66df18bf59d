#!/bin/bash
# fp32 training step (reference paper schedule numerics): split-bf16 MFMA update-block convs;
# MIOpen's exhaustive search of the fp32 encoder convs takes ~10 min on a fresh box
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out/c20
timeout -k 10 1000 python bench.py --precision fp32 --steps 20 --warmup 3 > gpurun_out/c20/fp32_split.log 2>&1 || { tail -3 gpurun_out/c20/fp32_split.log; exit 1; }
grep metric gpurun_out/c20/fp32_split.log | cut -c1-400
