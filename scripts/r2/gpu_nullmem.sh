#!/bin/bash
# update-block conv timings per layer: real operands vs loads-return-zero (RAFT_CONV_NULLMEM=1)
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
timeout -k 10 300 python scripts/r2/conv_bench.py all 20 > gpurun_out/nullmem_0.log 2>&1 || exit 1
RAFT_CONV_NULLMEM=1 timeout -k 10 300 python scripts/r2/conv_bench.py all 20 > gpurun_out/nullmem_1.log 2>&1 || exit 1
cat gpurun_out/nullmem_0.log gpurun_out/nullmem_1.log
