#!/bin/bash
# torch.profiler op-level attribution of one eager training step
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/tprof
timeout -k 10 300 python bench.py --steps 2 --warmup 3 --profile gpurun_out/tprof > gpurun_out/tprof/bench.log 2>&1 || exit $?
head -70 gpurun_out/tprof/ops.txt | cut -c1-200
