#!/bin/bash
# fp32 (paper-schedule) step: where the time goes (torch.profiler op table; MIOpen fast find so the
# fresh box does not spend ~10 min in the exhaustive fp32 solver search)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp MIOPEN_FIND_MODE=2
mkdir -p gpurun_out
timeout -k 10 500 python bench.py --precision fp32 --warmup 3 --steps 3 --profile gpurun_out/fp32_torchprof > gpurun_out/fp32_bench.log 2>&1 || { tail -5 gpurun_out/fp32_bench.log; exit 1; }
grep metric gpurun_out/fp32_bench.log | cut -c1-300
head -60 gpurun_out/fp32_torchprof/ops.txt | cut -c1-220
