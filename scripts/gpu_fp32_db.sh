#!/bin/bash
# fp32 step with MIOpen's find / perf databases written under gpurun_out/miopen_db (shipped back in
# the tree as miopen_db/ so later fp32 runs skip the ~10 min solver search), + torch.profiler table
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 1000 python bench.py --precision fp32 --warmup 3 --steps 3 --profile gpurun_out/fp32_torchprof > gpurun_out/fp32_bench.log 2>&1 || { tail -5 gpurun_out/fp32_bench.log; exit 1; }
grep metric gpurun_out/fp32_bench.log | cut -c1-300
grep -c alive gpurun_out/fp32_bench.log
ls -la gpurun_out/miopen_db
head -50 gpurun_out/fp32_torchprof/ops.txt | cut -c1-200
