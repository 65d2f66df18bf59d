#!/bin/bash
# session-3 iteration: full GPU suite, bench, steady-state profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | cut -c1-300
if [ "$1" != "" ]; then
  bash scripts/gpu_profile.sh $1 && python scripts/categorize.py gpurun_out/$1_summary.txt > gpurun_out/$1_categories.txt
  cat gpurun_out/$1_categories.txt
fi
