#!/bin/bash
# session-2 re-entry check: GPU tests, bench (eager / hipgraph / on-the-fly corr), conv microbench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --hipgraph > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_graph.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --alternate_corr > gpurun_out/bench_alt.log 2>&1 || exit $?
tail -1 gpurun_out/bench_alt.log | cut -c1-300
timeout -k 10 200 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || exit $?
cat gpurun_out/bench_conv.log
