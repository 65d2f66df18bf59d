#!/bin/bash
# Round-2 first contact: GPU tests, eager bench, hipGraph bench.
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_eager.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --hipgraph > gpurun_out/bench_graph.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -3 gpurun_out/bench_eager.log; tail -3 gpurun_out/bench_graph.log
exit $rc
