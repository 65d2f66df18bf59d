#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -x -q > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_conv.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_graph.log 2>&1
rc=$?; tail -3 gpurun_out/bench_graph.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --alternate_corr > gpurun_out/bench_graph_alt.log 2>&1
rc=$?; tail -3 gpurun_out/bench_graph_alt.log | cut -c1-600
exit $rc
