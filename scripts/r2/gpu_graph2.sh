#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_graph_gpu.py tests/test_dp_gpu.py -x -v -s --timeout 280 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1 || { tail -40 gpurun_out/pytest_graph.log; exit 1; }
grep -E "PASS|FAIL|dp rehearsal" gpurun_out/pytest_graph.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_graph.log 2>&1 || exit 1
grep metric gpurun_out/bench_graph.log
