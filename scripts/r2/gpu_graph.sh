#!/bin/bash
# graph-step GPU test, graph vs eager bench, steady-state kernel profile of the graphed step
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_graph_gpu.py -x -v --timeout 240 --timeout-method thread > gpurun_out/pytest_graph.log 2>&1 || { tail -30 gpurun_out/pytest_graph.log; exit 1; }
tail -4 gpurun_out/pytest_graph.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_graph.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --eager > gpurun_out/bench_eager.log 2>&1 || exit 1
grep metric gpurun_out/bench_graph.log gpurun_out/bench_eager.log
bash scripts/gpu_profile.sh graph
