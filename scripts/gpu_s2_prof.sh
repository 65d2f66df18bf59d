#!/bin/bash
# bench eager vs hipgraph + steady-state kernel profile of the eager step
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --hipgraph > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_graph.log | cut -c1-200; tail -1 gpurun_out/bench_graph.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_issue_ms'])"
bash scripts/gpu_profile.sh ${1:-s2} && python scripts/categorize.py gpurun_out/${1:-s2}_summary.txt
