#!/bin/bash
# kernel iteration: conv/model numerics, bench (eager + hipgraph), steady-state profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-iter}
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_model_gpu.py tests/test_update_hip_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', d['value'], d['ms_per_step'], d['host_issue_ms'])"
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --hipgraph > gpurun_out/bench_graph.log 2>&1 || exit $?
tail -1 gpurun_out/bench_graph.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph', d['value'], d['ms_per_step'], d['host_issue_ms'])"
bash scripts/gpu_profile.sh $TAG > /dev/null && python scripts/categorize.py gpurun_out/${TAG}_summary.txt && head -25 gpurun_out/${TAG}_summary.txt | cut -c1-150
