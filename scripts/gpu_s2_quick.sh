#!/bin/bash
# quick kernel iteration: numerics, conv PMC sweep (optional), microbench, full bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_model_gpu.py tests/test_update_hip_gpu.py tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_iter.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ -n "$PMC_LAYER" ]; then bash scripts/gpu_pmc_conv2.sh $PMC_LAYER $PMC_CFGS || exit $?; fi
timeout -k 10 200 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || exit $?
cat gpurun_out/bench_conv.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('eager', d['value'], d['ms_per_step'], d['host_issue_ms'])"
