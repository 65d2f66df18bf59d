#!/bin/bash
# conv kernel iteration: numerics (conv + update block + model), microbench, full bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py tests/test_model_gpu.py tests/test_update_hip_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_conv.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 200 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1 || exit $?
cat gpurun_out/bench_conv.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | cut -c1-400
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; exit $rc
