#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -x -q > gpurun_out/pytest_conv.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_conv.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python scripts/bench_conv.py > gpurun_out/bench_conv.log 2>&1
rc=$?; cat gpurun_out/bench_conv.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh hip
