#!/bin/bash
# First-contact GPU run: kernel numerics, model parity, stock baseline vs HIP path.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/pytest_gpu.log
tail -5 gpurun_out/pytest_gpu.log
# only plain test failures (rc 1) may be followed by more GPU work
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 5 --warmup 3 --impl torch > gpurun_out/bench_torch.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 10 --warmup 3 > gpurun_out/bench_hip.log 2>&1
rc=$?
echo "bench rc=$rc"
tail -2 gpurun_out/bench_torch.log; tail -2 gpurun_out/bench_hip.log
exit $rc
