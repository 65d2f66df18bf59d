#!/bin/bash
# session-3 iteration: selected GPU tests, full GPU suite, bench, inference bench
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_update_hip_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_update.log 2>&1
rc=$?; tail -12 gpurun_out/pytest_update.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -4 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | cut -c1-300
for extra in "" "--graph"; do
  timeout -k 10 300 python bench_infer.py --batch 16 --steps 5 --warmup 2 $extra > gpurun_out/bench_infer$extra.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_infer$extra.log
done
timeout -k 10 300 python bench_infer.py --batch 16 --steps 3 --warmup 1 --impl torch > gpurun_out/bench_infer_torch.log 2>&1 || exit $?
tail -1 gpurun_out/bench_infer_torch.log
