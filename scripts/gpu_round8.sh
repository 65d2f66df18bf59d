#!/bin/bash
# on-the-fly MFMA correlation: numerics, model parity, bench (all-pairs vs alternate), profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_kernels_gpu.py -k "onthefly" -x -q > gpurun_out/pytest_otf.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_otf.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -m pytest tests/test_model_gpu.py -x -q > gpurun_out/pytest_model.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_model.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --alternate_corr > gpurun_out/bench_alt.log 2>&1
rc=$?; tail -1 gpurun_out/bench_alt.log | cut -c1-600
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh alt --alternate_corr
