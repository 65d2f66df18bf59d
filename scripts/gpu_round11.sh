#!/bin/bash
# fused channels-last encoder: numerics, then bench + profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_encoder_gpu.py -q > gpurun_out/pytest_enc.log 2>&1
rc=$?; tail -15 gpurun_out/pytest_enc.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_all.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_all.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_fused.log 2>&1
rc=$?; tail -1 gpurun_out/bench_fused.log | cut -c1-400
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh fused && python scripts/categorize.py gpurun_out/fused_summary.txt
