#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_s3_var.sh
bash scripts/gpu_profile.sh ${1:-t2} > /dev/null && python scripts/categorize.py gpurun_out/${1:-t2}_summary.txt > gpurun_out/${1:-t2}_categories.txt
cat gpurun_out/${1:-t2}_categories.txt | head -8
grep -c "CUDAFunctor_add<c10::BFloat16>" gpurun_out/${1:-t2}_summary.txt || true
