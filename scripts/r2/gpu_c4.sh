#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_update_hip_gpu.py tests/test_kernels_gpu.py -m gpu -x -q -s --timeout 280 --timeout-method thread > gpurun_out/c4_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/c4_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|bad" gpurun_out/c4_pytest.log | head -30; fi
bash scripts/gpu_profile.sh c4alt --alternate_corr > gpurun_out/c4_prof.log 2>&1
python scripts/categorize.py gpurun_out/c4alt_summary.txt > gpurun_out/c4alt_categories.txt 2>&1
cat gpurun_out/c4alt_categories.txt
timeout -k 10 900 python bench.py --steps 50 --warmup 10 --impl torch --precision fp32 > gpurun_out/c4_stock_fp32.log 2>&1 || exit 1
grep metric gpurun_out/c4_stock_fp32.log | cut -c1-300
