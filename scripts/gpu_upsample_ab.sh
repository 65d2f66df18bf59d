#!/bin/bash
# convex-upsample kernel check: upsample + model GPU tests, bench, step profile -> gpurun_out/up_*
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_fp16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/up_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/up_pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/up_pytest.log | head; exit $rc; }
timeout -k 10 300 python bench.py > gpurun_out/up_bench.log 2>&1 || { tail -3 gpurun_out/up_bench.log; exit 1; }
grep -o '"value": [0-9.]*' gpurun_out/up_bench.log
bash scripts/gpu_profile.sh up > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/up_summary.txt > gpurun_out/up_categories.txt
grep -E "convex|seq_loss" gpurun_out/up_summary.txt | cut -c1-130
grep -E "upsample|total" gpurun_out/up_categories.txt
