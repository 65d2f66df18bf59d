#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_update_hip_gpu.py -m gpu -x -q -s -k small --timeout 280 --timeout-method thread > gpurun_out/c6_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/c6_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|bad|line" gpurun_out/c6_pytest.log | head -40; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/c6_bench.log 2>&1
grep metric gpurun_out/c6_bench.log | grep -o '"loss_finite.*'
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --small > gpurun_out/c6_bench_small.log 2>&1
grep metric gpurun_out/c6_bench_small.log | cut -c1-250
bash scripts/gpu_profile.sh c6 > gpurun_out/c6_prof.log 2>&1
python scripts/categorize.py gpurun_out/c6_summary.txt > gpurun_out/c6_categories.txt 2>&1
head -3 gpurun_out/c6_summary.txt; cat gpurun_out/c6_categories.txt
bash scripts/r2/pmc_step.sh s2
