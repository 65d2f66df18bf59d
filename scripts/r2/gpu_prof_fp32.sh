#!/bin/bash
# steady-state kernel profile of the fp32 (graphed) training step
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 1050 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_fp32 -o run -- python bench.py --precision fp32 --steps 3 --warmup 2 --trace_markers > gpurun_out/fp32_prof_bench.log 2>&1
echo "rocprof rc=$?"
python scripts/prof_diff.py --markers /tmp/prof_fp32 3 > gpurun_out/fp32_summary.txt 2>&1
python scripts/categorize.py gpurun_out/fp32_summary.txt > gpurun_out/fp32_categories.txt 2>&1
head -25 gpurun_out/fp32_summary.txt | cut -c1-160; cat gpurun_out/fp32_categories.txt
