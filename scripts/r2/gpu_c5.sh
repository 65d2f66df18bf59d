#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
bash scripts/gpu_profile.sh c5 || exit 1
python scripts/categorize.py gpurun_out/c5_summary.txt > gpurun_out/c5_categories.txt 2>&1
cat gpurun_out/c5_categories.txt
bash scripts/r2/pmc_step.sh s1
