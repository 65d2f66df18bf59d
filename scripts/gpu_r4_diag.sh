#!/bin/bash
# Targeted GPU check: bisect the split-bf16 fp32 encoder against fp64.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
timeout -k 10 200 python -u scripts/diag_fp32_enc2.py > $O/diag_enc.txt 2>&1 || { tail -5 $O/diag_enc.txt; exit 1; }
cat $O/diag_enc.txt
