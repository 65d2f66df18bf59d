#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tr_upd -o run -- python scripts/trace_update.py > gpurun_out/trace_update_run.log 2>&1 || exit $?
python scripts/trace_update.py --parse /tmp/tr_upd > gpurun_out/trace_update.txt 2>&1
cat gpurun_out/trace_update.txt
