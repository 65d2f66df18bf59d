#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_conv_fp32_gpu.py tests/test_graph_gpu.py > $O/pytest_fix.log 2>&1
rc=$?; tail -n 1 $O/pytest_fix.log; grep -E "^E  .*Error|FAILED" $O/pytest_fix.log | head
exit $rc
