#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 700 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_optim_gpu.py > $O/pytest_adam.log 2>&1
rc=$?; tail -n 1 $O/pytest_adam.log; grep -E "^E  .*Error|FAILED" $O/pytest_adam.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench_adam.log 2>&1 || { tail -3 $O/bench_adam.log; exit 1; }
echo "fused adamw: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench_adam.log | tr '\n' ' ')"
