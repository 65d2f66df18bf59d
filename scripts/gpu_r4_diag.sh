#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_update_hip_gpu.py tests/test_graph_gpu.py tests/test_dp_gpu.py > $O/pytest_carry.log 2>&1
rc=$?; tail -n 1 $O/pytest_carry.log; grep -E "^E  .*Error|FAILED" $O/pytest_carry.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench_carry.log 2>&1 || { tail -3 $O/bench_carry.log; exit 1; }
echo "bench: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench_carry.log | tr '\n' ' ')"
