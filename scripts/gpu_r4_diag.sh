#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_update_hip_gpu.py tests/test_model_gpu.py tests/test_graph_gpu.py tests/test_conv_gpu.py > $O/pytest_ctx.log 2>&1
rc=$?; tail -n 1 $O/pytest_ctx.log; grep -E "^E  .*Error|FAILED" $O/pytest_ctx.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py > $O/bench_ctx.log 2>&1 || { tail -3 $O/bench_ctx.log; exit 1; }
echo "bf16 ctx: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench_ctx.log | tr '\n' ' ')"
RAFT_CTX_BF16=0 timeout -k 10 300 python bench.py > $O/bench_ctx32.log 2>&1 || { tail -3 $O/bench_ctx32.log; exit 1; }
echo "fp32 ctx: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench_ctx32.log | tr '\n' ' ')"
