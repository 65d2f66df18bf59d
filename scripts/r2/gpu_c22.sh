#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_fp32_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/c22_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/c22_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/c22_pytest.log | head -20; exit $rc; fi
timeout -k 10 900 python bench.py --precision fp32 --steps 20 --warmup 3 > gpurun_out/c22_fp32_graph.log 2>&1 || { tail -3 gpurun_out/c22_fp32_graph.log; exit 1; }
grep -o '"value[^,]*\|"ms_per_step[^,]*\|"loss_finite[^,]*\|"hipgraph[^,]*' gpurun_out/c22_fp32_graph.log
