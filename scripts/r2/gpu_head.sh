#!/bin/bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_encoder_gpu.py tests/test_graph_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/head_pytest.log 2>&1
echo "pytest rc=$?"; tail -3 gpurun_out/head_pytest.log; grep -E "^E  |FAILED" gpurun_out/head_pytest.log | head
timeout -k 10 250 python -u scripts/r2/diag_poison.py graph_cmp > gpurun_out/cmp2.log 2>&1; grep replay gpurun_out/cmp2.log | cut -c1-700
timeout -k 10 250 python -u scripts/r2/diag_poison.py graph > gpurun_out/g2.log 2>&1; grep "graph" gpurun_out/g2.log | cut -c1-400
