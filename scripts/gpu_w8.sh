#!/bin/bash
# 8-wave conv kernel check: forced-config tests, per-layer config sweep (+ zero-memory floor)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-w8}
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q -k "halo" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python scripts/conv_cfg_sweep.py all 16,25,30,38,39,43,44 > gpurun_out/${TAG}_sweep.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_sweep.txt
RAFT_CONV_NULLMEM=1 timeout -k 10 300 python scripts/conv_cfg_sweep.py zr1,c2,head 16,38,43,44 > gpurun_out/${TAG}_sweep_nullmem.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_sweep_nullmem.txt
PYTHONPATH=. timeout -k 10 120 python scripts/gemm_ref.py > gpurun_out/${TAG}_gemm_ref.txt 2>&1
cat gpurun_out/${TAG}_gemm_ref.txt
