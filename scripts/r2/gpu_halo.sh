#!/bin/bash
# halo-tile conv kernel: correctness (forced configs), per-layer timings, then the full cycle
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-halo}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_conv_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_conv_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/${TAG}_conv_pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python scripts/r2/conv_bench.py all 20 > gpurun_out/${TAG}_convbench.log 2>&1 || exit 1
RAFT_CONV_HALO=0 timeout -k 10 300 python scripts/r2/conv_bench.py all 20 > gpurun_out/${TAG}_convbench_nohalo.log 2>&1 || exit 1
cat gpurun_out/${TAG}_convbench.log gpurun_out/${TAG}_convbench_nohalo.log
bash scripts/r2/gpu_cycle.sh ${TAG}
