#!/bin/bash
# halo conv kernel: forced-config correctness, per-config sweep, update-block tests, bench
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-halo2}
mkdir -p gpurun_out
timeout -k 10 120 python scripts/r2/dbg_halo.py > gpurun_out/${TAG}_dbg.log 2>&1; grep -c "nbad 0" gpurun_out/${TAG}_dbg.log; timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_conv_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${TAG}_conv_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/${TAG}_conv_pytest.log | head -30; exit $rc; fi
timeout -k 10 400 python scripts/r2/conv_cfg_sweep.py all > gpurun_out/${TAG}_cfgsweep.log 2>&1 || exit 1
cat gpurun_out/${TAG}_cfgsweep.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
grep metric gpurun_out/${TAG}_bench.log | cut -c1-330
