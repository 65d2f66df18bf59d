#!/bin/bash
# fp32-accurate on-the-fly backward tests, then the remaining BASELINE configs.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "onthefly" > $O/pytest_otf.log 2>&1
rc=$?; tail -n 2 $O/pytest_otf.log; grep -E "^E  .*Error|FAILED" $O/pytest_otf.log | head -20
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash scripts/gpu_configs_r4.sh things small chairs_otf infer
