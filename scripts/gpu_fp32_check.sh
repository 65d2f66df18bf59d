#!/bin/bash
# fp32 path check: fp32 conv / graph tests, then the fp32 bench + op table (MIOpen db from miopen_db/)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-f32}
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 600 python -u -m pytest tests/test_conv_fp32_gpu.py tests/test_graph_gpu.py -x -q --timeout 500 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 900 python bench.py --precision fp32 --warmup 3 --steps 5 --profile gpurun_out/${TAG}_torchprof > gpurun_out/${TAG}_bench.log 2>&1 || { tail -5 gpurun_out/${TAG}_bench.log; exit 1; }
grep metric gpurun_out/${TAG}_bench.log | cut -c1-300
head -45 gpurun_out/${TAG}_torchprof/ops.txt | cut -c1-180
