#!/bin/bash
# transposed GRU epilogue: DP graph rehearsal metrics + the remaining GPU tests
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
RAFT_DIST_BACKEND=gloo timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29533 scripts/dp_rehearsal.py --graph > gpurun_out/gru_dp.log 2>&1
echo "dp rc=$?"; grep -o "dp rehearsal.*" gpurun_out/gru_dp.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread \
  --deselect "tests/test_dp_gpu.py::test_dp_rehearsal[graph]" > gpurun_out/gru_pytest2.log 2>&1
rc=$?; tail -n 2 gpurun_out/gru_pytest2.log; grep -E "^E |FAILED" gpurun_out/gru_pytest2.log | head -20; exit $rc
