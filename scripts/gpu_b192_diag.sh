#!/bin/bash
# where does the batch-192 training step's first call spend its time?  Python stacks every 60 s
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/b192 gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
RAFT_STACK_DUMP=120 timeout -k 10 540 python -u bench.py --batch ${B:-192} --steps 3 --warmup 1 $EXTRA > gpurun_out/b192/b${B:-192}.log 2>&1
echo "b192 rc=$?"
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*' gpurun_out/b192/b${B:-192}.log | tr '\n' ' '
exit 0
