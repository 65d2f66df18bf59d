#!/bin/bash
# large-batch training (B=<per-GPU batch>, EXTRA=<bench flags>): Python stacks every 120 s (RAFT_STACK_DUMP)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/large gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
RAFT_STACK_DUMP=120 timeout -k 10 540 python -u bench.py --batch ${B:-192} --steps 3 --warmup 1 $EXTRA > gpurun_out/large/b${B:-192}.log 2>&1
echo "large-batch rc=$?"
grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"peak_hbm_gib_rank0": [0-9.]*' gpurun_out/large/b${B:-192}.log | tr '\n' ' '
exit 0
