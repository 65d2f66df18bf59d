#!/bin/bash
# fp16 / fp32 / RAFT-small benches of the current build -> gpurun_out/prec_*.log
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
for cfg in "fp16:--precision fp16" "fp32:--precision fp32" "small:--small" "small_fp16:--small --precision fp16"; do
  tag=${cfg%%:*}; args=${cfg#*:}
  timeout -k 10 400 python bench.py $args > gpurun_out/prec_$tag.log 2>&1 || { echo "$tag failed"; tail -3 gpurun_out/prec_$tag.log; exit 1; }
  echo "$tag $(grep -o '"value": [0-9.]*' gpurun_out/prec_$tag.log) $(grep -o '"hipgraph": [a-z]*' gpurun_out/prec_$tag.log)"
done
