#!/bin/bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
: > gpurun_out/poison.log
for m in poison poison_alt graph graph graph_nobench; do
  timeout -k 10 200 python -u scripts/r2/diag_poison.py $m >> gpurun_out/poison.log 2>&1
  rc=$?
  echo "$m rc=$rc" >> gpurun_out/poison.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then break; fi
done
grep -v amdgpu gpurun_out/poison.log | cut -c1-400
