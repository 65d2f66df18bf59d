#!/bin/bash
# run-to-run variance of the headline bench (fresh process each time: autotune + MIOpen find)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_var$k.log 2>&1 || exit $?
  tail -1 gpurun_out/bench_var$k.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
done
