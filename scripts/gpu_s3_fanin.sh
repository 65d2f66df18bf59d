#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for f in 24 48 96; do
  RAFT_WG_FANIN=$f timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_fanin$f.log 2>&1 || exit $?
  echo "fanin $f: $(tail -1 gpurun_out/bench_fanin$f.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
