#!/bin/bash
# host-side issue cost: same kernel/launch count as the chairs bench, negligible GPU work
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 1 --size 128 128 > gpurun_out/bench_host.log 2>&1
rc=$?; tail -1 gpurun_out/bench_host.log | cut -c1-900
exit $rc
