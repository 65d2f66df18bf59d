#!/bin/bash
# A/B: channels_last encoders; profile it
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 3 --channels_last > gpurun_out/bench_cl.log 2>&1
rc=$?; tail -1 gpurun_out/bench_cl.log | cut -c1-300
if [ $rc -ne 0 ]; then exit $rc; fi
bash scripts/gpu_profile.sh cl --channels_last
