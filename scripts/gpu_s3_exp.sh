#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_sel.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 3 > gpurun_out/bench_eager.log 2>&1 || exit $?
tail -1 gpurun_out/bench_eager.log | cut -c1-200
bash scripts/gpu_profile.sh ${1:-s9} > /dev/null && python scripts/categorize.py gpurun_out/${1:-s9}_summary.txt > gpurun_out/${1:-s9}_categories.txt
grep -E "window_reduce|steady" gpurun_out/${1:-s9}_summary.txt | cut -c1-120
