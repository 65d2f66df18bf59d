#!/bin/bash
# Steady-state per-kernel profile of the timed bench steps only: bench brackets its K timed steps
# with a marker spin kernel (--trace_markers) and prof_diff.py --markers aggregates exactly the
# kernels between them (no MIOpen solver search, no warm-up / capture kernels in the table).
# usage: gpu_profile.sh <tag> [bench args...]   -> gpurun_out/<tag>_summary.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-prof}; shift
mkdir -p gpurun_out
K=4
RAFT_PHASE_MARKS=1 timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_${TAG} -o run -- python bench.py --steps $K --warmup 3 --trace_markers "$@" > gpurun_out/${TAG}_prof_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
python scripts/prof_diff.py --phases /tmp/prof_${TAG} $K > gpurun_out/${TAG}_summary.txt 2>&1
head -40 gpurun_out/${TAG}_summary.txt | cut -c1-180
exit $rc
