#!/bin/bash
# rocprofv3 --kernel-trace --stats, steady state by differencing two runs (warmup only vs warmup+K).
# usage: gpu_profile.sh <tag> [bench args...]   -> gpurun_out/<tag>_summary.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-prof}; shift
mkdir -p gpurun_out
K=4
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${TAG}_a -o run -- python bench.py --steps 1 --warmup 3 "$@" > gpurun_out/${TAG}_bench_a.log 2>&1 && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_${TAG}_b -o run -- python bench.py --steps $((K+1)) --warmup 3 "$@" > gpurun_out/${TAG}_bench_b.log 2>&1
rc=$?
echo "rocprof rc=$rc"
python scripts/prof_diff.py /tmp/prof_${TAG}_a /tmp/prof_${TAG}_b $K > gpurun_out/${TAG}_summary.txt 2>&1
head -40 gpurun_out/${TAG}_summary.txt | cut -c1-180
exit $rc
