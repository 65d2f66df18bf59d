#!/bin/bash
# rocprofv3 kernel-trace + stats of the bench's TIMED steps only (roctx-selected region),
# summarised into gpurun_out/<tag>_summary.txt.   usage: gpu_profile.sh <tag> [bench args...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-prof}; shift
mkdir -p gpurun_out
timeout -k 10 600 rocprofv3 --selected-regions --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- python bench.py --steps 3 --warmup 3 --roctx_region "$@" > gpurun_out/${TAG}_bench.log 2>&1
rc=$?
echo "rocprof rc=$rc"
tail -1 gpurun_out/${TAG}_bench.log
python scripts/summarize_prof.py /tmp/prof_$TAG > gpurun_out/${TAG}_summary.txt 2>&1
head -45 gpurun_out/${TAG}_summary.txt
exit $rc
