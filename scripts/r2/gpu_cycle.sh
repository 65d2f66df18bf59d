#!/bin/bash
# standard build->measure cycle: all GPU tests, bench (graphed default), steady-state kernel profile
# usage: gpu_cycle.sh <tag> [pytest selection]
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
TAG=${1:-cyc}
SEL=${2:-tests}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest $SEL -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
tail -4 gpurun_out/${TAG}_pytest.log
if [ $rc -ne 0 ]; then grep -E "Error|assert|FAILED" gpurun_out/${TAG}_pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
grep metric gpurun_out/${TAG}_bench.log | cut -c1-330
bash scripts/gpu_profile.sh ${TAG} > /dev/null 2>&1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt 2>&1
head -3 gpurun_out/${TAG}_summary.txt; cat gpurun_out/${TAG}_categories.txt
