#!/bin/bash
# round-4 iteration check: the tests touched by a change + bench + phase-split step profile
# usage: gpu_r4.sh <tag> [pytest files...]
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4}; shift
mkdir -p gpurun_out/miopen_db
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
  rc=$?; tail -n 2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | grep -v "amdgpu.ids" | head -20; exit $rc; fi
fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -3 gpurun_out/${TAG}_bench.log; exit 1; }
grep metric gpurun_out/${TAG}_bench.log | cut -c150-330
bash scripts/gpu_profile.sh ${TAG} > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt
cat gpurun_out/${TAG}_categories.txt
