#!/bin/bash
# Every GPU test (up to 10 failures reported, not stopping at the first) + smoke().
#   usage: gpu_full.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-full}
O=gpurun_out/$TAG
mkdir -p $O gpurun_out/miopen_db
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=10 -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
rc=$?
tail -n 3 $O/pytest.log
grep -E "^FAILED|^ERROR" $O/pytest.log | head -20
# 1 = failed tests (still run smoke); anything else (timeout, crash) ends the call
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
exit $rc
