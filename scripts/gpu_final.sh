#!/bin/bash
# round-end style check of the final tree: every GPU test + smoke + bench (x2) + step profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-final}
mkdir -p gpurun_out
# liveness for long steps (MIOpen searches, multi-process tests): the per-step timeouts below
# bound real hangs
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -5 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -n 1 gpurun_out/${TAG}_smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench$i.log 2>&1 || { tail -3 gpurun_out/${TAG}_bench$i.log; exit 1; }
  grep metric gpurun_out/${TAG}_bench$i.log | cut -c1-300
done
bash scripts/gpu_profile.sh ${TAG} > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt
cat gpurun_out/${TAG}_categories.txt
