#!/bin/bash
# final tree check: every GPU test + smoke() + one bench run
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/final_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/final_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/final_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
timeout -k 10 300 python bench.py > gpurun_out/final_bench.log 2>&1 || exit 1
grep metric gpurun_out/final_bench.log | cut -c1-260
