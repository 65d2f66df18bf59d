#!/bin/bash
# Targeted GPU check: correlation fold variants (timing + tests), then the bench.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
for m in 1 0; do
  RAFT_TAPRED=$m timeout -k 10 120 python -u scripts/bench_tapred.py > $O/tapred_$m.txt 2>&1 || { tail -5 $O/tapred_$m.txt; exit 1; }
  echo "mode $m: $(grep us $O/tapred_$m.txt)"
done
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "tap_reduce or lookup" > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; grep -E "^E  .*Error|FAILED" $O/pytest.log | head -20
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -3 $O/bench.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench.log | tr '\n' ' '
