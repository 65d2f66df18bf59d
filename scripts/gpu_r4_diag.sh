#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
for t in 4 8; do
  RAFT_LOOKUP_TPV=$t timeout -k 10 120 python -u scripts/bench_lookup.py > $O/lookup_$t.txt 2>&1 || { tail -5 $O/lookup_$t.txt; exit 1; }
  echo "tpv $t: $(grep us $O/lookup_$t.txt)"
done
RAFT_LOOKUP_TPV=4 timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "lookup" > $O/pytest_lookup8.log 2>&1
rc=$?; tail -n 1 $O/pytest_lookup8.log; grep -E "^E  .*Error|FAILED" $O/pytest_lookup8.log | head
exit $rc
