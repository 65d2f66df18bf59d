#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
O=gpurun_out/diag; mkdir -p $O
for t in 0 1; do
  RAFT_BUILD_DEEP=$t timeout -k 10 120 python -u scripts/bench_lookup.py > $O/build_deep$t.txt 2>&1 || { tail -5 $O/build_deep$t.txt; exit 1; }
  echo "deep=$t: $(grep -h us $O/build_deep$t.txt | tr '\n' ' ')"
done
timeout -k 10 300 python -u -m pytest -q -x --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "build or allpairs" > $O/pytest_build.log 2>&1
rc=$?; tail -n 1 $O/pytest_build.log; grep -E "^E  .*Error|FAILED" $O/pytest_build.log | head
exit $rc
