#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp PYTHONPATH=.
O=gpurun_out/diag; mkdir -p $O
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_encoder_gpu.py > $O/pytest_enc.log 2>&1
rc=$?; tail -n 1 $O/pytest_enc.log; grep -E "^E  .*Error|FAILED" $O/pytest_enc.log | head
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for u in 1 4; do
  RAFT_NORM_UNROLL=$u timeout -k 10 300 python bench.py > $O/bench_u$u.log 2>&1 || { tail -3 $O/bench_u$u.log; exit 1; }
  echo "norm unroll=$u: $(grep -o '"ms_per_step": [0-9.]*\|"value": [0-9.]*' $O/bench_u$u.log | tr '\n' ' ')"
done
for u in 1 4; do
  RAFT_NORM_UNROLL=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st_u$u -o run -- python bench.py --steps 4 --warmup 3 > $O/st_u$u.log 2>&1 || { tail -3 $O/st_u$u.log; exit 1; }
  f=$(find $O/st_u$u -name "*kernel_stats.csv" | head -1)
  echo "u=$u"; grep -E "norm_apply|norm_bwd_apply|relu_mask" $f | cut -d, -f1-4 | cut -c1-160
done
