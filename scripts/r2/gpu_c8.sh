#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/c8_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/c8_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E  |FAILED" gpurun_out/c8_pytest.log | head -20; exit $rc; fi
for v in "graph:" "eager:--eager" "alt:--alternate_corr" "alt_eager:--alternate_corr --eager"; do
  n=${v%%:*}; a=${v#*:}
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 $a > gpurun_out/c8_bench_$n.log 2>&1 || exit 1
  echo "$n $(grep -o '"value[^,]*\|"ms_per_step[^,]*\|"loss_finite[^,]*\|"host_issue_ms[^,]*\|"peak_hbm[^,]*' gpurun_out/c8_bench_$n.log | tr '\n' ' ')"
done
