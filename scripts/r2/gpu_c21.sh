#!/bin/bash
# round-end style cycle: every GPU test, smoke(), bench x2, RAFT-small bench, steady-state profile
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
T=c21
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 280 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1
rc=$?
tail -3 gpurun_out/${T}_pytest.log
if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${T}_pytest.log | head -30; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${T}_smoke.log 2>&1 || { tail -5 gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
for r in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${T}_bench_rep$r.log 2>&1 || exit 1
  grep metric gpurun_out/${T}_bench_rep$r.log | cut -c1-300
done
timeout -k 10 300 python bench.py --small --steps 10 --warmup 3 > gpurun_out/${T}_small.log 2>&1 || exit 1
grep -o '"value[^,]*' gpurun_out/${T}_small.log
bash scripts/gpu_profile.sh ${T} > /dev/null 2>&1
python scripts/categorize.py gpurun_out/${T}_summary.txt > gpurun_out/${T}_categories.txt 2>&1
head -3 gpurun_out/${T}_summary.txt; cat gpurun_out/${T}_categories.txt
# fp32 (reference paper-schedule numerics), graphed decode: MIOpen's exhaustive search of the fp32
# encoder convs takes ~10 min on a fresh box before the first step
timeout -k 10 1000 python bench.py --precision fp32 --steps 20 --warmup 3 > gpurun_out/${T}_fp32_graph.log 2>&1 || { tail -3 gpurun_out/${T}_fp32_graph.log; exit 1; }
grep -o '"value[^,]*\|"ms_per_step[^,]*\|"loss_finite[^,]*\|"hipgraph[^,]*' gpurun_out/${T}_fp32_graph.log
