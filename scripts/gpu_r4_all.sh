#!/bin/bash
# One GPU call that does everything a build needs checked: every GPU test, smoke, the bench, a
# phase-split kernel profile, a stack-attributed op profile, a per-dispatch trace of one update
# block iteration, the step's MFMA PMC pass and the precision / KITTI configs.  Steps are chained:
# the first failure ends the call (failed test assertions excepted).   usage: [CONFIGS='fp32 fp16 ...'] gpu_r4_all.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r4}
mkdir -p gpurun_out/miopen_db gpurun_out/$TAG
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
O=gpurun_out/$TAG
step() { echo "== $1 $(date +%T)"; }
step pytest
timeout -k 10 900 python -u -m pytest tests -m gpu --maxfail=4 -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 2 $O/pytest.log; [ $rc -ne 0 ] && grep -E "^E |FAILED" $O/pytest.log | grep -v amdgpu.ids | head -20
# rc 1 = failed assertions (read the log, the rest of the call still runs); anything else (a
# timeout, a crash, a fault) ends the call here
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
step smoke
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -n 3 $O/smoke.log
step bench
timeout -k 10 300 python bench.py > $O/bench.log 2>&1 || { tail -3 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c150-330
step profile
RAFT_PHASE_MARKS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_$TAG -o run -- python bench.py --steps 4 --warmup 3 --trace_markers > $O/prof_bench.log 2>&1 || { tail -3 $O/prof_bench.log; exit 1; }
python scripts/prof_diff.py --phases /tmp/prof_$TAG 4 > $O/summary.txt 2>&1
python scripts/categorize.py $O/summary.txt > $O/categories.txt
cat $O/categories.txt
step stack
timeout -k 10 300 python bench.py --eager --steps 2 --warmup 3 --profile $O/torchprof --profile_stack > $O/stack_bench.log 2>&1 || { tail -3 $O/stack_bench.log; exit 1; }
step trace_update
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tu_$TAG -o run -- python scripts/trace_update.py > $O/trace_update_run.log 2>&1 || { tail -3 $O/trace_update_run.log; exit 1; }
python scripts/trace_update.py --parse /tmp/tu_$TAG > $O/trace_update.txt 2>&1
tail -n 1 $O/trace_update.txt
step pmc
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
timeout -s KILL 300 rocprofv3 --pmc $P1 --kernel-trace --output-format csv -d /tmp/pmc_${TAG}_1 -o run -- python bench.py --steps 2 --warmup 2 --trace_markers > $O/pmc1.log 2>&1 || { tail -3 $O/pmc1.log; exit 1; }
python scripts/pmc_summary.py /tmp/pmc_${TAG}_1 /tmp/pmc_${TAG}_1 /tmp/pmc_${TAG}_1 2 > $O/pmc_sq.txt 2>&1 || true
head -3 $O/pmc_sq.txt
if [ -n "$CONFIGS" ]; then
  step configs
  bash scripts/gpu_configs_r4.sh $CONFIGS
  cp -r gpurun_out/cfg4 $O/ 2>/dev/null
fi
step done
