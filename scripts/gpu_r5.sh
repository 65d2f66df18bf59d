#!/bin/bash
# Round-5 iteration recipe: selected GPU tests, bench, phase-split kernel profile, per-dispatch
# trace of one update-block iteration, optional stack-attributed op profile and PMC passes.
# Steps are chained: a failed / timed-out / crashed step ends the call (failed test assertions
# excepted: the rest of the call still runs).
#   usage: TESTS='tests/a.py tests/b.py' STACK=1 PMC=1 gpu_r5.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r5}
O=gpurun_out/$TAG
mkdir -p gpurun_out/miopen_db $O
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest $TESTS --maxfail=4 -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -n 2 $O/pytest.log; [ $rc -ne 0 ] && grep -E "^E |FAILED" $O/pytest.log | grep -v amdgpu.ids | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$TUNE" ]; then
  # fresh conv tile table: every key autotuned with $TUNE timing trials (no persisted picks),
  # written to $O/conv_gfx950.txt (copy it to pytorch_raft_amd/tune_db/ to persist it)
  step tune
  RAFT_CONV_TUNE_DB=0 RAFT_CONV_TUNE_TRIALS=$TUNE timeout -k 10 300 python bench.py $BENCH_ARGS --dump_tune $O/conv_gfx950.txt > $O/tune_bench.log 2>&1 || { tail -3 $O/tune_bench.log; exit 1; }
  grep metric $O/tune_bench.log | cut -c1-200
fi
step bench
timeout -k 10 300 python bench.py $BENCH_ARGS > $O/bench.log 2>&1 || { tail -3 $O/bench.log; exit 1; }
grep metric $O/bench.log | cut -c1-330
step profile
RAFT_PHASE_MARKS=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/prof_$TAG -o run -- python bench.py --steps 4 --warmup 3 --trace_markers $BENCH_ARGS > $O/prof_bench.log 2>&1 || { tail -3 $O/prof_bench.log; exit 1; }
python scripts/prof_diff.py --phases /tmp/prof_$TAG 4 > $O/summary.txt 2>&1 && python scripts/prof_diff.py --sequence /tmp/prof_$TAG > $O/sequence.txt 2>&1
python scripts/categorize.py $O/summary.txt > $O/categories.txt
cat $O/categories.txt
step trace_update
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tu_$TAG -o run -- python scripts/trace_update.py > $O/trace_update_run.log 2>&1 || { tail -3 $O/trace_update_run.log; exit 1; }
python scripts/trace_update.py --parse /tmp/tu_$TAG > $O/trace_update.txt 2>&1
tail -n 1 $O/trace_update.txt
if [ -n "$STACK" ]; then
  step stack
  timeout -k 10 300 python bench.py --eager --steps 2 --warmup 3 --profile $O/torchprof --profile_stack > $O/stack_bench.log 2>&1 || { tail -3 $O/stack_bench.log; exit 1; }
fi
if [ -n "$PMC" ]; then
  step pmc
  # one pass per counter group (rocprofv3 does not split counters over passes)
  P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
  P2="FETCH_SIZE"
  P3="WRITE_SIZE GRBM_GUI_ACTIVE"
  i=0
  for P in "$P1" "$P2" "$P3"; do
    i=$((i+1))
    timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/pmc_${TAG}_$i -o run -- python bench.py --steps 2 --warmup 2 --trace_markers $BENCH_ARGS > $O/pmc$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $O/pmc$i.log; exit 1; }
  done
  python scripts/pmc_summary.py /tmp/pmc_${TAG}_1 /tmp/pmc_${TAG}_2 /tmp/pmc_${TAG}_3 2 > $O/pmc.txt 2>&1 || true
  head -3 $O/pmc.txt
fi
if [ -n "$AB" ]; then
  # A/B on one box: alternating runs of the default build and the build under $AB (VAR=value)
  step ab
  for i in 1 2; do
    timeout -k 10 300 env $AB python bench.py $BENCH_ARGS > $O/ab_alt_$i.log 2>&1 || { tail -3 $O/ab_alt_$i.log; exit 1; }
    timeout -k 10 300 python bench.py $BENCH_ARGS > $O/ab_def_$i.log 2>&1 || { tail -3 $O/ab_def_$i.log; exit 1; }
    echo "$AB: $(grep -o '"value": [0-9.]*' $O/ab_alt_$i.log)   default: $(grep -o '"value": [0-9.]*' $O/ab_def_$i.log)"
  done
fi
step done
