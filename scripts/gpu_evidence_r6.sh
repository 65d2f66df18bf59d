#!/bin/bash
# Round-6 evidence runs: long-horizon training parity (HIP bf16 vs stock ops, 2,000 steps, same
# init and data order) and BASELINE config 5 (Sintel 436x1024 inference, iters 32) at saturating
# batch sizes.  Every GPU step has its own time limit; a failed step ends the call.
#   usage: PARITY=1 INFER=1 TESTS='...' gpu_evidence_r6.sh <tag>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-r6ev}
O=gpurun_out/$TAG
mkdir -p gpurun_out/miopen_db $O
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
step() { echo "== $1 $(date +%T)"; }
if [ -n "$TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest $TESTS --maxfail=4 -q --timeout 280 --timeout-method thread > $O/pytest.log 2>&1
  rc=$?; tail -n 2 $O/pytest.log; [ $rc -ne 0 ] && grep -E "^E |FAILED" $O/pytest.log | grep -v amdgpu.ids | head -20
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ -n "$PARITY" ]; then
  S=${PARITY_STEPS:-2000}
  step parity_hip
  timeout -k 10 600 python -u scripts/parity_train.py --impl hip --steps $S --out $O/parity_hip.jsonl 2> $O/parity_hip.log || { tail -3 $O/parity_hip.log; exit 1; }
  tail -1 $O/parity_hip.log
  step parity_torch
  timeout -k 10 900 python -u scripts/parity_train.py --impl torch --steps $S --out $O/parity_torch.jsonl 2> $O/parity_torch.log || { tail -3 $O/parity_torch.log; exit 1; }
  tail -1 $O/parity_torch.log
  python scripts/parity_train.py --compare $O/parity_hip.jsonl $O/parity_torch.jsonl > $O/parity_compare.txt 2>&1
  cat $O/parity_compare.txt
fi
if [ -n "$INFER" ]; then
  for cfg in "64 auto" "512 allpairs" "768 onthefly" "1024 auto"; do
    set -- $cfg
    step "infer b$1 $2"
    timeout -k 10 420 python -u bench_infer.py --graph --batch $1 --corr_mode $2 --steps 3 --warmup 1 > $O/infer_sat_b$1_$2.log 2>&1 || { tail -3 $O/infer_sat_b$1_$2.log; exit 1; }
    grep metric $O/infer_sat_b$1_$2.log | cut -c1-400
  done
fi
step done
