#!/bin/bash
# PMC counters of one graphed training step (timed region only), 3 passes (SQ, FETCH, WRITE).
# -> gpurun_out/pmc_<tag>_<pass>/ ; summarised by scripts/pmc_summary.py
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-step}; shift
mkdir -p gpurun_out
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
P2="FETCH_SIZE"
P3="WRITE_SIZE GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/pmc_${TAG}_$i -o run -- python bench.py --steps 2 --warmup 2 --trace_markers "$@" > gpurun_out/pmc_${TAG}_$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc_${TAG}_$i.log; exit 1; }
  echo "pass $i ok"
done
python scripts/pmc_summary.py /tmp/pmc_${TAG}_1 /tmp/pmc_${TAG}_2 /tmp/pmc_${TAG}_3 2 > gpurun_out/pmc_${TAG}_summary.txt 2>&1
head -60 gpurun_out/pmc_${TAG}_summary.txt
