#!/bin/bash
# PMC counters of one conv layer under forced configs (LDS-DMA 5x1 vs halo 5x1 / 5x2)
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmch
rm -f gpurun_out/pmch/summary.txt
LAYER=${1:-zr2}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VMEM SQ_BUSY_CYCLES"
for cfg in 16 30 31; do
for pi in 1 2; do
  if [ $pi = 1 ]; then P="$P1"; else P="$P2"; fi
  RAFT_CONV_CFG=$cfg timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/pmch_${cfg}_$pi -o run -- python scripts/conv_one.py $LAYER 10 > gpurun_out/pmch/run_${cfg}_$pi.log 2>&1 || { echo "cfg $cfg pass $pi failed"; tail -5 gpurun_out/pmch/run_${cfg}_$pi.log; exit 1; }
  f=$(find /tmp/pmch_${cfg}_$pi -name '*counter_collection.csv' | head -1)
  python - "$f" "cfg=$cfg pass=$pi" <<'PY' >> gpurun_out/pmch/summary.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if 'conv_fwd' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
d = {k: sum(v[2:]) / max(1, len(v[2:])) for k, v in acc.items()}
print(sys.argv[2], {k[3:]: round(v / 1e6, 3) for k, v in sorted(d.items())})
PY
done
done
cat gpurun_out/pmch/summary.txt
