#!/bin/bash
# PMC counters of one conv shape: normal vs loads-return-zero (RAFT_CONV_NULLMEM) per tile config
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
rm -f gpurun_out/pmc/summary.txt
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
LAYER=${1:-zr}
for nm in 0 1; do
for cfg in 1 0; do
  RAFT_CONV_NULLMEM=$nm RAFT_CONV_CFG=$cfg timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d /tmp/pmc_${nm}_$cfg -o run -- python scripts/conv_one.py $LAYER 10 > gpurun_out/pmc/run_${nm}_$cfg.log 2>&1 || exit $?
  f=$(find /tmp/pmc_${nm}_$cfg -name '*counter_collection.csv' | head -1)
  python - "$f" "nullmem=$nm cfg=$cfg" <<'PY' >> gpurun_out/pmc/summary.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if 'conv_fwd' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
d = {k: sum(v) / len(v) for k, v in acc.items()}
us = d['SQ_BUSY_CYCLES'] / 32 / 2400.0
print(sys.argv[2], 'est_us=%.1f' % us, 'mfma_util=%.2f' % (d['SQ_VALU_MFMA_BUSY_CYCLES'] / (d['SQ_BUSY_CYCLES'] / 32 * 1024)),
      {k[3:]: round(v / 1e6, 2) for k, v in d.items()})
PY
done
done
cat gpurun_out/pmc/summary.txt
