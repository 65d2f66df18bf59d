#!/bin/bash
# PMC counters of the zr conv at three tile configs (64x128, 128x128, 256x128)
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for cfg in 1 0 5 6; do
  RAFT_CONV_CFG=$cfg timeout -k 10 200 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d /tmp/pmc_$cfg -o run -- python scripts/conv_one.py zr 10 > gpurun_out/pmc/run_$cfg.log 2>&1 || exit $?
  f=$(find /tmp/pmc_$cfg -name '*counter_collection.csv' | head -1)
  python - "$f" $cfg <<'PY' >> gpurun_out/pmc/summary.txt
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if 'conv_fwd' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
print('cfg', sys.argv[2], {k: round(sum(v) / len(v)) for k, v in acc.items()})
PY
done
cat gpurun_out/pmc/summary.txt
