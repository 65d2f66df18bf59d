#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 python scripts/micro_tap.py > gpurun_out/micro_tap.log 2>&1 || exit $?
cat gpurun_out/micro_tap.log | grep corr_tap
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VMEM --output-format csv -d /tmp/pmc_tap -o run -- python scripts/micro_tap.py > gpurun_out/pmc_tap.log 2>&1 || exit $?
f=$(find /tmp/pmc_tap -name "*counter_collection*.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if 'tap_reduce' in r.get('Kernel_Name', ''):
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in acc.items():
    print('%-20s %.4g (mean over %d dispatches)' % (k, sum(v) / len(v), len(v)))
PY
