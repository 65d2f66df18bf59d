#!/bin/bash
# PMC counters + durations of one conv shape over tile configs.  usage: gpu_pmc_conv2.sh <layer> <cfg...>
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
LAYER=$1; shift
CTR="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
for cfg in "$@"; do
  RAFT_CONV_CFG=$cfg timeout -k 10 120 rocprofv3 --pmc $CTR --kernel-trace --output-format csv -d /tmp/pmc2_$cfg -o run -- python scripts/conv_one.py $LAYER 10 > gpurun_out/pmc/run2_$cfg.log 2>&1 || exit $?
  f=$(find /tmp/pmc2_$cfg -name '*counter_collection.csv' | head -1)
  k=$(find /tmp/pmc2_$cfg -name '*kernel_trace.csv' | head -1)
  python - "$f" "$k" "$LAYER cfg=$cfg" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
acc = collections.defaultdict(list)
for r in rows:
    if 'conv_fwd' in r['Kernel_Name']:
        acc[r['Counter_Name']].append(float(r['Counter_Value']))
d = {k: sum(v[2:]) / max(1, len(v[2:])) for k, v in acc.items()}
durs = [int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in csv.DictReader(open(sys.argv[2])) if 'conv_fwd' in r['Kernel_Name']]
durs = sorted(durs[2:])
busy = d['SQ_BUSY_CYCLES']
print(sys.argv[3], 'dur_us(med)=%.1f' % (durs[len(durs)//2] / 1e3), 'mfma_busy/busy=%.2f' % (d['SQ_VALU_MFMA_BUSY_CYCLES'] / max(1, busy)),
      {k[3:]: round(v / 1e6, 3) for k, v in d.items()})
PY
done
