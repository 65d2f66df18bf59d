#!/bin/bash
# PMC passes over scripts/bench_enc64.py (conv_enc64 kernels only) + the device's counter list
# -> gpurun_out/enc64pmc_*.csv, gpurun_out/counters.txt
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
R=$PWD
mkdir -p gpurun_out
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/counters.txt 2>&1 || { echo "list-avail failed"; tail -3 gpurun_out/counters.txt; }
pick() { for c in "$@"; do grep -qw "$c" gpurun_out/counters.txt && printf '%s ' "$c"; done; }
P1="SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT"
P2=$(pick SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM)
P3=$(pick SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INSTS_MFMA SQ_LDS_IDX_ACTIVE SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL SQ_ACTIVE_INST_MISC)
echo "P2: $P2"; echo "P3: $P3"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  [ -z "$P" ] && continue
  cd /tmp && RAFT_ENC64_HALF=${HALF:-1} PYTHONPATH=$R timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/ep$i -o run -- python $R/scripts/bench_enc64.py > $R/gpurun_out/enc64pmc_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $R/gpurun_out/enc64pmc_$i.log; exit 1; }
  cd $R
  f=$(find /tmp/ep$i -name "*counter_collection.csv" | head -1)
  [ -n "$f" ] && python - "$f" <<'PY' > gpurun_out/enc64pmc_$i.txt
import csv, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(float))
n = collections.Counter()
for r in csv.DictReader(open(sys.argv[1])):
    k = r['Kernel_Name']
    if 'enc64' not in k:
        continue
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, d in acc.items():
    print(k[:80])
    for c, v in sorted(d.items()):
        print('   %-28s %.4g' % (c, v))
PY
  cat gpurun_out/enc64pmc_$i.txt
done
