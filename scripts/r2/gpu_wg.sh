#!/bin/bash
# tap-fused wgrad: numerics tests, per-geometry micro-bench, kernel trace + PMC of the 3x3 launch
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-wg}
timeout -k 10 300 python -m pytest tests/test_conv_gpu.py -q -x -k taps > gpurun_out/${T}_test.log 2>&1
rc=$?; tail -1 gpurun_out/${T}_test.log; [ $rc -eq 0 ] || exit $rc
[ -n "$SKIPB" ] || timeout -k 10 300 python scripts/r2/wgrad_bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
cat gpurun_out/${T}_bench.log | grep -v amdgpu.ids
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/${T}_kt -o kt -- python3 scripts/r2/wgrad_bench.py c2,head taps > gpurun_out/${T}_rp.log 2>&1 || exit 1
f=$(find /tmp/${T}_kt -name '*kernel_stats.csv' | head -1); cp "$f" gpurun_out/${T}_kstats.csv
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d /tmp/${T}_p1 -o p1 -- python3 scripts/r2/wgrad_bench.py c2 taps > gpurun_out/${T}_rp.log 2>&1 || exit 1
f=$(find /tmp/${T}_p1 -name '*counter_collection.csv' | head -1); cp "$f" gpurun_out/${T}_pmc1.csv
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d /tmp/${T}_p2 -o p2 -- python3 scripts/r2/wgrad_bench.py c2 taps > gpurun_out/${T}_rp.log 2>&1 || exit 1
f=$(find /tmp/${T}_p2 -name '*counter_collection.csv' | head -1); cp "$f" gpurun_out/${T}_pmc2.csv
echo done
