#!/bin/bash
# implicit-GEMM conv: per-geometry micro-bench + PMC of one geometry
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-cv}
G=${2:-zr1}
timeout -k 10 300 python scripts/r2/conv_bench.py > gpurun_out/${T}_bench.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/${T}_bench.log
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d /tmp/${T}_p1 -o p1 -- python3 scripts/r2/conv_bench.py $G 5 > gpurun_out/${T}_rp.log 2>&1 || exit 1
f=$(find /tmp/${T}_p1 -name '*counter_collection.csv' | head -1); cp "$f" gpurun_out/${T}_pmc1.csv
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE TCP_TOTAL_CACHE_ACCESSES_sum --output-format csv -d /tmp/${T}_p2 -o p2 -- python3 scripts/r2/conv_bench.py $G 5 > gpurun_out/${T}_rp.log 2>&1 || exit 1
f=$(find /tmp/${T}_p2 -name '*counter_collection.csv' | head -1); cp "$f" gpurun_out/${T}_pmc2.csv
echo done
