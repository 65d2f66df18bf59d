#!/bin/bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 250 python -u scripts/r2/diag_poison.py graph_cmp > gpurun_out/cmp3.log 2>&1; grep replay gpurun_out/cmp3.log | cut -c1-500
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 250 python -u scripts/r2/diag_poison.py graph > gpurun_out/g3.log 2>&1; grep "graph" gpurun_out/g3.log | cut -c1-400
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 250 python bench.py --steps 20 --warmup 5 > gpurun_out/bwd0_bench.log 2>&1; grep -o '"value[^,]*,\|"ms_per_step[^,]*\|"loss_finite[^,]*\|"nonfinite[^,]*' gpurun_out/bwd0_bench.log | tr '\n' ' '
