#!/bin/bash
# A/B: MIOpen asm implicit-GEMM NHWC weight-gradient solvers (split-K with zero-fill) on / off
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_mi_a.log 2>&1 || exit $?
echo "default: $(tail -1 gpurun_out/bench_mi_a.log | cut -c90-140)"
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_mi_b.log 2>&1 || exit $?
echo "no asm wrw nhwc: $(tail -1 gpurun_out/bench_mi_b.log | cut -c90-140)"
MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_mi_c.log 2>&1 || exit $?
echo "no asm bwd nhwc: $(tail -1 gpurun_out/bench_mi_c.log | cut -c90-140)"
