#!/bin/bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/miopen_graph.log
: > $L
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 200 python -u scripts/r2/diag_poison.py graph > /tmp/mg.log 2>&1
  echo "$n rc=$? $(grep -v amdgpu /tmp/mg.log | grep 'graph \[' | cut -c1-200)" >> $L
}
run wrw0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
run bwd0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
run fwd0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
run all0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_FWD_GTC_XDLOPS_NHWC=0
run igemm0 MIOPEN_DEBUG_CONV_IMPLICIT_GEMM=0
cat $L
