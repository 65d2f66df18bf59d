#!/bin/bash
set -o pipefail
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u scripts/r2/diag_graph.py ${1:-all} > gpurun_out/diag_graph.log 2>&1
rc=$?; tail -20 gpurun_out/diag_graph.log; exit $rc
