#!/bin/bash
cd "$(dirname "$0")/../.."
export TMPDIR=/tmp
mkdir -p gpurun_out
L=gpurun_out/pool.log
: > $L
RAFT_GRAPH_SHARED_POOL=0 timeout -k 10 200 python -u scripts/r2/diag_poison.py graph >> $L 2>&1; echo "sep-pool rc=$?" >> $L
RAFT_GRAPH_SHARED_POOL=0 timeout -k 10 200 python -u scripts/r2/diag_poison.py graph_which >> $L 2>&1; echo "sep-pool which rc=$?" >> $L
grep -v amdgpu $L | grep -v "finite \[" | cut -c1-300
