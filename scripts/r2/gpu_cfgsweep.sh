#!/bin/bash
# time every conv tile config (RAFT_CONV_CFG) on the update-block geometries
set -o pipefail
cd "$(dirname "$0")/../.."
mkdir -p gpurun_out
G=${1:-zr1,c2,head,c1}
for i in $(seq 0 29); do
  echo "cfg $i"
  RAFT_CONV_CFG=$i timeout -k 10 60 python scripts/r2/conv_bench.py $G 20 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/cfgsweep.log
echo done
