#!/bin/bash
# A/B of the encoder-norm launch sizing (RAFT_NORM_MIN_WG): encoder GPU tests, then the step
# profile and bench per setting -> gpurun_out/norm_<wg>_{summary,categories}.txt, norm_<wg>_bench.log
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/norm_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/norm_pytest.log; [ $rc -ne 0 ] && exit $rc
for wg in ${@:-0 1024 2048}; do
  RAFT_NORM_MIN_WG=$wg timeout -k 10 300 python bench.py > gpurun_out/norm_${wg}_bench.log 2>&1 || { tail -3 gpurun_out/norm_${wg}_bench.log; exit 1; }
  echo "wg=$wg $(grep -o '"value": [0-9.]*' gpurun_out/norm_${wg}_bench.log)"
  RAFT_NORM_MIN_WG=$wg bash scripts/gpu_profile.sh norm_${wg} > /dev/null 2>&1 || exit 1
  python scripts/categorize.py gpurun_out/norm_${wg}_summary.txt > gpurun_out/norm_${wg}_categories.txt
  grep -E "encoder norm|^total" gpurun_out/norm_${wg}_categories.txt
done
