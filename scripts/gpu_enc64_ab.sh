#!/bin/bash
# conv_enc64 kernel A/B (RAFT_ENC64_KERNEL): encoder GPU tests, per-call times
# (scripts/bench_enc64.py), bench per kernel, step profile of the default -> gpurun_out/enc64t_*
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out/miopen_db
[ -d miopen_db ] && cp -r miopen_db/. gpurun_out/miopen_db/
export MIOPEN_USER_DB_PATH=$PWD/gpurun_out/miopen_db
timeout -k 10 400 python -u -m pytest tests/test_encoder_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/enc64t_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/enc64t_pytest.log; [ $rc -ne 0 ] && { grep -E "^E |FAILED" gpurun_out/enc64t_pytest.log | head; exit $rc; }
for v in wg1 half pipe; do
  RAFT_ENC64_KERNEL=$v PYTHONPATH=. timeout -k 10 120 python -u scripts/bench_enc64.py > gpurun_out/enc64t_${v}_micro.log 2>&1 || { tail -3 gpurun_out/enc64t_${v}_micro.log; exit 1; }
  cat gpurun_out/enc64t_${v}_micro.log | grep -v amdgpu.ids
done
for v in pipe half pipe; do
  RAFT_ENC64_KERNEL=$v timeout -k 10 300 python bench.py > gpurun_out/enc64t_${v}_bench.log 2>&1 || { tail -3 gpurun_out/enc64t_${v}_bench.log; exit 1; }
  echo "kernel=$v $(grep -o '"value": [0-9.]*' gpurun_out/enc64t_${v}_bench.log)"
done
bash scripts/gpu_profile.sh enc64t > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/enc64t_summary.txt > gpurun_out/enc64t_categories.txt
grep -E "enc64" gpurun_out/enc64t_summary.txt | cut -c1-120
head -8 gpurun_out/enc64t_categories.txt
