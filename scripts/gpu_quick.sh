#!/bin/bash
# quick check after a kernel change: the kernel GPU tests + one bench run + a profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
# liveness for long steps (MIOpen searches, multi-process tests): the per-step timeouts below
# bound real hangs
(while sleep 50; do date +%T >> gpurun_out/heartbeat.txt; done) &
HB=$!
trap 'kill $HB 2>/dev/null' EXIT
TAG=${1:-quick}
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
grep metric gpurun_out/${TAG}_bench.log | cut -c150-260
bash scripts/gpu_profile.sh ${TAG} > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt
grep "corr" gpurun_out/${TAG}_summary.txt | cut -c1-120
timeout -k 10 300 python bench.py --steps 4 --warmup 3 --profile gpurun_out/${TAG}_torchprof > gpurun_out/${TAG}_tprof_bench.log 2>&1 || exit 1
head -45 gpurun_out/${TAG}_torchprof/ops.txt | cut -c1-200
