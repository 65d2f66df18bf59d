#!/bin/bash
# on-the-fly correlation check: its kernel tests, an onthefly bench + profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${1:-otf}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "onthefly" --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py --corr_mode onthefly > gpurun_out/${TAG}_bench.log 2>&1 || exit 1
grep metric gpurun_out/${TAG}_bench.log | cut -c1-300
bash scripts/gpu_profile.sh ${TAG} --corr_mode onthefly > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt
grep "corr" gpurun_out/${TAG}_summary.txt | cut -c1-140
