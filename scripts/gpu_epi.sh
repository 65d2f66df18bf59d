#!/bin/bash
# conv / kernel / model GPU tests + bench + step profile
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
TAG=${1:-epi}
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_update_hip_gpu.py tests/test_encoder_gpu.py tests/test_model_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?; tail -n 2 gpurun_out/${TAG}_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/${TAG}_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1 || { tail -3 gpurun_out/${TAG}_bench.log; exit 1; }
grep metric gpurun_out/${TAG}_bench.log | cut -c1-330
bash scripts/gpu_profile.sh ${TAG} > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/${TAG}_summary.txt > gpurun_out/${TAG}_categories.txt
cat gpurun_out/${TAG}_categories.txt
