set -o pipefail
cd /root/repo
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py tests/test_update_hip_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/v3_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/v3_pytest.log; if [ $rc -ne 0 ]; then grep -E "^E |FAILED" gpurun_out/v3_pytest.log | head -20; exit $rc; fi
timeout -k 10 300 python bench.py > gpurun_out/v3_bench.log 2>&1 || exit 1
grep metric gpurun_out/v3_bench.log | cut -c1-300
RAFT_CONV_V3=0 timeout -k 10 300 python bench.py > gpurun_out/v3off_bench.log 2>&1 || exit 1
grep metric gpurun_out/v3off_bench.log | cut -c1-300
