set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
PYTHONPATH=. timeout -k 10 200 python -u scripts/norm_bench.py > gpurun_out/norm_bench.log 2>&1 || exit 1
cd /tmp && PYTHONPATH=$GRAFT_REPO_ROOT timeout -k 10 200 rocprofv3 --kernel-trace --stats -d /tmp/nb -o nb -- python $GRAFT_REPO_ROOT/scripts/norm_bench.py > $GRAFT_REPO_ROOT/gpurun_out/norm_bench_prof.log 2>&1 || exit 1
cp $(find /tmp/nb -name "*kernel_stats.csv") $GRAFT_REPO_ROOT/gpurun_out/norm_bench_stats.csv
