#!/bin/bash
# Stock reference-semantics baseline (no HIP kernels of ours) + the 2-rank DP / graph rehearsals.
set -o pipefail
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_dp_gpu.py tests/test_graph_gpu.py -v --timeout 170 --timeout-method thread -s > gpurun_out/dp_graph.log 2>&1
rc=$?; grep -E "passed|failed|dp rehearsal" gpurun_out/dp_graph.log | tail -6; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --impl torch --warmup 10 --steps 50 > gpurun_out/stock_bf16_10w50.log 2>&1 || exit 1
grep metric gpurun_out/stock_bf16_10w50.log | cut -c1-400
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/stockprof -o run -- python bench.py --impl torch --warmup 2 --steps 2 > gpurun_out/stock_prof.log 2>&1 || exit 1
python - <<'PY' > gpurun_out/stock_kernel_names.txt
import csv, glob, collections
f = glob.glob('/tmp/stockprof/**/*kernel_trace.csv', recursive=True)[0]
c = collections.Counter(r['Kernel_Name'] for r in csv.DictReader(open(f)))
ours = ('corr_', 'conv_fwd', 'conv_wgrad', 'norm_', 'convex_up', 'seq_loss', 'fh2_', 'gru_', 'relu_mask',
        'relu_bwd', 'f1_patch', 'sum_bf16', 'partial_reduce', 'warp_', 'add_relu')
hits = {k: v for k, v in c.items() if any(o in k for o in ours)}
print('kernels:', len(c), 'launches:', sum(c.values()))
print('raft_amd kernels in the stock run:', len(hits))
for k, v in sorted(hits.items(), key=lambda x: -x[1]):
    print(v, k[:200])
for k, v in c.most_common(40):
    print('%6d  %s' % (v, k[:160]))
PY
head -5 gpurun_out/stock_kernel_names.txt
# where the fp32 (paper schedule) and the on-the-fly correlation steps spend their time
bash scripts/gpu_profile.sh otf --corr_mode onthefly > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/otf_summary.txt > gpurun_out/otf_categories.txt
grep metric gpurun_out/otf_prof_bench.log | cut -c1-200
bash scripts/gpu_profile.sh fp32 --precision fp32 > /dev/null 2>&1 || exit 1
python scripts/categorize.py gpurun_out/fp32_summary.txt > gpurun_out/fp32_categories.txt
grep metric gpurun_out/fp32_prof_bench.log | cut -c1-200
