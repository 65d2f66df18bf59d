"""One fused update-block iteration (forward + backward) at the chairs training shape, for a
per-dispatch rocprofv3 kernel trace:  rocprofv3 --kernel-trace --output-format csv -d D -o run --
python scripts/trace_update.py ; then  python scripts/trace_update.py --parse D"""
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run():
    import torch
    from pytorch_raft_amd.models.update import BasicUpdateBlock
    from pytorch_raft_amd.ops.update_hip import HipUpdateBlock, CORR_BUF
    import argparse
    args = argparse.Namespace(corr_levels=4, corr_radius=4)
    dev = 'cuda'
    ub = BasicUpdateBlock(args, hidden_dim=128).to(dev)
    B, H, W = 12, 46, 62
    from pytorch_raft_amd.ops import _ext
    for it in range(3):
        torch.cuda.synchronize()
        if it == 2:
            _ext.ops().phase_mark()   # the parse starts after the last marker (tuning runs before)
        hub = HipUpdateBlock(ub)
        h = torch.randn(B, H, W, 128, device=dev).tanh().to(torch.bfloat16).requires_grad_(True)
        x = torch.randn(B, H, W, 128, device=dev).relu().to(torch.bfloat16)
        corr = torch.randn(B, H, W, CORR_BUF, device=dev).to(torch.bfloat16).requires_grad_(True)
        flow = torch.randn(B, 2, H, W, device=dev)
        h2, delta, mask = hub(h, x, corr, flow)
        (h2.float().sum() + delta.sum() + mask.float().sum()).backward()
        torch.cuda.synchronize()


def parse(d):
    import csv
    f = glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    marks = [k for k, r in enumerate(rows) if 'phase_marker' in r['Kernel_Name']]
    rows = rows[marks[-1] + 1:] if marks else rows
    tot = 0.0
    for r in rows:
        us = (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
        tot += us
        print('%8.1f  %s' % (us, r['Kernel_Name'][:150]))
    print('total %.1f us' % tot)


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--parse':
        parse(sys.argv[2])
    else:
        run()
