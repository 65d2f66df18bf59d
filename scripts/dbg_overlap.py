"""Which update-block gradients differ between the inline and the side-stream wgrad flush?"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_raft_amd import RAFT
from pytorch_raft_amd.data.synthetic import make_pair_batch
from pytorch_raft_amd.ops import update_hip
from pytorch_raft_amd.ops.loss import sequence_loss

i1, i2, flow, valid = make_pair_batch(2, 128, 160, device='cuda')
runs = []
for mode in ('inline', 'inline', 'overlap', 'overlap', 'overlap_sync'):
    update_hip.set_wgrad_overlap(mode != 'inline')
    os.environ['RAFT_DBG_SYNC'] = '1' if mode == 'overlap_sync' else '0'
    torch.manual_seed(0)
    m = RAFT(argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip')).cuda().train()
    preds = m(i1, i2, iters=3)
    loss, _ = sequence_loss(preds, flow, valid, 0.8, impl='hip')
    loss.backward()
    torch.cuda.synchronize()
    runs.append({n: p.grad.clone() for n, p in m.update_block.named_parameters()})
names = list(runs[0])
for n in names:
    d = ['%.2e' % (runs[k][n] - runs[0][n]).abs().max().item() for k in range(1, len(runs))]
    print('%-28s scale %.2e  diffs vs inline#1: %s' % (n, runs[0][n].abs().max().item(), d))
