"""Diagnose hipGraph inference replay vs eager (per-item differences, repeatability)."""
import argparse, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_raft_amd import RAFT
from pytorch_raft_amd.data.synthetic import make_pair_batch
from pytorch_raft_amd.engine.inference import FlowInference
args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip')
torch.manual_seed(0)
m = RAFT(args).cuda().eval()
i1, i2, _, _ = make_pair_batch(2, 124, 156, device='cuda')
def d(a, b):
    return [float((a[k] - b[k]).abs().max()) for k in range(a.shape[0])]
e = FlowInference(m, iters=5)
a1 = e(i1, i2)[1]; a2 = e(i1, i2)[1]; b1 = e(i2, i1)[1]; b2 = e(i2, i1)[1]
print('eager repeat', d(a1, a2), d(b1, b2), 'magnitude', float(a1.abs().max()), 'swap diff', d(a1, b1))
g = FlowInference(m, iters=5, graph=True)
ga = g(i1, i2)[1]; gb = g(i2, i1)[1]; ga2 = g(i1, i2)[1]
print('graph vs eager', d(ga, a1), d(gb, b1), d(ga2, a1))
# capture with swapped inputs first
g2 = FlowInference(m, iters=5, graph=True)
hb = g2(i2, i1)[1]; ha = g2(i1, i2)[1]
print('graph2 vs eager', d(hb, b1), d(ha, a1))
# low-res flow and per-iteration check with iters=1
for it in (1, 2):
    e1 = FlowInference(m, iters=it); g1 = FlowInference(m, iters=it, graph=True)
    x = g1(i1, i2); y = g1(i2, i1); ye = e1(i2, i1)
    print('iters', it, 'low', d(y[0], ye[0]), 'up', d(y[1], ye[1]))
