"""Update-block gradients: unfused x2 vs fused gate epilogues (relative norm differences)."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd import RAFT  # noqa: E402
from pytorch_raft_amd.data.synthetic import make_pair_batch  # noqa: E402
from pytorch_raft_amd.ops import update_hip  # noqa: E402
from pytorch_raft_amd.ops.loss import sequence_loss  # noqa: E402

dev = 'cuda'
i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=dev)
grads = []
for fused in (False, False, True, True):
    update_hip._GATES_FUSED = fused
    args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip')
    torch.manual_seed(0)
    m = RAFT(args).to(dev).train()
    preds = m(i1, i2, iters=int(sys.argv[1]) if len(sys.argv) > 1 else 3)
    loss, _ = sequence_loss(preds, flow, valid, 0.8)
    loss.backward()
    grads.append({n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None})


def rel(x, y):
    return ((x - y).norm() / y.norm().clamp_min(1e-12)).item()


for n in grads[0]:
    if n.startswith('update_block') or n in ('fnet.conv1.weight', 'cnet.conv1.weight', 'fnet.conv2.weight'):
        print('%-50s unf-unf %.2e  fus-fus %.2e  fus-unf %.2e' % (
            n, rel(grads[1][n], grads[0][n]), rel(grads[3][n], grads[2][n]), rel(grads[2][n], grads[0][n])))
