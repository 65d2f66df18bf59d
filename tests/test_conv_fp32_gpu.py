"""fp32 update-block convs on the bf16 MFMA kernels (split-bf16, ops/conv_fp32.py) vs fp64 / fp32
references: forward, input gradient, weight and bias gradients; and a whole fp32 RAFT step with
the split path vs the plain fp32 (MIOpen) update block."""
import argparse

import pytest
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import conv_fp32

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('cin,cout,k', [
    (384, 256, (1, 5)), (384, 128, (5, 1)), (256, 192, (3, 3)), (128, 64, (3, 3)),
    (324, 256, (1, 1)), (256, 2, (3, 3)), (256, 576, (1, 1)), (146, 96, (3, 3)), (2, 128, (7, 7)),
])
def test_split_bf16_conv_matches_fp64(ext_ops, cin, cout, k):
    torch.manual_seed(0)
    B, H, W = 2, 13, 21
    pad = (k[0] // 2, k[1] // 2)
    x = torch.randn(B, cin, H, W, device=DEV, requires_grad=True)
    w = (torch.randn(cout, cin, *k, device=DEV) / (cin * k[0] * k[1]) ** 0.5).requires_grad_()
    b = torch.randn(cout, device=DEV, requires_grad=True)
    g = torch.randn(B, cout, H, W, device=DEV)
    y = conv_fp32.conv2d(x, w, b, pad)
    dx, dw, db = torch.autograd.grad(y, (x, w, b), g)
    xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, w, b))
    yr = F.conv2d(xd, wd, bd, padding=pad)
    dxr, dwr, dbr = torch.autograd.grad(yr, (xd, wd, bd), g.double())
    # split-bf16: ~2^-16 relative per product (fp32 MIOpen itself is ~1e-7)
    assert _rel(y.double(), yr) < 5e-5
    assert _rel(dx.double(), dxr) < 5e-5
    assert _rel(dw.double(), dwr) < 5e-5
    assert _rel(db.double(), dbr) < 1e-6


def test_fp32_model_update_block_split_vs_miopen(ext_ops):
    """fp32 RAFT (no mixed precision): the split-bf16 update-block convs give the plain fp32
    model's flow and parameter gradients."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    torch.manual_seed(0)
    outs = {}
    for impl in ('auto', 'torch'):
        args = argparse.Namespace(small=False, mixed_precision=False, update_impl=impl)
        torch.manual_seed(0)
        m = RAFT(args).to(DEV).train()
        i1, i2, flow, valid = (t.to(DEV) for t in make_pair_batch(2, 128, 160, seed=3))
        assert m._use_fp32_mfma(i1) == (impl == 'auto')
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        outs[impl] = (preds[-1].detach(), {n: p.grad.detach().clone() for n, p in m.named_parameters()
                                           if p.grad is not None})
    (fa, ga), (fb, gb) = outs['auto'], outs['torch']
    assert _rel(fa, fb) < 1e-3
    for n in gb:
        if n.startswith('update_block'):
            assert _rel(ga[n], gb[n]) < 2e-3, n
