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


@pytest.mark.parametrize('layout', ['nchw', 'channels_last', 'strided'])
@pytest.mark.parametrize('c,cpad', [(70, 128), (2, 64), (256, 256), (126, 128)])
def test_split_hilo_kernel_matches_torch(ext_ops, c, cpad, layout):
    """split_hilo kernel == the reference torch formulation, bit for bit, for NCHW, channels_last
    and non-contiguous (sliced) inputs, with the zero padding of both halves."""
    torch.manual_seed(12)
    x = torch.randn(3, c + (5 if layout == 'strided' else 0), 17, 70, device=DEV) * 7
    if layout == 'channels_last':
        x = x.contiguous(memory_format=torch.channels_last)
    if layout == 'strided':
        x = x[:, 3:3 + c]
    got = conv_fp32._split_nhwc(x, cpad)
    want = conv_fp32._split_nhwc_torch(x, cpad)
    assert torch.equal(got, want)


@pytest.mark.parametrize('k', [(3, 3), (1, 5), (7, 7)])
def test_module_token_batched_wgrad_vs_fp64(ext_ops, k):
    """MfmaConv2d called 3 times in one decode scope: the calls share one weight token and their
    weight / bias gradients come from ONE deferred batched launch pair -- vs fp64 autograd."""
    from pytorch_raft_amd.models.update import MfmaConv2d
    torch.manual_seed(11)
    cin = 2 if k == (7, 7) else 96
    m = MfmaConv2d(cin, 64, k, padding=(k[0] // 2, k[1] // 2)).to(DEV)
    xs = [torch.randn(2, cin, 13, 21, device=DEV, requires_grad=True) for _ in range(3)]
    gs = [torch.randn(2, 64, 13, 21, device=DEV) for _ in range(3)]
    with conv_fp32.enabled():
        outs = [m(x) for x in xs]
    sum((o * g).sum() for o, g in zip(outs, gs)).backward()
    w64 = m.weight.detach().double().requires_grad_(True)
    b64 = m.bias.detach().double().requires_grad_(True)
    x64 = [x.detach().double().requires_grad_(True) for x in xs]
    refs = [F.conv2d(x, w64, b64, padding=m.padding) for x in x64]
    sum((r * g.double()).sum() for r, g in zip(refs, gs)).backward()
    for o, r in zip(outs, refs):
        assert _rel(o.double(), r) < 5e-5
    assert _rel(m.weight.grad.double(), w64.grad) < 5e-5
    assert _rel(m.bias.grad.double(), b64.grad) < 1e-5
    for x, x6 in zip(xs, x64):
        assert _rel(x.grad.double(), x6.grad) < 5e-5


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
    # one ReLU pre-activation within the split scheme's ~2^-16 of zero flips its mask and moves a
    # 16 x 20-cell decode's upstream gradients by ~1e-2; the kernels' precision itself is pinned
    # with shared masks by test_fp32_fused_gpu.py::test_fp32_fused_update_iteration_vs_fp64 (1e-4)
    for n in gb:
        if n.startswith('update_block'):
            assert _rel(ga[n], gb[n]) < 2e-2, n


def test_fp32_training_trajectory_split_vs_miopen(ext_ops):
    """End-to-end pin of the split-bf16 fp32 update block (fp32 semantics): 6 AdamW
    steps of an fp32 model (reference paper schedule: no mixed precision) with the update-block
    convs on the split-bf16 MFMA kernels vs the same steps on MIOpen fp32 convs; the loss
    trajectories agree to 1e-3 relative and the final update-block weights to 2e-3 (biases 1e-2:
    AdamW turns a ~2^-16 gradient difference into a full +-lr step wherever a gradient component
    is near zero)."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    batches = [tuple(t.to(DEV) for t in make_pair_batch(2, 128, 160, seed=10 + s)) for s in range(6)]
    runs = {}
    for impl in ('auto', 'torch'):
        args = argparse.Namespace(small=False, mixed_precision=False, update_impl=impl)
        torch.manual_seed(0)
        m = RAFT(args).to(DEV).train()
        opt = torch.optim.AdamW(m.parameters(), lr=2e-4, weight_decay=1e-4, eps=1e-8)
        losses = []
        for i1, i2, flow, valid in batches:
            opt.zero_grad(set_to_none=True)
            loss, _ = sequence_loss(m(i1, i2, iters=3), flow, valid, 0.8)
            loss.backward()
            torch.nn.utils.clip_grad_norm_(m.parameters(), 1.0)
            opt.step()
            losses.append(loss.item())
        runs[impl] = (losses, {n: p.detach().clone() for n, p in m.named_parameters()})
    (la, wa), (lb, wb) = runs['auto'], runs['torch']
    for a, b in zip(la, lb):
        assert abs(a - b) <= 1e-3 * abs(b) + 1e-5, (la, lb)
    for n in wb:
        if n.startswith('update_block'):
            # biases: few entries of small norm, where one sign-flipped AdamW step shows most
            assert _rel(wa[n], wb[n]) < (2e-3 if wb[n].dim() > 1 else 1e-2), n


def _emulated_split_conv(x, w, b, pad):
    """fp64 emulation of the split-bf16 forward (3 products of bf16-rounded hi / lo parts)."""
    def bf(t):
        return t.float().to(torch.bfloat16).double()
    xh, wh = bf(x), bf(w)
    xl, wl = bf(x - xh), bf(w - wh)
    y = (F.conv2d(xh, wh, None, padding=pad) + F.conv2d(xl, wh, None, padding=pad) +
         F.conv2d(xh, wl, None, padding=pad))
    return y + b.view(1, -1, 1, 1)


class _EmuSplit(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad):
        ctx.save_for_backward(x, w)
        ctx.pad = pad
        return _emulated_split_conv(x, w, b, pad)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        return (torch.nn.grad.conv2d_input(x.shape, w, g, padding=ctx.pad),
                torch.nn.grad.conv2d_weight(x, w.shape, g, padding=ctx.pad), g.sum((0, 2, 3)), None)


@pytest.mark.parametrize('norm', ['instance', 'batch'])
def test_fp32_encoder_split_vs_fp64(ext_ops, norm):
    """fp32 BasicEncoder (fnet: instance norm, cnet: batch norm): with ``conv_fp32.enabled()`` its
    stride-1 convs (12 of 15) run as split-bf16 MFMA products.  Output, input gradient and every
    parameter gradient are compared with an fp64 CPU run of the same module.

    The encoder's gradients at init are very sensitive to the forward's rounding: the split-bf16
    forward ALONE, emulated in fp64 with exact backward convs, moves the input gradient by ~7e-3
    (an fp32 forward by ~2e-7; profiles/r4/fp32_encoder_conditioning.txt), while every split conv
    is at ~4e-6 given the gradient it receives.  So the GPU run is bounded per tensor by 3x the
    larger of MIOpen fp32's error and that emulation's (computed here for the same module and
    inputs), with a 1e-2 floor for the backward's own split-bf16 rounding: the kernels implement
    the scheme (a kernel bug gives O(1) errors), the scheme's sensitivity is documented.  The
    output itself must stay within 1e-4."""
    import copy
    from pytorch_raft_amd.models import update as U
    from pytorch_raft_amd.models.extractor import BasicEncoder
    torch.manual_seed(0)
    enc = BasicEncoder(output_dim=256, norm_fn=norm).to(DEV).train()
    x0 = torch.randn(3, 3, 96, 128, device=DEV)
    gout = torch.randn(3, 256, 12, 16, device=DEV)

    def run(m, x, g, on=False, emulate=False):
        m.zero_grad(set_to_none=True)
        x = x.clone().requires_grad_(True)
        orig = U.MfmaConv2d.forward
        if emulate:
            def fwd(self, xx):
                if self.stride == (1, 1):
                    return _EmuSplit.apply(xx, self.weight, self.bias, self.padding)
                return torch.nn.Conv2d.forward(self, xx)
            U.MfmaConv2d.forward = fwd
        try:
            with conv_fp32.enabled(on):
                y = m(x)
        finally:
            U.MfmaConv2d.forward = orig
        (y * g).sum().backward()
        return {'out': y.detach().double().cpu(), 'dx': x.grad.detach().double().cpu(),
                **{n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}}

    m64 = copy.deepcopy(enc).double().cpu()
    ref = run(m64, x0.double().cpu(), gout.double().cpu())
    emu = run(m64, x0.double().cpu(), gout.double().cpu(), emulate=True)
    split = run(enc, x0, gout, True)
    miop = run(enc, x0, gout, False)
    assert _rel(split['out'], ref['out']) < 1e-4
    for n in ref:
        if n.endswith('.bias') and n != 'conv2.bias' and ('conv' in n or 'downsample.0' in n):
            continue   # a conv bias feeding a norm has an exactly-zero gradient (rounding noise)
        es, em, ee = _rel(split[n], ref[n]), _rel(miop[n], ref[n]), _rel(emu[n], ref[n])
        # the emulation covers the forward's rounding; the backward's split-bf16 products add
        # their own (the strided layer-3 conv's weight gradient: 9e-4 vs 2e-5 emulated), so the
        # floor is the 1e-2 scale the emulation shows for the input gradient -- a kernel bug
        # gives O(1) errors
        assert es <= max(3 * max(em, ee), 1e-2), (n, es, em, ee)
