"""Channels-last fused encoder path (ops/encoder.py + encoder_norm.hip) vs the eager encoder."""
import pytest
import torch

from pytorch_raft_amd.models.extractor import BasicEncoder, SmallEncoder
from pytorch_raft_amd.ops import encoder as fast

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _cos(a, b):
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


H16 = torch.float16


@pytest.mark.parametrize('cls,norm,train,dt', [
    (BasicEncoder, 'instance', True, torch.bfloat16), (BasicEncoder, 'batch', True, torch.bfloat16),
    (BasicEncoder, 'batch', False, torch.bfloat16), (SmallEncoder, 'instance', True, torch.bfloat16),
    (SmallEncoder, 'none', True, torch.bfloat16),
    # fp16 autocast (the reference's --mixed_precision): fp16 MFMA convs and fp16 norm kernels
    (BasicEncoder, 'instance', True, H16), (BasicEncoder, 'batch', True, H16),
    (SmallEncoder, 'instance', True, H16)])
def test_fast_encoder_matches_eager(ext_ops, cls, norm, train, dt):
    torch.manual_seed(0)
    enc = cls(output_dim=256 if cls is BasicEncoder else 128, norm_fn=norm).to(DEV)
    for m in enc.modules():  # non-trivial affine / conv biases / running stats
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.8, 1.2)
        if isinstance(m, torch.nn.Conv2d):
            m.bias.data.uniform_(-0.1, 0.1)
    enc.train(train)
    x = torch.randn(4, 3, 96, 128, device=DEV)
    state = {k: v.clone() for k, v in enc.state_dict().items()}
    outs, grads, bufs = {}, {}, {}
    for path in ('fp32', 'eager', 'fast'):
        enc.load_state_dict(state)
        enc.zero_grad(set_to_none=True)
        orig = fast.fast_path_ok
        if path != 'fast':
            fast.fast_path_ok = lambda *a: False
        try:
            with torch.autocast('cuda', dtype=dt, enabled=path != 'fp32'):
                if path == 'fast':
                    assert fast.fast_path_ok(enc, x)
                y = enc(x)
                if path != 'fp32':
                    assert y.dtype == dt
        finally:
            fast.fast_path_ok = orig
        (y.float() * torch.linspace(-1, 1, y.numel(), device=DEV).view(y.shape)).sum().backward()
        outs[path] = y.float()
        grads[path] = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
        bufs[path] = {k: v.clone() for k, v in enc.state_dict().items() if 'running' in k}
    ref = outs['fp32']
    rel = {p: ((outs[p] - ref).norm() / ref.norm()).item() for p in ('eager', 'fast')}
    # bf16 activations: the fused path must be about as close to fp32 as eager bf16 autocast
    assert rel['fast'] < max(5e-2, 1.5 * rel['eager']), rel
    report = []
    for n, g in grads['fp32'].items():
        normed_bias = n != 'conv2.bias' and n.endswith(('conv1.bias', 'conv2.bias', 'conv3.bias',
                                                         'downsample.0.bias'))
        if normed_bias and norm != 'none' and not (norm == 'batch' and not train):
            # exactly zero in exact arithmetic (the bias cancels in a batch-statistics norm)
            assert grads['fast'][n].abs().max() < 1e-2, n
            continue
        ce, cf = _cos(grads['eager'][n], g), _cos(grads['fast'][n], g)
        report.append((n, round(ce, 4), round(cf, 4)))
    print(report)
    for n, ce, cf in report:
        # the fused path must be as close to the fp32 gradients as eager bf16 autocast is
        assert cf > min(0.99, ce - 0.05), (n, ce, cf)
    for k, v in bufs['eager'].items():
        torch.testing.assert_close(bufs['fast'][k], v, atol=2e-3, rtol=2e-2)


@pytest.mark.parametrize('dt', [torch.bfloat16, H16])
def test_native_head_1x1_matches_conv2d(ext_ops, dt):
    """Encoder head 1x1 conv on the MFMA kernels (ops/encoder.py _Head1x1) vs F.conv2d in fp32 on
    the same 16-bit operands: output and all three gradients."""
    from pytorch_raft_amd.ops.encoder import _Head1x1
    g = torch.Generator(device='cpu').manual_seed(2)
    x = torch.randn(3, 128, 23, 31, generator=g).to('cuda', dt)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(256, 128, 1, 1, generator=g) * 0.05).cuda().requires_grad_(True)
    b = torch.randn(256, generator=g).cuda().requires_grad_(True)
    y = _Head1x1.apply(x, w, b)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().to(dt).float().requires_grad_(True)
    br = b.detach().clone().requires_grad_(True)
    ref = torch.nn.functional.conv2d(xr, wr, br)
    assert y.shape == ref.shape and y.dtype == dt
    torch.testing.assert_close(y.float(), ref, atol=3e-2, rtol=1e-2)
    gy = torch.randn(ref.shape, generator=g).cuda()
    (y.float() * gy).sum().backward()
    (ref * gy.to(dt).float()).sum().backward()
    rel = lambda a, r: ((a.float() - r).norm() / r.norm()).item()
    assert rel(x.grad, xr.grad) < 1e-2
    assert rel(w.grad, wr.grad) < 1e-2
    assert rel(b.grad, br.grad) < 1e-3


@pytest.mark.parametrize('cin,cout', [(64, 64), (96, 96), (128, 128), (96, 64), (64, 128)])
def test_native_wgrad_3x3_matches_conv2d(ext_ops, cin, cout):
    """Stride-1 3x3 encoder conv with the tap-fused weight gradient (Cout <= 64 -> 64-wide Cout
    tiles; Cin = 96 -> a 32-channel tail chunk) vs the autograd of F.conv2d at the same bf16
    inputs (fp32 reference of the products)."""
    torch.manual_seed(3)
    x = torch.randn(3, cin, 37, 45, device=DEV).to(torch.bfloat16)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.05).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    dy = torch.randn(3, cout, 37, 45, device=DEV).to(torch.bfloat16)
    dy = dy.contiguous(memory_format=torch.channels_last)
    y = fast._Conv3x3WgradNative.apply(x, w)
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, 1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    s = wr.grad.abs().max().item()
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=1e-2 * s, rtol=1e-2)
    assert w.grad.dtype == torch.bfloat16 and w.grad.shape == w.shape
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2 * xr.grad.abs().max().item(),
                               rtol=2e-2)


@pytest.mark.parametrize('cin,cout,hw', [(64, 64, (37, 45)), (64, 64, (8, 16)), (64, 64, (19, 70)),
                                         (128, 128, (37, 45)), (64, 128, (37, 45)),
                                         (96, 96, (23, 31)), (64, 96, (11, 19)), (96, 128, (9, 14))])
@pytest.mark.parametrize('packed', [False, True])
@pytest.mark.parametrize('dt', [torch.bfloat16, H16])
def test_native_conv_3x3_matches_conv2d(ext_ops, cin, cout, hw, packed, dt):
    """Stride-1 3x3 encoder conv entirely on the MFMA kernels (forward implicit GEMM -- or, 64 -> 64,
    the persistent 2-D halo-tile kernel --, input gradient on the flipped weight, tap-fused weight
    gradient) vs the fp32 autograd of F.conv2d at the same bf16 inputs, across image and batch
    borders and partial 8 x 16 tiles."""
    torch.manual_seed(4)
    h, wd = hw
    x = torch.randn(3, cin, h, wd, device=DEV).to(dt)
    x = x.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) * 0.05).to(dt)
    w = w.contiguous(memory_format=torch.channels_last).requires_grad_(True)
    dy = torch.randn(3, cout, h, wd, device=DEV).to(dt)
    dy = dy.contiguous(memory_format=torch.channels_last)
    wd = wf = None
    if packed:
        # the batched cast's adjoint / padded forward packs (96-channel K slots read zeros)
        conv = torch.nn.Conv2d(cin, cout, 3, padding=1).to(DEV)
        with torch.no_grad():
            conv.weight.copy_(w.float())
        _, adj, fwd = fast.cast_conv_weights([conv], dt)
        wd, wf = adj[conv], fwd.get(conv)
        assert (wf is not None) == (cin % 64 != 0)
    y = fast._Conv3x3Native.apply(x, w, wd, wf)
    assert y.is_contiguous(memory_format=torch.channels_last) and y.dtype == dt
    assert w.grad is None
    y.backward(dy)
    xr = x.detach().float().requires_grad_(True)
    wr = w.detach().float().requires_grad_(True)
    yr = torch.nn.functional.conv2d(xr, wr, None, 1, 1)
    yr.backward(dy.float())
    torch.testing.assert_close(y.float(), yr, atol=3e-2, rtol=2e-2)
    s = wr.grad.abs().max().item()
    torch.testing.assert_close(w.grad.float(), wr.grad, atol=1e-2 * s, rtol=1e-2)
    assert w.grad.dtype == dt
    torch.testing.assert_close(x.grad.float(), xr.grad, atol=3e-2 * xr.grad.abs().max().item(),
                               rtol=2e-2)
    # no-grad path (inference) gives the same forward
    with torch.no_grad():
        y2 = fast._conv3x3_native_fwd(x.detach(), w.detach(), wf)
    assert torch.equal(y2, y.detach())


@pytest.mark.parametrize('cls,norm,train', [
    (BasicEncoder, 'instance', True), (BasicEncoder, 'batch', True), (BasicEncoder, 'batch', False),
    (SmallEncoder, 'instance', True)])
def test_fast_encoder_fp32_matches_eager_split(ext_ops, cls, norm, train):
    """fp32 model (no autocast) inside the split-conv scope: the channels-last fast path (fp32
    norm kernels, split-bf16 stride-1 convs, MIOpen fp32 strided convs) gives the eager module
    path's outputs, parameter gradients and BatchNorm running statistics (same split convs,
    ATen norms) to fp32 rounding."""
    from pytorch_raft_amd.ops import conv_fp32
    torch.manual_seed(0)
    enc = cls(output_dim=256 if cls is BasicEncoder else 128, norm_fn=norm).to(DEV)
    for m in enc.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
            m.running_mean.uniform_(-0.1, 0.1)
            m.running_var.uniform_(0.8, 1.2)
        if isinstance(m, torch.nn.Conv2d):
            m.bias.data.uniform_(-0.1, 0.1)
    enc.train(train)
    x = torch.randn(4, 3, 96, 128, device=DEV)
    state = {k: v.clone() for k, v in enc.state_dict().items()}
    outs, grads, bufs = {}, {}, {}
    for path in ('eager', 'fast'):
        enc.load_state_dict(state)
        enc.zero_grad(set_to_none=True)
        orig = fast.fast_path_ok
        if path == 'eager':
            fast.fast_path_ok = lambda *a: False
        try:
            with conv_fp32.enabled():
                if path == 'fast':
                    assert fast.fast_path_ok(enc, x)
                y = enc(x)
        finally:
            fast.fast_path_ok = orig
        assert y.dtype == torch.float32
        (y * torch.linspace(-1, 1, y.numel(), device=DEV).view(y.shape)).sum().backward()
        outs[path] = y.detach()
        grads[path] = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
        bufs[path] = {k: v.clone() for k, v in enc.state_dict().items() if 'running' in k}
    rel = ((outs['fast'] - outs['eager']).norm() / outs['eager'].norm()).item()
    assert rel < 1e-4, rel
    for n, g in grads['eager'].items():
        normed_bias = n != 'conv2.bias' and n.endswith(('conv1.bias', 'conv2.bias', 'conv3.bias',
                                                         'downsample.0.bias'))
        if normed_bias and norm != 'none' and not (norm == 'batch' and not train):
            continue   # ~0 in exact arithmetic (the bias cancels in a batch-statistics norm)
        # the two paths round differently near ReLU kinks (norm statistics summed in another
        # order, conv bias folded into the norm): gradients agree to ~1e-4 in direction
        assert _cos(grads['fast'][n], g) > 0.999, (n, _cos(grads['fast'][n], g))
    for k, v in bufs['eager'].items():
        torch.testing.assert_close(bufs['fast'][k], v, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize('C', [64, 96, 128])
def test_instance_norm_kernels_match_fp32(ext_ops, C):
    """Instance-norm kernels (statistics, fixed-order reduce + finalize, apply; backward): forward
    and backward match the fp32 instance norm, and repeated calls with different batch sizes are
    bitwise reproducible."""
    import torch.nn.functional as F
    outs = []
    for n in (3, 5, 3):
        torch.manual_seed(7 if n == 3 else 8)
        x = (torch.randn(n, C, 40, 52, device=DEV) * 2 + 0.5).to(torch.bfloat16)
        x = x.contiguous(memory_format=torch.channels_last)
        cb = torch.randn(C, device=DEV) * 0.1
        y = torch.empty_like(x)
        mean, invstd = ext_ops.norm_fwd_(x, 0, 1, None, None, cb, None, None, 0.1, 1e-5, None, y)
        dy = torch.randn(x.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        dc = torch.empty(C, device=DEV)
        ext_ops.norm_bwd_(dy, x, None, mean, invstd, 0, 1, None, None, None, None, dc, dx)
        xr = x.float().requires_grad_(True)
        cr = cb.clone().requires_grad_(True)
        yr = F.relu(F.instance_norm(xr + cr.view(1, -1, 1, 1), eps=1e-5))
        yr.backward(dy.float())
        torch.testing.assert_close(y.float(), yr.detach(), atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(dx.float(), xr.grad, atol=3e-2, rtol=3e-2)
        outs.append((y.clone(), dx.clone(), mean.clone(), invstd.clone()))
    for a, b in zip(outs[0], outs[2]):
        assert torch.equal(a, b)


@pytest.mark.parametrize('C,hw', [(64, (160, 120)), (128, (48, 64))])
def test_batch_norm_kernels_match_fp32(ext_ops, C, hw):
    """Training-mode batch norm with a long partial list (C=64 here: 75 per-workgroup partial
    rows, the 16-lane reduce + finalize): forward, running stats and backward vs the fp32 batch
    norm, bitwise reproducible across calls."""
    import torch.nn.functional as F
    outs = []
    for rep in range(2):
        torch.manual_seed(3)
        x = (torch.randn(4, C, *hw, device=DEV) * 1.5 - 0.3).to(torch.bfloat16)
        x = x.contiguous(memory_format=torch.channels_last)
        gm = torch.rand(C, device=DEV) + 0.5
        bt = torch.randn(C, device=DEV) * 0.2
        rm, rv = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        y = torch.empty_like(x)
        mean, invstd = ext_ops.norm_fwd_(x, 1, 1, gm, bt, None, rm, rv, 0.1, 1e-5, None, y)
        dy = torch.randn(x.shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x)
        dg, db = torch.empty(C, device=DEV), torch.empty(C, device=DEV)
        ext_ops.norm_bwd_(dy, x, None, mean, invstd, 1, 1, gm, bt, dg, db, None, dx)
        xr = x.float().requires_grad_(True)
        gr, br = gm.clone().requires_grad_(True), bt.clone().requires_grad_(True)
        rm2, rv2 = torch.zeros(C, device=DEV), torch.ones(C, device=DEV)
        yr = F.relu(F.batch_norm(xr, rm2, rv2, gr, br, training=True, momentum=0.1, eps=1e-5))
        yr.backward(dy.float())
        torch.testing.assert_close(y.float(), yr.detach(), atol=3e-2, rtol=2e-2)
        torch.testing.assert_close(rm, rm2, atol=1e-4, rtol=1e-4)
        torch.testing.assert_close(rv, rv2, atol=1e-4, rtol=1e-3)
        torch.testing.assert_close(dx.float(), xr.grad, atol=3e-2, rtol=3e-2)
        torch.testing.assert_close(dg, gr.grad, atol=5e-2, rtol=1e-2)
        torch.testing.assert_close(db, br.grad, atol=5e-2, rtol=1e-2)
        outs.append((y.clone(), dx.clone(), dg.clone(), db.clone()))
    for a, b in zip(outs[0], outs[1]):
        assert torch.equal(a, b)


@pytest.mark.parametrize('dt,hd,c', [(torch.bfloat16, 128, 256), (torch.float16, 128, 256),
                                     (torch.bfloat16, 96, 160)])
def test_context_act_matches_eager(ext_ops, dt, hd, c):
    """net, inp = tanh / relu of the context encoder's halves in one native pass (NHWC outputs)
    vs the eager split + tanh + relu, forward and backward (one missing gradient included)."""
    torch.manual_seed(0)
    cnet = (torch.randn(3, c, 23, 31, device=DEV) * 2).to(dt).contiguous(memory_format=torch.channels_last)
    gh = torch.randn(3, hd, 23, 31, device=DEV).to(dt)
    gx = torch.randn(3, c - hd, 23, 31, device=DEV).to(dt)
    for use_gh in (True, False):
        a = cnet.clone().requires_grad_(True)
        net, inp = fast.context_act(a, hd)
        assert net.permute(0, 2, 3, 1).is_contiguous() and inp.permute(0, 2, 3, 1).is_contiguous()
        b = cnet.clone().requires_grad_(True)
        rn, ri = torch.split(b, [hd, c - hd], dim=1)
        rn, ri = torch.tanh(rn), torch.relu(ri)
        torch.testing.assert_close(net.float(), rn.float(), atol=0, rtol=1e-2)
        assert torch.equal(inp, ri)
        # without use_gh the net output takes no part: its gradient arrives as None
        (((net * gh).float().sum() if use_gh else 0) + (inp * gx).float().sum()).backward()
        (((rn * gh).float().sum() if use_gh else 0) + (ri * gx).float().sum()).backward()
        torch.testing.assert_close(a.grad.float(), b.grad.float(), atol=1e-2, rtol=2e-2)


@pytest.mark.parametrize('C', [64, 96])
def test_norm_split_outputs_match_split_hilo(ext_ops, C):
    """fp32 schedule: the norm apply passes also write y / dx as the split-bf16 conv operand --
    bitwise what split_hilo makes of them, padding channels zero."""
    from pytorch_raft_amd.ops import conv_fp32
    torch.manual_seed(0)
    x = torch.randn(2, C, 19, 27, device=DEV).contiguous(memory_format=torch.channels_last)
    pad = (C + 63) // 64 * 64
    y = torch.empty_like(x)
    ys = torch.full((2, 19, 27, 2 * pad), 3.0, device=DEV, dtype=torch.bfloat16)
    mean, invstd = ext_ops.norm_fwd_(x, 0, 1, None, None, None, None, None, 0.1, 1e-5, None, y, ys)
    assert torch.equal(ys, conv_fp32._split_nhwc(y, pad))
    dy = torch.randn(x.shape, device=DEV).contiguous(memory_format=torch.channels_last)
    dx = torch.empty_like(x)
    dxs = torch.full((2, 19, 27, 2 * pad), 3.0, device=DEV, dtype=torch.bfloat16)
    ext_ops.norm_bwd_(dy, x, None, mean, invstd, 0, 1, None, None, None, None, None, dx,
                      None, None, None, dxs)
    assert torch.equal(dxs, conv_fp32._split_nhwc(dx, pad))


@pytest.mark.parametrize('dt', [torch.bfloat16, H16])
@pytest.mark.parametrize('n,hw', [(6, (184, 248)), (5, (37, 45)), (1, (9, 17))])
def test_enc64_plain_kernel_matches(ext_ops, dt, n, hw):
    """The plain conv_enc64 launch (the producer / MFMA-wave kernel; RAFT_ENC64_KERNEL=half / wg1
    select the others) gives bitwise the output of the one-workgroup-per-CU kernel (the
    statistics launch), over many persistent items per workgroup (6 x 184 x 248: 2,208 tiles),
    with partial edge tiles and with a tile count that is not a multiple of 8 (dead work items);
    and both match an fp32 conv."""
    from pytorch_raft_amd.ops.encoder import _enc64_tiles
    torch.manual_seed(11)
    h, w = hw
    x = torch.randn(n, h, w, 64, device=DEV).to(dt)
    wt = (torch.randn(64, 64, 3, 3, device=DEV) / 24.0).to(dt)
    wpk = wt.permute(0, 2, 3, 1).reshape(64, 576).contiguous()
    out = torch.full((n, h, w, 64), 7.0, device=DEV, dtype=dt)
    ext_ops.conv_enc64_(x, wpk, out)
    ref_out = torch.empty_like(out)
    part = torch.empty(n * _enc64_tiles(h, w), 4, 64, device=DEV)
    ext_ops.conv_enc64_(x, wpk, ref_out, part)
    assert torch.equal(out, ref_out)
    ref = torch.nn.functional.conv2d(x.permute(0, 3, 1, 2).float(), wt.float(), None, 1, 1)
    err = (out.permute(0, 3, 1, 2).float() - ref).abs().max() / ref.abs().max()
    assert err.item() < 1e-2


@pytest.mark.parametrize('mode,dt', [(0, torch.bfloat16), (1, torch.bfloat16), (0, H16)])
@pytest.mark.parametrize('hw', [(40, 64), (23, 37)])
def test_enc64_tile_stats_feed_the_norm(ext_ops, mode, dt, hw):
    """conv_enc64's epilogue statistics (per 8 x 16 tile: shifted sums, shift, count) give the
    norm the same mean / invstd / output as its own statistics pass over the conv output, also
    with partial edge tiles (23 x 37) and a mean far from zero."""
    from pytorch_raft_amd.ops.encoder import _enc64_tiles
    torch.manual_seed(5)
    n, (h, w) = 3, hw
    x = (torch.randn(n, h, w, 64, device=DEV) + 0.3).to(dt)
    # weights with a positive mean: conv outputs with a per-channel mean of ~3.5 at std ~1
    wpk = (torch.randn(64, 9 * 64, device=DEV) / 24 + 0.02).to(dt)
    out = torch.empty(n, h, w, 64, device=DEV, dtype=dt)
    tiles = _enc64_tiles(h, w)
    part = torch.empty(n * tiles, 4, 64, device=DEV)
    ext_ops.conv_enc64_(x, wpk, out, part)
    out2 = torch.empty_like(out)
    ext_ops.conv_enc64_(x, wpk, out2)
    assert torch.equal(out, out2)
    assert (part[:, 3].sum(0) == n * h * w).all()
    xc = out.permute(0, 3, 1, 2)                 # channels_last (B, C, H, W) view
    assert xc.is_contiguous(memory_format=torch.channels_last)
    assert out.float().mean().item() > 2.0
    gm = torch.rand(64, device=DEV) + 0.5 if mode == 1 else None
    bt = torch.randn(64, device=DEV) * 0.2 if mode == 1 else None
    res = {}
    for key, extra in (('pass', ()), ('tiles', (part, tiles))):
        rm = torch.zeros(64, device=DEV) if mode == 1 else None
        rv = torch.ones(64, device=DEV) if mode == 1 else None
        y = torch.empty_like(xc)
        mean, invstd = ext_ops.norm_fwd_(xc, mode, 1, gm, bt, None, rm, rv, 0.1, 1e-5, None, y,
                                         None, *extra)
        res[key] = (mean, invstd, y, rm, rv)
    (m0, i0, y0, rm0, rv0), (m1, i1, y1, rm1, rv1) = res['pass'], res['tiles']
    torch.testing.assert_close(m1, m0, atol=1e-5, rtol=1e-5)   # same values, other sum order
    torch.testing.assert_close(i1, i0, atol=1e-5, rtol=1e-4)
    torch.testing.assert_close(y1.float(), y0.float(), atol=2e-2, rtol=1e-2)
    if mode == 1:
        torch.testing.assert_close(rm1, rm0, atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(rv1, rv0, atol=1e-5, rtol=1e-4)


@pytest.mark.parametrize('C,dt', [(64, torch.bfloat16), (32, torch.bfloat16), (64, H16)])
@pytest.mark.parametrize('hw', [(40, 64), (37, 50)])
def test_stem_conv_matches_fp32(ext_ops, C, dt, hw):
    """The encoders' 7x7 stride-2 stem conv on stem_conv.hip (forward and weight gradient) vs the
    fp32 conv of the same 16-bit operands, also with partial edge tiles (37 x 50 -> 19 x 25)."""
    import torch.nn.functional as F
    torch.manual_seed(2)
    B, (H, W) = 3, hw
    x = torch.randn(B, 3, H, W, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(C, 3, 7, 7, device=DEV) / 8).to(dt).contiguous(memory_format=torch.channels_last)
    y = fast._stem_fwd(x, w)
    ref = F.conv2d(x.float(), w.float(), stride=2, padding=3)
    assert y.shape == ref.shape and y.dtype == dt
    err = (y.float() - ref).abs().max().item()
    assert err <= 2 ** -7 * ref.abs().max().item(), err
    gy = torch.randn(ref.shape, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
    dw = ext_ops.stem_conv_wgrad(x.permute(0, 2, 3, 1), gy.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
    wr = w.float().requires_grad_(True)
    F.conv2d(x.float(), wr, stride=2, padding=3).backward(gy.float())
    assert dw.shape == w.shape
    rel = ((dw.float() - wr.grad).norm() / wr.grad.norm()).item()
    assert rel < 5e-3, rel
    # deterministic: fixed-order partial sums
    dw2 = ext_ops.stem_conv_wgrad(x.permute(0, 2, 3, 1), gy.permute(0, 2, 3, 1)).permute(0, 3, 1, 2)
    assert torch.equal(dw, dw2)
    # the autograd node (weight gradient through the kernel, input gradient through ATen)
    xg = x.clone().requires_grad_(True)
    wg = w.clone().requires_grad_(True)
    fast._StemConv.apply(xg, wg).backward(gy)
    assert torch.equal(wg.grad.contiguous(), dw.contiguous())
    xr = x.float().requires_grad_(True)
    F.conv2d(xr, w.float(), stride=2, padding=3).backward(gy.float())
    rel = ((xg.grad.float() - xr.grad).norm() / xr.grad.norm()).item()
    assert rel < 1e-2, rel
