"""Split-fp32 operands on the MFMA kernels (the reference's fp32 schedule, `train_standard.sh`: no
--mixed_precision): every 16-bit activation is an fp32 value carried as a bf16 pair [hi | lo]
(hi at channel c, lo at c + C), each conv three bf16 products (ConvFwdArgs.spl, EPI_SPL).  Each
kernel is compared with a plain PyTorch fp64 op of the same fp32 operands; the bound is the
scheme's ~2^-16 relative rounding (a kernel bug gives O(1) errors)."""
import argparse

import pytest
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import conv as C

pytestmark = pytest.mark.gpu
DEV = 'cuda'
BF = torch.bfloat16
# LDS-DMA and halo configs of conv_igemm.hip's kCfgs (split fp32 runs only those kernel families)
SPL_CFGS = (10, 17, 16, 26, 30, 33)


def _split(x):
    """fp32 NHWC (..., C) -> bf16 [hi | lo] (..., 2C)."""
    hi = x.to(BF)
    return torch.cat([hi, (x - hi.float()).to(BF)], -1).contiguous()


def _join(xs):
    c = xs.shape[-1] // 2
    return xs[..., :c].double() + xs[..., c:].double()


def _nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def _rel(a, b):
    return ((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)).item()


def _pack(w, segs):
    return C.split_weight(C.pack_weight(w.float(), segs, segs, dtype=torch.float32),
                          w.shape[2] * w.shape[3])


@pytest.mark.parametrize('cfg', (-1,) + SPL_CFGS)
@pytest.mark.parametrize('cin,cout,k,epi', [
    (256, 192, (3, 3), C.EPI_RELU_BF16),
    (256, 256, (1, 5), C.EPI_BF16),
    (128, 128, (5, 1), C.EPI_F32),
    (256, 2, (3, 3), C.EPI_F32_NCHW),
])
def test_split_conv_fwd(ext_ops, cfg, cin, cout, k, epi):
    torch.manual_seed(0)
    B, H, W = 2, 13, 21
    x = torch.randn(B, cin, H, W, device=DEV)
    w = torch.randn(cout, cin, *k, device=DEV) / (cin * k[0] * k[1]) ** 0.5
    b = torch.randn(cout, device=DEV)
    pad = (k[0] // 2, k[1] // 2)
    ref = F.conv2d(x.double(), w.double(), b.double(), padding=pad)
    if epi == C.EPI_RELU_BF16:
        ref = ref.relu()
    if epi == C.EPI_F32_NCHW:
        out = torch.empty(B, cout, H, W, device=DEV)
    elif epi == C.EPI_F32:
        out = torch.empty(B, H, W, cout, device=DEV)
    else:
        out = torch.empty(B, H, W, 2 * cout, device=DEV, dtype=BF)
    ext_ops.conv_set_forced_cfg(cfg)
    try:
        C.conv_fwd([(_split(_nhwc(x)), 0, cin)], _pack(w, [cin]), b, k, pad, cout, epi | C.EPI_SPL,
                   [out], [0])
    finally:
        ext_ops.conv_set_forced_cfg(-1)
    if epi == C.EPI_F32_NCHW:
        got = out.double()
    elif epi == C.EPI_F32:
        got = out.double().permute(0, 3, 1, 2)
    else:
        got = _join(out).permute(0, 3, 1, 2)
    assert _rel(got, ref) < 3e-5, _rel(got, ref)


def test_split_gru_epilogues(ext_ops):
    """z | r gates and the q gate + state update on split operands, fp32 bias maps."""
    torch.manual_seed(2)
    B, H, W, hd = 2, 11, 17, 128
    h = torch.randn(B, hd, H, W, device=DEV).tanh()
    x = torch.randn(B, 128, H, W, device=DEV)
    wzr = torch.randn(2 * hd, hd + 128, 1, 5, device=DEV) / 40
    wq = torch.randn(hd, hd + 128, 1, 5, device=DEV) / 40
    bzr = torch.randn(B, H, W, 2 * hd, device=DEV) * 0.1   # per-pixel fp32 bias map
    bq = torch.randn(B, H, W, hd, device=DEV) * 0.1
    hs, xs = _split(_nhwc(h)), _split(_nhwc(x))
    z, rh, r = (torch.empty(B, H, W, 2 * hd, device=DEV, dtype=BF) for _ in range(3))
    C.conv_fwd([(hs, 0, hd), (xs, 0, 128)], _pack(wzr, [hd, 128]), bzr, (1, 5), (0, 2), 2 * hd,
               C.EPI_GRU_ZR | C.EPI_SPL, [z, rh, r], [0, 0, 0], aux=[hs], aux_offs=[0], split=hd)
    pre = F.conv2d(torch.cat([h, x], 1).double(), wzr.double(), None, padding=(0, 2)) + \
        bzr.double().permute(0, 3, 1, 2)
    z_ref, r_ref = torch.sigmoid(pre[:, :hd]), torch.sigmoid(pre[:, hd:])
    zf = _join(z).permute(0, 3, 1, 2)
    rf = _join(r).permute(0, 3, 1, 2)
    assert _rel(zf, z_ref) < 2e-5 and _rel(rf, r_ref) < 2e-5
    assert _rel(_join(rh).permute(0, 3, 1, 2), r_ref * h.double()) < 3e-5
    h2, q = torch.empty_like(z), torch.empty_like(z)
    C.conv_fwd([(rh, 0, hd), (xs, 0, 128)], _pack(wq, [hd, 128]), bq, (1, 5), (0, 2), hd,
               C.EPI_GRU_Q | C.EPI_SPL, [h2, q], [0, 0], aux=[hs, z], aux_offs=[0, 0])
    rhd = _join(rh).permute(0, 3, 1, 2)
    q_ref = torch.tanh(F.conv2d(torch.cat([rhd, x.double()], 1), wq.double(), None, padding=(0, 2)) +
                       bq.double().permute(0, 3, 1, 2))
    assert _rel(_join(q).permute(0, 3, 1, 2), q_ref) < 3e-5
    want = h.double() + zf * (q_ref - h.double())
    assert _rel(_join(h2).permute(0, 3, 1, 2), want) < 3e-5


def test_split_dgrad_and_wgrad(ext_ops):
    """Input gradient (fp32 output, ReLU-gated split output) and the tap-fused weight / bias
    gradient (three products per item: g_hi x_hi + g_lo x_hi + g_hi x_lo) vs fp64 autograd."""
    torch.manual_seed(3)
    B, H, W, cin, cout, k = 2, 13, 19, 128, 256, (3, 3)
    x = torch.randn(B, cin, H, W, device=DEV)
    w = torch.randn(cout, cin, *k, device=DEV) / 30
    g = torch.randn(B, cout, H, W, device=DEV)
    xr = x.double().requires_grad_(True)
    wr = w.double().requires_grad_(True)
    br = torch.zeros(cout, device=DEV, dtype=torch.float64, requires_grad=True)
    F.conv2d(xr, wr, br, padding=1).backward(g.double())
    wd = _pack(w.flip(2, 3).transpose(0, 1).contiguous(), [cout])
    gs = _split(_nhwc(g))
    dx = torch.empty(B, H, W, cin, device=DEV)
    ext_ops.conv_dgrad_([gs], [0], [cout], wd, 3, 3, 1, 1, 0, 1.0, [dx], [0], [cin], [cin], [0],
                        [dx], [0], [], [], [], True)
    assert _rel(dx.permute(0, 3, 1, 2), xr.grad) < 3e-5
    # ReLU-gated split output
    y = torch.randn(B, cin, H, W, device=DEV).relu()
    ys = _split(_nhwc(y))
    dxg = torch.empty(B, H, W, 2 * cin, device=DEV, dtype=BF)
    ext_ops.conv_dgrad_([gs], [0], [cout], wd, 3, 3, 1, 1, 0, 1.0, [dxg], [0], [cin], [cin], [0],
                        [ys], [0], [], [], [], True)
    want = xr.grad * (y > 0)
    assert _rel(_join(dxg).permute(0, 3, 1, 2), want) < 3e-5
    # weight / bias gradient over two items (iterations)
    dw = torch.zeros(cout, 9 * cin, device=DEV)
    db = torch.zeros(cout, device=DEV)
    xs = _split(_nhwc(x))
    C.conv_wgrad_multi([(gs, [xs]), (gs, [xs])], 0, [0], [cin], k, (1, 1), cout, dw, db, split=True)
    got = C.unpack_weight_grad(dw, cout, [cin], [cin], k)
    assert _rel(got, 2 * wr.grad) < 3e-5
    assert _rel(db, 2 * br.grad) < 1e-5


@pytest.mark.parametrize('w', [31, 32])
def test_split_lookup_patch_and_fold(ext_ops, w):
    """Split taps from the fp32 pyramid == the fp32 lookup to 2^-16; the fold of split tap
    gradients (even width: the union-box fold with fp32 dC) == the generic fp32 lookup
    backward; the split im2col patch == the fp32 flow."""
    b, c, h = 2, 256, 23
    f1 = torch.randn(b, c, h, w, device=DEV)
    f2 = torch.randn(b, c, h, w, device=DEV)
    pyr = ext_ops.corr_build(f1, f2, 4)
    ys, xs_ = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    gen = torch.Generator(device='cpu').manual_seed(0)
    coords = (torch.stack([xs_, ys])[None].repeat(b, 1, 1, 1) +
              3 * torch.randn(b, 2, h, w, generator=gen)).to(DEV)
    out = torch.empty(b, h, w, 768, device=DEV, dtype=BF)
    ext_ops.corr_lookup_nhwc_(pyr, coords, 4, out, True)
    ref = ext_ops.corr_lookup_fwd(pyr, coords, 4).permute(0, 2, 3, 1)
    got = _join(out)
    assert (got[..., 324:384] == 0).all()
    err = (got[..., :324] - ref.double()).abs().max().item()
    assert err <= 2.0 ** -15 * ref.abs().max().item(), err
    taps = [torch.randn(b, h, w, 384, device=DEV) for _ in range(3)]
    cs = [coords + k * 0.3 for k in range(3)]
    dsplit = ext_ops.corr_tap_reduce(cs, [_split(t) for t in taps], h, w, 4, 4, 1 / 16, False, 0, True)
    gp = [torch.zeros_like(p) for p in pyr]
    for cc, t in zip(cs, taps):
        ext_ops.corr_lookup_bwd_(gp, cc, t.contiguous(), 4)
    dref = ext_ops.corr_pyr_grad_reduce(gp, 1 / 16)
    assert _rel(dsplit, dref) < 3e-5
    # convf1's split im2col patch + the flow slot of the motion features
    flow = torch.randn(b, 2, h, w, device=DEV) * 20
    patch = torch.empty(b, h, w, 256, device=DEV, dtype=BF)
    mf = torch.zeros(b, h, w, 256, device=DEV, dtype=BF)
    ext_ops.f1_patch_(flow, patch, mf, 126)
    unf = F.unfold(flow.double(), 7, padding=3).view(b, 2, 49, h, w)
    want = unf.permute(0, 3, 4, 2, 1).reshape(b, h, w, 98)
    pj = _join(patch)
    assert (pj[..., 98:] == 0).all()
    assert (pj[..., :98] - want).abs().max().item() <= 2.0 ** -16 * 20 * 8
    assert (_join(mf)[..., 126:128] - flow.double().permute(0, 2, 3, 1)).abs().max().item() <= 2.0 ** -16 * 20 * 8


@pytest.mark.parametrize('iters,wm,wd_', [(2, 1.0, 1.0), (1, 0.0, 1.0), (1, 1.0, 0.0)])
def test_fp32_fused_update_iteration_vs_fp64(ext_ops, iters, wm, wd_):
    """Two iterations of the fused update block on split-fp32 operands (HipUpdateBlock(dtype=
    fp32)) vs the module's eager fp64 forward / backward: h', delta, mask and every parameter,
    state, context and correlation gradient."""
    from pytorch_raft_amd.models.update import BasicUpdateBlock
    from pytorch_raft_amd.ops.update_hip import HipUpdateBlock, CORR_BUF, split_nhwc
    torch.manual_seed(5)
    args = argparse.Namespace(corr_levels=4, corr_radius=4)
    ub = BasicUpdateBlock(args, hidden_dim=128).to(DEV)
    for p in ub.parameters():
        p.data.mul_(1.5)
    B, H, W = 2, 12, 15
    net = torch.randn(B, 128, H, W, device=DEV).tanh()
    inp = torch.randn(B, 128, H, W, device=DEV).relu()
    corrs = [torch.randn(B, 324, H, W, device=DEV) for _ in range(2)]
    flows = [torch.randn(B, 2, H, W, device=DEV) * 3 for _ in range(2)]
    gd = [torch.randn(B, 2, H, W, device=DEV) * wd_ for _ in range(2)]
    gm = [torch.randn(B, 576, H, W, device=DEV) * wm for _ in range(2)]
    # fused, split fp32; its ReLU outputs are kept to replay the same ReLU masks in the eager
    # references (a pre-activation within the split scheme's ~2^-16 rounding of zero flips its
    # mask -- one flip in a 12 x 15 test image moves the upstream gradients by ~1e-2)
    from pytorch_raft_amd.ops import update_hip as U
    saved = []
    orig_fwd = U._iter_forward

    def keep(*a, **k):
        out = orig_fwd(*a, **k)
        saved.append(out[3])
        return out

    U._iter_forward = keep
    leaves = [t.clone().requires_grad_(True) for t in [net, inp] + corrs]
    hub = HipUpdateBlock(ub, dtype=torch.float32)
    h = split_nhwc(leaves[0])
    x = split_nhwc(leaves[1])
    loss = 0
    for i in range(iters):
        cs = split_nhwc(leaves[2 + i], CORR_BUF)
        h, delta, mask = hub(h, x, cs, flows[i])
        assert mask.dtype == torch.float32 and delta.dtype == torch.float32
        loss = loss + (delta * gd[i]).sum() + (mask.permute(0, 3, 1, 2) * gm[i]).sum()
    hf = h
    U._iter_forward = orig_fwd
    loss.backward()
    masks = []   # ReLU call order of one eager iteration (models/update.py)
    for sv in saved:
        c1, cf, f1, mf, fm = (_join(t.detach()).permute(0, 3, 1, 2) > 0 for t in
                              (sv[2], sv[3], sv[4], sv[5], sv[-1]))
        masks += [c1, cf[:, :192], f1, cf[:, 192:256], mf[:, :126], fm[:, :256], fm[:, 256:512]]
    grads = {n: (p.grad.clone() if p.grad is not None else torch.zeros_like(p))
             for n, p in ub.named_parameters()}
    lgrads = [t.grad.clone() if t.grad is not None else None for t in leaves]
    # eager fp64 reference, and eager fp32 (MIOpen / ATen) as the yardstick of fp32 rounding
    def eager(dtype):
        m = BasicUpdateBlock(args, hidden_dim=128).to(DEV).to(dtype)
        m.load_state_dict(ub.state_dict())
        lv = [t.detach().to(dtype).requires_grad_(True) for t in [net, inp] + corrs]
        hh, tot = lv[0], 0
        queue = list(masks)
        relu = F.relu
        F.relu = lambda x, inplace=False: x * queue.pop(0).to(x.dtype)
        try:
            for i in range(iters):
                hh, mk, dl = m(hh, lv[1], lv[2 + i], flows[i].to(dtype))
                tot = tot + (dl * gd[i].to(dtype)).sum() + (mk * gm[i].to(dtype)).sum()
        finally:
            F.relu = relu
        assert not queue
        tot.backward()
        return hh.detach(), tot.item(), {n: (p.grad if p.grad is not None else torch.zeros_like(p))
                                          for n, p in m.named_parameters()}, [t.grad for t in lv]

    h64, loss64, g64, l64 = eager(torch.float64)
    _, _, g32, l32 = eager(torch.float32)
    assert _rel(_join(hf).permute(0, 3, 1, 2), h64) < 1e-4
    assert abs(loss.item() - loss64) <= 1e-4 * abs(loss64)
    # the split scheme rounds every operand to ~2^-16 (fp32: 2^-24), and the backward through two
    # GRU iterations amplifies that; bounded by 1e-3 and by 50x eager fp32's own error
    report = [(n, _rel(grads[n], g64[n]), _rel(g32[n], g64[n])) for n in g64 if g64[n].norm() > 0]
    report += [('input%d' % i, _rel(a, b64), _rel(b32, b64))
               for i, (a, b64, b32) in enumerate(zip(lgrads, l64, l32)) if b64 is not None]
    # with the masks shared, the split scheme's ~2^-16 rounding through two GRU iterations:
    # ~1e-5 measured (eager fp32: ~7e-7)
    bad = [r for r in report if not r[1] < max(1e-4, 50 * r[2])]
    for r in report:
        print('%-32s %.3e %.3e' % r)
    assert not bad, bad[:4]


def test_fp32_model_uses_fused_split_block(ext_ops):
    """An fp32 RAFT (no mixed precision) decodes through the fused split-fp32 block: a training
    step's flow and update-block gradients match the MIOpen fp32 eager block (update_impl=
    'torch') to the split scheme's rounding."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    from pytorch_raft_amd.ops import update_hip
    outs = {}
    calls = {'n': 0}
    orig = update_hip._iter_forward

    def counting(pk, *a, **k):
        calls['n'] += int(pk.spl)
        return orig(pk, *a, **k)

    update_hip._iter_forward = counting
    try:
        for impl in ('auto', 'torch'):
            args = argparse.Namespace(small=False, mixed_precision=False, update_impl=impl)
            torch.manual_seed(0)
            m = RAFT(args).to(DEV).train()
            i1, i2, flow, valid = (t.to(DEV) for t in make_pair_batch(2, 128, 160, seed=3))
            preds = m(i1, i2, iters=3)
            loss, _ = sequence_loss(preds, flow, valid, 0.8)
            loss.backward()
            outs[impl] = (preds[-1].detach(), {n: p.grad.detach().clone()
                                               for n, p in m.named_parameters() if p.grad is not None})
    finally:
        update_hip._iter_forward = orig
    assert calls['n'] == 3
    (fa, ga), (fb, gb) = outs['auto'], outs['torch']
    assert _rel(fa, fb) < 1e-3
    # ReLU-mask flips at this tiny size (see test_conv_fp32_gpu.py): the kernels' own precision
    # is pinned by test_fp32_fused_update_iteration_vs_fp64
    for n in gb:
        if n.startswith('update_block'):
            assert _rel(ga[n], gb[n]) < 2e-2, n


@pytest.mark.parametrize('cfg', (-1,) + SPL_CFGS)
def test_split_dgrad_1x1_sliced_relu_output(ext_ops, cfg):
    """The mask head's input gradient on split operands: 1x1, 576 -> 256 channels written with
    scale 0.25 into channels [256, 512) of a 512-wide split buffer, ReLU-gated by channels
    [256, 512) of a 512-wide split forward output."""
    torch.manual_seed(8)
    B, H, W = 2, 12, 15
    g = torch.randn(B, 576, H, W, device=DEV)
    w = torch.randn(576, 256, 1, 1, device=DEV) / 16
    fm = torch.randn(B, 512, H, W, device=DEV).relu()
    wd = _pack(w.flip(2, 3).transpose(0, 1).contiguous(), [576])
    from pytorch_raft_amd.ops.update_hip import _to_split
    gs = _to_split(g)
    assert torch.equal(gs, _split(_nhwc(g)))
    fms = _split(_nhwc(fm))
    out = torch.zeros(B, H, W, 1024, device=DEV, dtype=BF)
    ext_ops.conv_set_forced_cfg(cfg)
    try:
        ext_ops.conv_dgrad_([gs], [0], [576], wd, 1, 1, 0, 0, 0, 0.25, [out], [256], [256], [256],
                            [0], [fms], [256], [], [], [], True)
    finally:
        ext_ops.conv_set_forced_cfg(-1)
    ref = 0.25 * F.conv2d(g.double(), w.double().transpose(0, 1)) * (fm[:, 256:] > 0)
    got = _join(out)
    assert (got[..., :256] == 0).all()
    assert _rel(got[..., 256:].permute(0, 3, 1, 2), ref) < 3e-5


def test_split_gru_relu_bwd_kernels_vs_fp64(ext_ops):
    """gru_q_bwd_ / gru_zr_bwd_ / relu_bwd_ on split pair buffers (the small block's fp32
    schedule): the GRU gate algebra and the ReLU-gated cast on hi + lo values, outputs re-split."""
    torch.manual_seed(11)
    B, H, W, hd = 2, 6, 7, 128
    z, q, r, hp = (torch.rand(B, H, W, hd, device=DEV) * 2 - 1 for _ in range(4))
    z, r = z.sigmoid(), r.sigmoid()
    zs, qs, rs, hs = (_split(t) for t in (z, q, r, hp))
    zd, qd, rd, hd_ = (_join(t) for t in (zs, qs, rs, hs))
    dh = torch.randn(B, H, W, hd, device=DEV)
    dpre_q = torch.empty(B, H, W, 2 * hd, device=DEV, dtype=BF)
    dz = torch.empty(B, H, W, hd, device=DEV)
    dhp = torch.empty(B, H, W, hd, device=DEV)
    ext_ops.gru_q_bwd_(dh, zs, qs, hs, dpre_q, dz, dhp)
    g = dh.double()
    assert _rel(_join(dpre_q), g * zd * (1 - qd * qd)) < 1e-5
    assert _rel(dz, g * (qd - hd_)) < 1e-6
    assert _rel(dhp, g * (1 - zd)) < 1e-6
    drh = torch.randn(B, H, W, hd, device=DEV)
    dhp0 = dhp.double().clone()
    dzr = torch.empty(B, H, W, 4 * hd, device=DEV, dtype=BF)
    ext_ops.gru_zr_bwd_(drh, dz, zs, rs, hs, dzr, dhp)
    zr_hi, zr_lo = dzr[..., :2 * hd].double(), dzr[..., 2 * hd:].double()
    zr = zr_hi + zr_lo
    assert _rel(zr[..., :hd], dz.double() * zd * (1 - zd)) < 1e-5
    assert _rel(zr[..., hd:], drh.double() * hd_ * rd * (1 - rd)) < 1e-5
    assert _rel(dhp, dhp0 + drh.double() * rd) < 1e-6
    # relu_bwd_: channels [0, 80) of a 128-wide fp32 gradient, gated by a split forward output
    gm = torch.randn(B, H, W, 128, device=DEV)
    y = torch.randn(B, H, W, 128, device=DEV)
    ys = _split(y)
    out = torch.zeros(B, H, W, 256, device=DEV, dtype=BF)
    ext_ops.relu_bwd_(gm, 0, ys, 0, out, 0, 80, 1.0, True)
    got = _join(out)
    assert (got[..., 80:] == 0).all()
    assert _rel(got[..., :80], gm[..., :80].double() * (_join(ys)[..., :80] > 0)) < 1e-5


def test_fp32_small_fused_iteration_vs_fp64(ext_ops):
    """Two iterations of the fused RAFT-small block on split-fp32 operands
    (HipSmallUpdateBlock(dtype=fp32)) vs the module's eager fp64 forward / backward, ReLU masks
    shared (see test_fp32_fused_update_iteration_vs_fp64): h', delta and every parameter,
    state, context and correlation gradient."""
    from pytorch_raft_amd.models.update import SmallUpdateBlock
    from pytorch_raft_amd.ops import update_hip_small as S
    from pytorch_raft_amd.ops.update_hip import split_nhwc
    torch.manual_seed(6)
    args = argparse.Namespace(corr_levels=4, corr_radius=3)
    ub = SmallUpdateBlock(args, hidden_dim=96).to(DEV)
    for p in ub.parameters():
        p.data.mul_(1.5)
    B, H, W, iters = 2, 12, 15, 2
    net = torch.randn(B, 96, H, W, device=DEV).tanh()
    inp = torch.randn(B, 64, H, W, device=DEV).relu()
    corrs = [torch.randn(B, 196, H, W, device=DEV) for _ in range(iters)]
    flows = [torch.randn(B, 2, H, W, device=DEV) * 3 for _ in range(iters)]
    gd = [torch.randn(B, 2, H, W, device=DEV) for _ in range(iters)]
    saved = []
    orig_fwd = S._iter_forward

    def keep(*a, **k):
        out = orig_fwd(*a, **k)
        saved.append(out[2])
        return out

    S._iter_forward = keep
    try:
        leaves = [t.clone().requires_grad_(True) for t in [net, inp] + corrs]
        hub = S.HipSmallUpdateBlock(ub, dtype=torch.float32)
        h = split_nhwc(leaves[0], S.HDP)
        x = split_nhwc(leaves[1])
        loss = 0
        for i in range(iters):
            cs = split_nhwc(leaves[2 + i], S.CORR_BUF_SMALL)
            h, delta = hub(h, x, cs, flows[i])
            assert delta.dtype == torch.float32
            loss = loss + (delta * gd[i]).sum()
        hf = h
    finally:
        S._iter_forward = orig_fwd
    loss.backward()
    masks = []   # ReLU call order of one eager iteration (models/update.py SmallUpdateBlock)
    for sv in saved:   # (corr, patch, cf, f1, mf, inp, h, z, rh, r, q, hn, fm)
        cf, f1, mf, fm = (_join(t.detach()).permute(0, 3, 1, 2) > 0 for t in
                          (sv[2], sv[3], sv[4], sv[12]))
        masks += [cf[:, :96], f1, cf[:, 96:128], mf[:, :80], fm[:, :128]]
    grads = {n: (p.grad.clone() if p.grad is not None else torch.zeros_like(p))
             for n, p in ub.named_parameters()}
    lgrads = [t.grad.clone() if t.grad is not None else None for t in leaves]

    def eager(dtype):
        m = SmallUpdateBlock(args, hidden_dim=96).to(DEV).to(dtype)
        m.load_state_dict(ub.state_dict())
        lv = [t.detach().to(dtype).requires_grad_(True) for t in [net, inp] + corrs]
        hh, tot = lv[0], 0
        queue = list(masks)
        relu = F.relu
        F.relu = lambda x, inplace=False: x * queue.pop(0).to(x.dtype)
        try:
            for i in range(iters):
                hh, _, dl = m(hh, lv[1], lv[2 + i], flows[i].to(dtype))
                tot = tot + (dl * gd[i].to(dtype)).sum()
        finally:
            F.relu = relu
        assert not queue
        tot.backward()
        return hh.detach(), tot.item(), {n: (p.grad if p.grad is not None else torch.zeros_like(p))
                                          for n, p in m.named_parameters()}, [t.grad for t in lv]

    h64, loss64, g64, l64 = eager(torch.float64)
    _, _, g32, l32 = eager(torch.float32)
    hj = _join(hf).permute(0, 3, 1, 2)
    assert (hj[:, 96:] == 0).all()   # the padded state channels stay exact zeros
    assert _rel(hj[:, :96], h64) < 1e-4
    assert abs(loss.item() - loss64) <= 1e-4 * abs(loss64)
    report = [(n, _rel(grads[n], g64[n]), _rel(g32[n], g64[n])) for n in g64 if g64[n].norm() > 0]
    report += [('input%d' % i, _rel(a, b64), _rel(b32, b64))
               for i, (a, b64, b32) in enumerate(zip(lgrads, l64, l32)) if b64 is not None]
    for r in report:
        print('%-32s %.3e %.3e' % r)
    bad = [r for r in report if not r[1] < max(1e-4, 50 * r[2])]
    assert not bad, bad[:4]


def test_fp32_small_model_uses_fused_split_block(ext_ops):
    """An fp32 RAFT-small decodes through the fused split-fp32 small block: a training step's
    flow and update-block gradients match the eager fp32 block (update_impl='torch')."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    from pytorch_raft_amd.ops import update_hip_small as S
    outs = {}
    calls = {'n': 0}
    orig = S._iter_forward

    def counting(pk, *a, **k):
        calls['n'] += int(pk.spl)
        return orig(pk, *a, **k)

    S._iter_forward = counting
    try:
        for impl in ('auto', 'torch'):
            args = argparse.Namespace(small=True, mixed_precision=False, update_impl=impl)
            torch.manual_seed(0)
            m = RAFT(args).to(DEV).train()
            i1, i2, flow, valid = (t.to(DEV) for t in make_pair_batch(2, 128, 160, seed=3))
            preds = m(i1, i2, iters=3)
            loss, _ = sequence_loss(preds, flow, valid, 0.8)
            loss.backward()
            outs[impl] = (preds[-1].detach(), {n: p.grad.detach().clone()
                                               for n, p in m.named_parameters() if p.grad is not None})
    finally:
        S._iter_forward = orig
    assert calls['n'] == 3
    (fa, ga), (fb, gb) = outs['auto'], outs['torch']
    assert _rel(fa, fb) < 1e-3
    for n in gb:
        if n.startswith('update_block'):
            assert _rel(ga[n], gb[n]) < 2e-2, n
