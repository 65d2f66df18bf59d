"""Numerics of every HIP kernel against a plain PyTorch fp32 reference of the same op (GPU only)."""
import math

import pytest
import torch
import torch.nn.functional as F

from pytorch_raft_amd.models.corr import (torch_corr_pyramid, torch_corr_lookup,
                                          torch_onthefly_corr, CorrBlock, AlternateCorrBlock)
from pytorch_raft_amd.ops.upsample import torch_convex_upsample, convex_upsample
from pytorch_raft_amd.ops.loss import torch_sequence_loss, sequence_loss

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _coords(b, h, w, spread=6.0, seed=0):
    g = torch.Generator(device='cpu').manual_seed(seed)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    base = torch.stack([xs, ys])[None].repeat(b, 1, 1, 1)
    c = base + spread * torch.randn(b, 2, h, w, generator=g)
    # a few far out-of-range coordinates exercise the zero padding
    c[:, :, 0, 0] = -50.0
    c[:, :, -1, -1] = 500.0
    return c.to(DEV)


@pytest.mark.parametrize('shape', [(2, 256, 16, 20), (1, 256, 46, 62), (2, 128, 13, 19)])
def test_corr_build_matches_torch(ext_ops, shape):
    b, c, h, w = shape
    f1 = torch.randn(shape, device=DEV)
    f2 = torch.randn(shape, device=DEV)
    levels = 4 if min(h, w) >= 16 else 3
    got = ext_ops.corr_build(f1, f2, levels)
    ref = torch_corr_pyramid(f1, f2, levels)
    for g, r in zip(got, ref):
        r = r.view(b, h * w, *r.shape[-2:])
        assert g.shape == r.shape
        torch.testing.assert_close(g, r, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize('shape', [(2, 256, 16, 20), (2, 256, 46, 62), (1, 128, 13, 19),
                                   (1, 256, 11, 70), (1, 256, 55, 128)])
def test_corr_build_bf16_matches_torch(ext_ops, shape):
    """bf16-MFMA build from NHWC bf16 fmaps vs the fp32 pyramid of the same (bf16-valued) maps:
    identical products, fp32 accumulation in another order.  Odd sizes exercise floor pooling,
    W > 64 the multi-band column tiling."""
    b, c, h, w = shape
    f1 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    f2 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    levels = 4 if min(h, w) >= 8 else 3
    got = ext_ops.corr_build_bf16(f1, f2, levels)
    ref = torch_corr_pyramid(f1.permute(0, 3, 1, 2).float(), f2.permute(0, 3, 1, 2).float(), levels)
    for g, r in zip(got, ref):
        r = r.view(b, h * w, *r.shape[-2:])
        assert g.shape == r.shape
        torch.testing.assert_close(g, r, atol=2e-4, rtol=1e-4)


@pytest.mark.parametrize('shape', [(2, 256, 46, 62), (1, 128, 13, 19)])
def test_corr_build_bf16_pyramid_and_lookup(ext_ops, shape):
    """bf16 pyramid (the fused path's storage): every level is the bf16 rounding of the fp32
    build, and the NHWC window lookup reading it matches the lookup of the fp32 pyramid to bf16
    resolution."""
    b, c, h, w = shape
    f1 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    f2 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    levels = 4 if min(h, w) >= 8 else 3
    p32 = ext_ops.corr_build_bf16(f1, f2, levels, False)
    p16 = ext_ops.corr_build_bf16(f1, f2, levels, True)
    for a, q in zip(p16, p32):
        assert a.dtype == torch.bfloat16 and a.shape == q.shape
        torch.testing.assert_close(a.float(), q.to(torch.bfloat16).float(), atol=0, rtol=0)
    coords = _coords(b, h, w, spread=6.0)
    o32 = torch.zeros(b, h, w, 384, device=DEV, dtype=torch.bfloat16)
    o16 = torch.zeros_like(o32)
    ext_ops.corr_lookup_nhwc_(p32, coords, 4 if levels == 4 else 3, o32)
    ext_ops.corr_lookup_nhwc_(p16, coords, 4 if levels == 4 else 3, o16)
    assert _rel(o16.float(), o32.float()) < 1e-2


@pytest.mark.parametrize('shape,radius,spread', [((2, 256, 46, 62), 4, 6.0), ((1, 128, 13, 19), 3, 6.0),
                                                  ((2, 64, 23, 30), 4, 40.0), ((3, 32, 11, 17), 4, 2.0)])
def test_lookup_rows_bf16_vs_oracle(ext_ops, shape, radius, spread):
    """Row-vector NHWC lookup on the bf16 pyramid (aligned 16-B row pieces, plane-edge masking,
    dword reads for the pieces at a workgroup range's end) vs the grid_sample oracle on the same
    bf16 values: equal up to the bf16 rounding of the output; the padded channels stay zero."""
    b, c, h, w = shape
    f1 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    f2 = torch.randn(b, h, w, c, device=DEV).to(torch.bfloat16)
    # the oracle's align_corners normalisation divides by (size - 1): every level >= 2 x 2
    levels = 4 if min(h, w) >= 16 else 3
    pyr = ext_ops.corr_build_bf16(f1, f2, levels, True)
    coords = _coords(b, h, w, spread=spread, seed=3)
    out = torch.full((b, h, w, 384), 7.0, device=DEV, dtype=torch.bfloat16)
    ext_ops.corr_lookup_nhwc_(pyr, coords, radius, out)
    ref = torch_corr_lookup([p.float().reshape(b * h * w, 1, *p.shape[-2:]) for p in pyr],
                            coords, radius)
    ctot = levels * (2 * radius + 1) ** 2
    got = out[..., :ctot].permute(0, 3, 1, 2).float()
    err = (got - ref).abs()
    # bf16 output rounding (<= 2^-8 relative) + the oracle's own coordinate normalisation
    # (grid_sample maps x -> [-1, 1] -> x: ~1e-6 px, i.e. ~1e-5 absolute on the taps)
    bound = ref.abs() * 2.0 ** -8 + 1e-4 * ref.abs().max()
    assert (err <= bound).all(), ((err - bound).max().item(), err.max().item())
    assert (out[..., ctot:] == 0).all()


def test_corrblock_bf16_fmaps_fwd_bwd(ext_ops):
    """Mixed-precision CorrBlock: bf16 channels_last fmaps in (as the encoders produce them),
    fp32 lookups out, bf16 fmap gradients back (bf16 dcorr: ~1e-2 relative)."""
    b, c, h, w = 2, 256, 23, 30
    g = torch.Generator(device='cpu').manual_seed(1)
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV, torch.bfloat16)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV, torch.bfloat16)
    f1 = f1.contiguous(memory_format=torch.channels_last).requires_grad_()
    f2 = f2.contiguous(memory_format=torch.channels_last).requires_grad_()
    coords = _coords(b, h, w, spread=3.0)
    r1 = f1.detach().float().requires_grad_()
    r2 = f2.detach().float().requires_grad_()
    ref = torch_corr_lookup(torch_corr_pyramid(r1, r2, 4), coords, 4)
    blk = CorrBlock(f1, f2, num_levels=4, radius=4, impl='hip', precision='bf16')
    out = blk.lookup_nhwc(coords, 384)[..., :324].permute(0, 3, 1, 2).float()
    assert _rel(out, ref) < 5e-3
    gout = torch.randn_like(ref)
    (ref * gout).sum().backward()
    (out * gout).sum().backward()
    assert f1.grad.dtype == torch.bfloat16 and f1.grad.shape == f1.shape
    assert _rel(f1.grad.float(), r1.grad) < 2e-2
    assert _rel(f2.grad.float(), r2.grad) < 2e-2


@pytest.mark.parametrize('radius,c', [(4, 256), (3, 128)])
@pytest.mark.parametrize('hw', [(16, 20), (13, 19)])
def test_lookup_fwd_bwd_matches_grid_sample(ext_ops, radius, c, hw):
    h, w = hw
    b = 2
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    coords = _coords(b, h, w)
    levels = 3 if min(h, w) < 16 else 4

    # torch oracle through grid_sample autograd
    pyr = torch_corr_pyramid(f1, f2, levels)
    ref = torch_corr_lookup(pyr, coords, radius)
    gout = torch.randn_like(ref)
    (ref * gout).sum().backward()
    g1_ref, g2_ref = f1.grad.clone(), f2.grad.clone()
    f1.grad = f2.grad = None

    blk = CorrBlock(f1, f2, num_levels=levels, radius=radius, impl='hip')
    assert blk.hip
    out = blk(coords)
    torch.testing.assert_close(out, ref, atol=2e-4, rtol=1e-4)
    # two lookups share the volume -> gradients accumulate in the persistent buffer
    out2 = blk(coords + 0.37)
    ref2 = torch_corr_lookup(pyr, coords + 0.37, radius)
    torch.testing.assert_close(out2, ref2, atol=2e-4, rtol=1e-4)
    (out * gout).sum().backward()
    torch.testing.assert_close(f1.grad, g1_ref, atol=2e-3, rtol=1e-3)
    torch.testing.assert_close(f2.grad, g2_ref, atol=2e-3, rtol=1e-3)


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-12)).item()


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
@pytest.mark.parametrize('radius,c', [(4, 256), (3, 128)])
@pytest.mark.parametrize('hw,spread', [((16, 24), 6.0), ((13, 19), 2.0), ((46, 62), 3.0)])
def test_onthefly_matches_allpairs(ext_ops, radius, c, hw, spread, precision):
    """MFMA on-the-fly lookup (split-bf16 or bf16 operands, fp32 accumulation) vs the fp32
    grid_sample oracle.  fp32: the forward AND the backward (three bf16-product passes: dS_hi F_hi,
    dS_lo F_hi, dS_hi F_lo) are fp32-accurate to 1e-4 relative."""
    h, w = hw
    b = 2
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    coords = _coords(b, h, w, spread=spread, seed=3)
    levels = 4 if min(h, w) >= 16 else 3
    pyr = torch_corr_pyramid(f1, f2, levels)
    refs = [torch_corr_lookup(pyr, coords, radius), torch_corr_lookup(pyr, coords + 1.3, radius)]
    gouts = [torch.randn_like(r) for r in refs]
    sum((r * g).sum() for r, g in zip(refs, gouts)).backward()
    g1_ref, g2_ref = f1.grad.clone(), f2.grad.clone()
    f1.grad = f2.grad = None

    blk = AlternateCorrBlock(f1, f2, num_levels=levels, radius=radius, impl='hip',
                             precision=precision)
    assert blk.hip
    outs = [blk(coords), blk(coords + 1.3)]
    for o, r in zip(outs, refs):
        if precision == 'fp32':
            torch.testing.assert_close(o, r.detach(), atol=1e-3, rtol=1e-3)
            assert _rel(o, r.detach()) < 1e-4
        else:
            torch.testing.assert_close(o, r.detach(), atol=3e-2, rtol=2e-2)
            assert _rel(o, r.detach()) < 5e-3
    sum((o * g).sum() for o, g in zip(outs, gouts)).backward()
    tol = 1e-4 if precision == 'fp32' else 1e-2
    assert _rel(f1.grad, g1_ref) < tol
    assert _rel(f2.grad, g2_ref) < tol


@pytest.mark.parametrize('drift', [False, True])
@pytest.mark.parametrize('hw', [(46, 62), (13, 19)])
def test_onthefly_nhwc_bf16(ext_ops, hw, drift):
    """Fused-path lookups (bf16 NHWC) over 3 iterations; backward = window-compact gradients
    folded by ONE corr_otf_window_bwd_ launch.  Also checks it is deterministic in dF1.
    drift=True moves each pixel's window by a pixel or two per iteration (as RAFT's refinement
    does), so every tile takes the union-grid path of the backward; drift=False scatters the
    windows independently, so level 0 mostly falls back to the per-iteration sum.  dF1 is always
    deterministic; dF2 is whenever the tiles' union boxes fit their slab rows (drift=True)."""
    h, w = hw
    b, c, radius = 2, 256, 4
    levels = 4 if min(h, w) >= 16 else 3
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    if drift:
        c0 = _coords(b, h, w, spread=3.0, seed=5)
        g = torch.Generator(device='cpu').manual_seed(9)
        coords = [c0 + 0.6 * s * torch.randn(c0.shape, generator=g).clamp(-1.5, 1.5).to(DEV)
                  for s in range(3)]
    else:
        coords = [_coords(b, h, w, spread=2.0 + s, seed=5 + s) for s in range(3)]
    nc = levels * 81
    pyr = torch_corr_pyramid(f1, f2, levels)
    gouts = [torch.randn(b, h, w, 384, device=DEV) for _ in coords]
    refs = [torch_corr_lookup(pyr, co, radius).permute(0, 2, 3, 1) for co in coords]
    sum((r * g[..., :nc]).sum() for r, g in zip(refs, gouts)).backward()
    g1_ref, g2_ref = f1.grad.clone(), f2.grad.clone()
    runs = []
    for _ in range(2):
        f1.grad = f2.grad = None
        blk = AlternateCorrBlock(f1, f2, num_levels=levels, radius=radius, impl='hip',
                                 precision='bf16')
        outs = [blk.lookup_nhwc(co, 384) for co in coords]
        for o, r in zip(outs, refs):
            assert o.shape == (b, h, w, 384) and o.dtype == torch.bfloat16
            assert torch.all(o[..., nc:] == 0)
            assert _rel(o[..., :nc].float(), r.detach()) < 8e-3
        sum((o.float() * g).sum() for o, g in zip(outs, gouts)).backward()
        assert _rel(f1.grad, g1_ref) < 1e-2
        assert _rel(f2.grad, g2_ref) < 1e-2
        runs.append((f1.grad.clone(), f2.grad.clone()))
    assert torch.equal(runs[0][0], runs[1][0])
    if drift:
        # dF2 through per-tile slab rows + a fixed-order reduce (no float atomics): bitwise
        # reproducible while every tile's union box fits its slab (RAFT-like drifting windows)
        assert torch.equal(runs[0][1], runs[1][1])


def test_onthefly_slab_budget_falls_back_to_atomics(ext_ops, monkeypatch):
    """The deterministic dF2 scratch (per-tile slab rows, ~170 KB per query pixel) is bounded by
    RAFT_OTF_SLAB_GB: past it the call takes the float-atomic dF2 path, with the same gradients
    up to summation order and no slab allocation (peak memory stays at the fmaps' scale)."""
    b, c, h, w, radius, levels = 2, 256, 46, 62, 4, 4
    g = torch.Generator(device='cpu').manual_seed(3)
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    c0 = _coords(b, h, w, spread=3.0, seed=5)
    coords = [c0 + 0.5 * torch.randn(c0.shape, generator=g).clamp(-1, 1).to(DEV) for _ in range(3)]
    gouts = [torch.randn(b, h, w, 384, device=DEV) for _ in coords]

    def run():
        f1.grad = f2.grad = None
        blk = AlternateCorrBlock(f1, f2, num_levels=levels, radius=radius, impl='hip',
                                 precision='bf16')
        outs = [blk.lookup_nhwc(co, 384) for co in coords]
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        sum((o.float() * gg).sum() for o, gg in zip(outs, gouts)).backward()
        torch.cuda.synchronize()
        return f1.grad.clone(), f2.grad.clone(), torch.cuda.max_memory_allocated() - base

    g1_s, g2_s, peak_slab = run()
    monkeypatch.setenv('RAFT_OTF_SLAB_GB', '0.001')
    g1_a, g2_a, peak_atomic = run()
    assert _rel(g1_a, g1_s) < 1e-5 and _rel(g2_a, g2_s) < 1e-4
    caps, hh, ww = 0, h, w
    for lvl in range(levels):
        caps += min(hh * ww, 1024 if lvl == 0 else 576)
        hh, ww = hh // 2, ww // 2
    slab_bytes = b * ((h + 7) // 8) * ((w + 7) // 8) * caps * c * 4
    assert peak_atomic < peak_slab - 0.5 * slab_bytes, (peak_atomic, peak_slab, slab_bytes)


@pytest.mark.parametrize('mask_dtype', [torch.float32, torch.bfloat16])
@pytest.mark.parametrize('hw', [(8, 9), (46, 62), (5, 70)])
def test_convex_upsample_fwd_bwd(ext_ops, mask_dtype, hw):
    h, w = hw
    b = 2
    flow = torch.randn(b, 2, h, w, device=DEV, requires_grad=True)
    mask = (3 * torch.randn(b, 576, h, w, device=DEV)).to(mask_dtype).requires_grad_(True)
    ref = torch_convex_upsample(flow, mask.float())
    g = torch.randn_like(ref)
    (ref * g).sum().backward()
    gf_ref, gm_ref = flow.grad.clone(), mask.grad.clone().float()
    flow.grad = mask.grad = None
    out = convex_upsample(flow, mask, impl='hip')
    torch.testing.assert_close(out.float(), ref, atol=1e-4, rtol=1e-4)
    (out.float() * g).sum().backward()
    torch.testing.assert_close(flow.grad, gf_ref, atol=1e-3, rtol=1e-4)
    tol = 1e-4 if mask_dtype == torch.float32 else 2e-2
    torch.testing.assert_close(mask.grad.float(), gm_ref, atol=tol, rtol=tol)


def test_sequence_loss_fwd_bwd(ext_ops):
    b, h, w, n = 2, 40, 56, 5
    gt = 30 * torch.randn(b, 2, h, w, device=DEV)
    gt[0, :, :4] = 500.0  # beyond MAX_FLOW -> masked
    valid = (torch.rand(b, h, w, device=DEV) > 0.2).float()
    preds = [(gt + torch.randn_like(gt) * (i + 1)).requires_grad_(True) for i in range(n)]
    lr, mr = torch_sequence_loss(preds, gt, valid, 0.8)
    lr.backward()
    gref = [p.grad.clone() for p in preds]
    for p in preds:
        p.grad = None
    lh, mh = sequence_loss(preds, gt, valid, 0.8, impl='hip')
    torch.testing.assert_close(lh, lr, atol=1e-5, rtol=1e-5)
    for k in ('epe', '1px', '3px', '5px'):
        torch.testing.assert_close(mh[k], mr[k], atol=1e-5, rtol=1e-5)
    lh.backward()
    for p, g in zip(preds, gref):
        torch.testing.assert_close(p.grad, g, atol=1e-9, rtol=1e-5)


def test_lookup_deterministic(ext_ops):
    b, c, h, w = 2, 256, 16, 16
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    coords = _coords(b, h, w)
    grads = []
    for _ in range(2):
        blk = CorrBlock(f1, f2, radius=4, impl='hip')
        out = blk(coords)
        out.square().sum().backward()
        grads.append((f1.grad.clone(), f2.grad.clone()))
        f1.grad = f2.grad = None
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


@pytest.mark.parametrize('precision', ['fp32', 'bf16'])
@pytest.mark.parametrize('hw', [(16, 20), (13, 19), (46, 62)])
def test_lookup_nhwc_window_backward(ext_ops, hw, precision):
    """bf16 NHWC lookup (fused update-block input) + compact window backward vs grid_sample."""
    h, w = hw
    b, c, radius = 2, 256, 4
    f1 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    f2 = torch.randn(b, c, h, w, device=DEV, requires_grad=True)
    levels = 3 if min(h, w) < 16 else 4
    coords = [_coords(b, h, w, seed=s) for s in range(3)]
    pyr = torch_corr_pyramid(f1, f2, levels)
    gouts = [torch.randn(b, h, w, 384, device=DEV).to(torch.bfloat16) for _ in coords]
    loss = 0
    for co, go in zip(coords, gouts):
        ref = torch_corr_lookup(pyr, co, radius)  # (b, L*81, h, w)
        loss = loss + (ref.permute(0, 2, 3, 1) * go[..., :ref.shape[1]].float()).sum()
    loss.backward()
    g1_ref, g2_ref = f1.grad.clone(), f2.grad.clone()
    f1.grad = f2.grad = None

    blk = CorrBlock(f1, f2, num_levels=levels, radius=radius, impl='hip', precision=precision)
    loss = 0
    for co, go in zip(coords, gouts):
        out = blk.lookup_nhwc(co, 384)
        assert out.shape == (b, h, w, 384) and out.dtype == torch.bfloat16
        nc = levels * 81
        ref = torch_corr_lookup(pyr, co, radius).permute(0, 2, 3, 1)
        torch.testing.assert_close(out[..., :nc].float(), ref.detach(), atol=3e-2, rtol=1e-2)
        assert torch.all(out[..., nc:] == 0)
        loss = loss + (out.float() * go.float()).sum()
    loss.backward()
    # bf16: dcorr rounded to bf16 before the (fp32-accumulating) backward GEMMs
    tol = 3e-3 if precision == 'fp32' else 1e-2 * max(g1_ref.abs().max().item(), 1.0)
    torch.testing.assert_close(f1.grad, g1_ref, atol=tol, rtol=3e-3 if precision == 'fp32' else 2e-2)
    torch.testing.assert_close(f2.grad, g2_ref, atol=tol, rtol=3e-3 if precision == 'fp32' else 2e-2)


@pytest.mark.parametrize('mask_dtype', [torch.bfloat16, torch.float32, 'channels_last'])
@pytest.mark.parametrize('hw', [(8, 9), (46, 62)])
def test_convex_upsample_nhwc(ext_ops, hw, mask_dtype):
    """NHWC mask: bf16 (fused bf16 block), fp32 (B,H,W,576), and an fp32 channels_last
    (B,576,H,W) tensor -- the fp32 model's mask head output, routed to the NHWC kernel."""
    h, w = hw
    b = 2
    flow = torch.randn(b, 2, h, w, device=DEV, requires_grad=True)
    m = 3 * torch.randn(b, h, w, 576, device=DEV)
    if mask_dtype == 'channels_last':
        mask = m.permute(0, 3, 1, 2).requires_grad_(True)   # (B,576,H,W), channels_last strides
        nhwc, ref_mask = False, mask
    else:
        mask = m.to(mask_dtype).requires_grad_(True)
        nhwc, ref_mask = True, mask.float().permute(0, 3, 1, 2)
    ref = torch_convex_upsample(flow, ref_mask)
    g = torch.randn_like(ref)
    (ref * g).sum().backward()
    gf_ref, gm_ref = flow.grad.clone(), mask.grad.clone().float()
    flow.grad = mask.grad = None
    out = convex_upsample(flow, mask, impl='hip', nhwc=nhwc)
    torch.testing.assert_close(out.float(), ref, atol=1e-4, rtol=1e-4)
    (out.float() * g).sum().backward()
    torch.testing.assert_close(flow.grad, gf_ref, atol=1e-3, rtol=1e-4)
    tol = 2e-2 if mask_dtype == torch.bfloat16 else 1e-4
    torch.testing.assert_close(mask.grad.float(), gm_ref, atol=tol, rtol=tol)


@pytest.mark.parametrize('radius,levels,hw', [(4, 4, (46, 62)), (3, 4, (24, 31)), (4, 3, (13, 19))])
def test_tap_reduce_matches_window_path(ext_ops, radius, levels, hw):
    """One-pass fold from the bf16 tap gradients == per-iteration compact windows + fold."""
    h, w = hw
    b = 2
    D = 2 * radius + 1
    coords = [_coords(b, h, w, seed=s) for s in range(7)]      # > one 6-iteration chunk
    douts = [torch.randn(b, h, w, 384, device=DEV).to(torch.bfloat16) for _ in coords]
    s = 1.0 / 16
    wgs = [ext_ops.corr_window_grad(c, g, levels, radius) for c, g in zip(coords, douts)]
    ref = ext_ops.corr_window_reduce(coords, wgs, h, w, levels, radius, s, False)
    got = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, False)
    assert levels * D * D <= 384
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)
    got16 = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, True)
    torch.testing.assert_close(got16.float(), ref, atol=1e-2, rtol=1e-2)
    # fixed fold order: bitwise reproducible
    assert torch.equal(ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, False), got)


@pytest.mark.parametrize('radius,levels,hw,drift', [(4, 4, (46, 62), 0.7), (3, 4, (24, 32), 0.7),
                                                     (4, 3, (14, 20), 0.7), (4, 4, (46, 62), 3.0)])
def test_tap_reduce_box_path(ext_ops, radius, levels, hw, drift):
    """Union-box fold (the default for bf16 dC at even W): windows that drift a little per
    iteration (the training case) fit the 24 x 24 boxes; drift 3.0 pushes some pixels past the cap
    onto the listed workgroup-per-pixel fold.  Both == the window path up to the bf16 output
    rounding, and bitwise reproducible."""
    h, w = hw
    b = 2
    g = torch.Generator(device='cpu').manual_seed(4)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    c = torch.stack([xs, ys])[None].repeat(b, 1, 1, 1) + 4 * torch.randn(b, 2, h, w, generator=g)
    coords = []
    for _ in range(12):
        c = c + drift * torch.randn(b, 2, h, w, generator=g)
        coords.append(c.clone().to(DEV))
    coords[3][:, :, 0, 0] = -50.0      # one iteration's window leaves the map
    douts = [torch.randn(b, h, w, 384, device=DEV).to(torch.bfloat16) for _ in coords]
    s = 1.0 / 16
    wgs = [ext_ops.corr_window_grad(cc, gg, levels, radius) for cc, gg in zip(coords, douts)]
    ref = ext_ops.corr_window_reduce(coords, wgs, h, w, levels, radius, s, False)
    got = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, True)
    err = (got.float() - ref).abs()
    assert (err <= ref.abs() * 2.0 ** -8 + 1e-6).all(), err.max().item()
    assert torch.equal(ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, True), got)


@pytest.mark.parametrize('radius,levels,hw,bf16', [(4, 4, (46, 62), True), (4, 4, (23, 31), True),
                                                   (3, 4, (24, 31), False), (4, 3, (13, 19), True)])
def test_tap_reduce_padded_pitch(ext_ops, radius, levels, hw, bf16):
    """pitch_mult: every fold variant (box at even W, workgroup / listed at odd W) writes rows of
    round_up(N, 64) with the same first N columns and zero padding."""
    h, w = hw
    b, n = 2, hw[0] * hw[1]
    coords = [_coords(b, h, w, seed=s) for s in range(5)]
    douts = [torch.randn(b, h, w, 384, device=DEV).to(torch.bfloat16) for _ in coords]
    s = 1.0 / 16
    ref = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, bf16)
    got = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, bf16, 64)
    ld = (n + 63) // 64 * 64
    assert got.shape == (b, n, ld)
    assert torch.equal(got[..., :n], ref)
    assert (got[..., n:] == 0).all()


@pytest.mark.parametrize('b,hw,c', [(2, (46, 62), 256), (3, (7, 9), 128), (1, (23, 31), 256)])
def test_corr_bwd_fmaps_matches_fp32(ext_ops, b, hw, c):
    """corr_bwd.hip: dF1 = dC F2 and dF2 = dC^T F1 (the all-pairs correlation's feature-map
    gradients, `core/corr.py:52-60`) on bf16 operands vs fp32 matmuls of the same bf16 values,
    with a padded dC pitch (odd N: padded K and M tails)."""
    h, w = hw
    n = h * w
    ld = (n + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(11)
    dc = torch.zeros(b, n, ld, device=DEV, dtype=torch.bfloat16)
    dc[..., :n] = torch.randn(b, n, n, device=DEV, generator=g).to(torch.bfloat16)
    f1 = torch.randn(b, h, w, c, device=DEV, generator=g).to(torch.bfloat16)
    f2 = torch.randn(b, h, w, c, device=DEV, generator=g).to(torch.bfloat16)
    g1, g2 = ext_ops.corr_bwd_fmaps(dc, f1, f2)
    d = dc[..., :n].float()
    r1 = torch.bmm(d, f2.float().view(b, n, c)).view(b, h, w, c)
    r2 = torch.bmm(d.transpose(1, 2), f1.float().view(b, n, c)).view(b, h, w, c)
    for got, ref in ((g1, r1), (g2, r2)):
        assert got.shape == ref.shape and got.dtype == torch.bfloat16
        # fp32 accumulation, one bf16 rounding of the result
        err = (got.float() - ref).abs().max().item()
        assert err <= 2.0 ** -7 * ref.abs().max().item(), err
    # deterministic: no atomics
    g1b, g2b = ext_ops.corr_bwd_fmaps(dc, f1, f2)
    assert torch.equal(g1, g1b) and torch.equal(g2, g2b)


@pytest.mark.parametrize('convention', ['reference', 'exact'])
@pytest.mark.parametrize('shape', [(1, 3, 37, 53), (2, 3, 64, 96)])
def test_warp_sampler_matches_grid_sample(ext_ops, convention, shape):
    """sampler.hip (demo warping, reference `demo_warp.py:27-56`) vs F.grid_sample: forward and
    both gradients, with flows that push samples off the image (zero padding)."""
    from pytorch_raft_amd.ops.sampler import warp_image, torch_warp
    b, c, h, w = shape
    g = torch.Generator(device='cpu').manual_seed(11)
    x = (torch.rand(shape, generator=g) * 255).to(DEV).requires_grad_(True)
    flo = (torch.randn(b, 2, h, w, generator=g) * 6).to(DEV)
    flo[:, 0, :, :4] -= 20.0      # off the left edge
    flo = flo.requires_grad_(True)
    out = warp_image(x, flo, convention=convention, impl='hip')
    x2 = x.detach().clone().requires_grad_(True)
    f2 = flo.detach().clone().requires_grad_(True)
    ref = torch_warp(x2, f2, convention)
    # fp32 coordinate normalisation is done in a different order than grid_sample's unnormalise:
    # ~1e-5 px position rounding x image gradients of up to ~255 / px
    torch.testing.assert_close(out, ref, atol=1e-2, rtol=1e-4)
    gout = torch.randn_like(ref)
    (out * gout).sum().backward()
    (ref * gout).sum().backward()
    torch.testing.assert_close(x.grad, x2.grad, atol=5e-3, rtol=1e-3)
    torch.testing.assert_close(flo.grad, f2.grad, atol=5e-2, rtol=1e-3)


@pytest.mark.parametrize('b,hw,c', [(2, (46, 62), 256), (3, (7, 9), 128), (1, (23, 31), 256)])
def test_corr_bwd_fmaps_split_matches_fp64(ext_ops, b, hw, c):
    """The fp32 correlation's feature-map gradients (fp16 / fp32 schedules, `core/corr.py:52-60`
    in fp32): dC and the fp32 fmaps as split-bf16 pairs, three MFMA passes per GEMM, fp32 output,
    vs fp64 matmuls -- fp32-accurate (~2^-16 relative to the largest entry)."""
    h, w = hw
    n = h * w
    ld = (n + 63) // 64 * 64
    g = torch.Generator(device=DEV).manual_seed(12)
    d = torch.randn(b, n, n, device=DEV, generator=g)
    dc2 = torch.zeros(2, b, n, ld, device=DEV, dtype=torch.bfloat16)
    hi = d.to(torch.bfloat16)
    dc2[0, ..., :n] = hi
    dc2[1, ..., :n] = (d - hi.float()).to(torch.bfloat16)
    f1 = torch.randn(b, c, h, w, device=DEV, generator=g)
    f2 = torch.randn(b, c, h, w, device=DEV, generator=g)
    g1, g2 = ext_ops.corr_bwd_fmaps_split(dc2, f1, f2)
    dd = d.double()
    r1 = torch.bmm(dd, f2.double().view(b, c, n).transpose(1, 2)).view(b, h, w, c)
    r2 = torch.bmm(dd.transpose(1, 2), f1.double().view(b, c, n).transpose(1, 2)).view(b, h, w, c)
    for got, ref in ((g1, r1), (g2, r2)):
        assert got.shape == ref.shape and got.dtype == torch.float32
        err = (got.double() - ref).abs().max().item()
        assert err <= 1e-4 * ref.abs().max().item(), err
    g1b, g2b = ext_ops.corr_bwd_fmaps_split(dc2, f1, f2)
    assert torch.equal(g1, g1b) and torch.equal(g2, g2b)


@pytest.mark.parametrize('hw', [(12, 16), (23, 30)])
def test_tap_reduce_split_planes(ext_ops, hw):
    """corr_tap_reduce(split_out=True): the fp32 dC of the fold as bf16 planes hi + lo (padded
    pitch, zero columns) -- hi + lo reproduces the fp32 fold to ~2^-16."""
    h, w = hw
    b, levels, radius = 2, 4, 4
    n = h * w
    g = torch.Generator(device=DEV).manual_seed(5)
    coords = [(torch.rand(b, 2, h, w, device=DEV, generator=g) * torch.tensor([w, h], device=DEV).view(1, 2, 1, 1)).contiguous()
              for _ in range(3)]
    douts = [torch.randn(b, h, w, 328, device=DEV, generator=g).to(torch.bfloat16) for _ in range(3)]
    s = 1 / 16
    ref = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, False, 64)
    got = ext_ops.corr_tap_reduce(coords, douts, h, w, levels, radius, s, False, 64, False, True)
    assert got.shape == (2, b, n, ref.shape[-1]) and got.dtype == torch.bfloat16
    v = got[0].float() + got[1].float()
    assert (v - ref).abs().max().item() <= 2.0 ** -15 * ref.abs().max().item()
    assert (got[..., n:] == 0).all()
