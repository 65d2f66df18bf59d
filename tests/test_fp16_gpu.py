"""fp16 operands on the MFMA kernels (fp16 autocast, the reference's `--mixed_precision`,
`core/raft.py:99,110,127`): every kernel of the fused update block's fp16 path against a plain
PyTorch fp32 op on the same fp16-rounded operands."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import conv as C

pytestmark = pytest.mark.gpu
DEV = 'cuda'
H16 = torch.float16

# LDS-DMA and halo configs of conv_igemm.hip's kCfgs (fp16 runs only those kernel families)
FP16_CFGS = (10, 17, 16, 26, 30, 33)


def _h(x):
    return x.to(H16).float()


@pytest.mark.parametrize('cfg', (-1,) + FP16_CFGS)
@pytest.mark.parametrize('cin,cout,k,epi', [
    (256, 192, (3, 3), C.EPI_RELU_BF16),
    (256, 256, (1, 5), C.EPI_BF16),
    (128, 128, (5, 1), C.EPI_F32),
])
def test_conv_fwd_fp16(ext_ops, cfg, cin, cout, k, epi):
    torch.manual_seed(0)
    B, H, W = 2, 13, 21
    x = torch.randn(B, cin, H, W, device=DEV)
    w = torch.randn(cout, cin, *k, device=DEV) / (cin * k[0] * k[1]) ** 0.5
    b = torch.randn(cout, device=DEV)
    pad = (k[0] // 2, k[1] // 2)
    ref = F.conv2d(_h(x), _h(w), b, padding=pad)
    if epi == C.EPI_RELU_BF16:
        ref = ref.relu()
    f32 = epi == C.EPI_F32
    out = torch.zeros(B, H, W, cout, device=DEV, dtype=torch.float32 if f32 else H16)
    ext_ops.conv_set_forced_cfg(cfg)
    try:
        C.conv_fwd([(C.nhwc(x, H16), 0, cin)], C.pack_weight(w, [cin], [cin], dtype=H16), b, k, pad,
                   cout, epi, [out], [0])
    finally:
        ext_ops.conv_set_forced_cfg(-1)
    got = C.nchw(out).float()
    # fp16 products, fp32 accumulation; one fp16 rounding of a 16-bit output (2^-11)
    tol = 2e-3 if f32 else 4e-3
    torch.testing.assert_close(got, ref, atol=tol * max(1.0, ref.abs().max().item()), rtol=tol)


def test_conv_gru_epilogues_fp16(ext_ops):
    """z | r gates (sigmoid, r*h) and the q gate + state update (tanh, h + z (q - h)) on fp16."""
    torch.manual_seed(2)
    B, H, W, hd = 2, 11, 17, 128
    h = torch.randn(B, hd, H, W, device=DEV).tanh()
    x = torch.randn(B, 128, H, W, device=DEV)
    wzr = torch.randn(2 * hd, hd + 128, 1, 5, device=DEV) / 40
    wq = torch.randn(hd, hd + 128, 1, 5, device=DEV) / 40
    bzr = torch.randn(2 * hd, device=DEV) * 0.1
    bq = torch.randn(hd, device=DEV) * 0.1
    hn, xn = C.nhwc(h, H16), C.nhwc(x, H16)
    z, rh, r = (torch.empty(B, H, W, hd, device=DEV, dtype=H16) for _ in range(3))
    C.conv_fwd([(hn, 0, hd), (xn, 0, 128)], C.pack_weight(wzr, [hd, 128], [hd, 128], dtype=H16), bzr,
               (1, 5), (0, 2), 2 * hd, C.EPI_GRU_ZR, [z, rh, r], [0, 0, 0], aux=[hn], aux_offs=[0],
               split=hd)
    pre = F.conv2d(torch.cat([_h(h), _h(x)], 1), _h(wzr), bzr, padding=(0, 2))
    z_ref, r_ref = torch.sigmoid(pre[:, :hd]), torch.sigmoid(pre[:, hd:])
    torch.testing.assert_close(C.nchw(z).float(), z_ref, atol=3e-3, rtol=3e-3)
    torch.testing.assert_close(C.nchw(r).float(), r_ref, atol=3e-3, rtol=3e-3)
    torch.testing.assert_close(C.nchw(rh).float(), r_ref * _h(h), atol=3e-3, rtol=3e-3)
    h2, q = torch.empty_like(z), torch.empty_like(z)
    C.conv_fwd([(rh, 0, hd), (xn, 0, 128)], C.pack_weight(wq, [hd, 128], [hd, 128], dtype=H16), bq,
               (1, 5), (0, 2), hd, C.EPI_GRU_Q, [h2, q], [0, 0], aux=[hn, z], aux_offs=[0, 0])
    q_ref = torch.tanh(F.conv2d(torch.cat([C.nchw(rh).float(), _h(x)], 1), _h(wq), bq, padding=(0, 2)))
    zf = C.nchw(z).float()
    torch.testing.assert_close(C.nchw(q).float(), q_ref, atol=3e-3, rtol=3e-3)
    torch.testing.assert_close(C.nchw(h2).float(), _h(h) + zf * (q_ref - _h(h)), atol=4e-3, rtol=3e-3)


def test_conv_dgrad_and_wgrad_fp16(ext_ops):
    """Input gradient (flipped-weight conv, fp32 output + ReLU-gated fp16 output) and the
    tap-fused weight / bias gradient with fp16 operands."""
    torch.manual_seed(3)
    B, H, W, cin, cout, k = 2, 13, 19, 128, 256, (3, 3)
    x = torch.randn(B, cin, H, W, device=DEV)
    w = torch.randn(cout, cin, *k, device=DEV) / 30
    g = torch.randn(B, cout, H, W, device=DEV)
    xr = _h(x).requires_grad_(True)
    wr = _h(w).requires_grad_(True)
    br = torch.zeros(cout, device=DEV, requires_grad=True)
    F.conv2d(xr, wr, br, padding=1).backward(_h(g))
    wd = C.pack_weight(w.flip(2, 3).transpose(0, 1).contiguous(), [cout], [cout], dtype=H16)
    gn = C.nhwc(g, H16)
    dx = torch.empty(B, H, W, cin, device=DEV)
    ext_ops.conv_dgrad_([gn], [0], [cout], wd, 3, 3, 1, 1, 0, 1.0, [dx], [0], [cin], [cin], [0],
                        [dx], [0], [], [])
    scale = xr.grad.abs().max().item()
    torch.testing.assert_close(C.nchw(dx), xr.grad, atol=2e-3 * scale, rtol=2e-3)
    # ReLU-gated fp16 output (gradient w.r.t. the pre-activation of a ReLU whose output is y)
    y = C.nhwc(torch.randn(B, cin, H, W, device=DEV).relu(), H16)
    dxg = torch.empty(B, H, W, cin, device=DEV, dtype=H16)
    ext_ops.conv_dgrad_([gn], [0], [cout], wd, 3, 3, 1, 1, 0, 1.0, [dxg], [0], [cin], [cin], [0],
                        [y], [0], [], [])
    want = C.nchw(dx) * (C.nchw(y).float() > 0)
    torch.testing.assert_close(C.nchw(dxg).float(), want, atol=4e-3 * scale, rtol=4e-3)
    # weight / bias gradient, two items (iterations) summed
    dw = torch.zeros(cout, 9 * cin, device=DEV)
    db = torch.zeros(cout, device=DEV)
    C.conv_wgrad_taps([(gn, [C.nhwc(x, H16)]), (gn, [C.nhwc(x, H16)])], 0, [0], [cin], k, (1, 1),
                      cout, dw, db)
    got = C.unpack_weight_grad(dw, cout, [cin], [cin], k)
    s = wr.grad.abs().max().item()
    torch.testing.assert_close(got, 2 * wr.grad, atol=4e-3 * s, rtol=2e-3)
    torch.testing.assert_close(db, 2 * br.grad, atol=2e-3 * br.grad.abs().max().item(), rtol=2e-3)


def test_flow_head2_fp16(ext_ops):
    """flow_head.conv2 VALU kernels on fp16 (v_dot2_f32_f16): forward, ReLU-gated input gradient
    and the multi-item weight gradient."""
    B, H, W = 2, 11, 13
    g = torch.Generator(device=DEV).manual_seed(3)
    w = torch.randn(2, 256, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(2, device=DEV, generator=g)
    fm = torch.relu(torch.randn(B, H, W, 256, device=DEV, generator=g)).to(H16)
    x = fm.float().permute(0, 3, 1, 2)
    wb = w.to(H16)
    out = torch.empty(B, 2, H, W, device=DEV)
    ext_ops.fh2_fwd_(fm, wb.permute(2, 3, 0, 1).contiguous(), b, out)
    torch.testing.assert_close(out, F.conv2d(x, wb.float(), b, padding=1), atol=5e-3, rtol=2e-3)
    gout = torch.randn(B, 2, H, W, device=DEV, generator=g)
    dx = torch.empty(B, H, W, 256, device=DEV, dtype=H16)
    ext_ops.fh2_dgrad_(gout, wb.permute(2, 3, 1, 0).contiguous(), fm, dx)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, wb.float(), b, padding=1).backward(_h(gout))
    torch.testing.assert_close(dx.float(), (xr.grad * (x > 0)).permute(0, 2, 3, 1), atol=5e-3, rtol=3e-3)
    part = torch.empty(4, 2 * 9 * 256 + 2, device=DEV)
    ext_ops.fh2_wgrad_([gout], [fm], part)
    ps = part.sum(0)
    wr = wb.float().clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    F.conv2d(x, wr, br, padding=1).backward(gout)
    torch.testing.assert_close(ps[:-2].view(2, 9 * 256), wr.grad.permute(0, 2, 3, 1).reshape(2, -1),
                               atol=1e-2, rtol=1e-3)


@pytest.mark.parametrize('w', [31, 32])
def test_lookup_and_fold_fp16(ext_ops, w):
    """fp16 taps from the fp32 pyramid (the reference's fp32 correlation under fp16 autocast)
    and the correlation fold from fp16 tap gradients (even width: the union-box fold with fp32
    dC): equal to the bf16 / fp32 paths up to the 16-bit rounding of the taps."""
    b, c, h = 2, 256, 23
    f1 = torch.randn(b, c, h, w, device=DEV)
    f2 = torch.randn(b, c, h, w, device=DEV)
    pyr = ext_ops.corr_build(f1, f2, 4)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    g = torch.Generator(device='cpu').manual_seed(0)
    coords = (torch.stack([xs, ys])[None].repeat(b, 1, 1, 1) +
              3 * torch.randn(b, 2, h, w, generator=g)).to(DEV)
    o16 = torch.empty(b, h, w, 384, device=DEV, dtype=H16)
    o32 = torch.empty(b, h, w, 384, device=DEV, dtype=torch.bfloat16)
    ext_ops.corr_lookup_nhwc_(pyr, coords, 4, o16)
    ext_ops.corr_lookup_nhwc_(pyr, coords, 4, o32)
    ref = ext_ops.corr_lookup_fwd(pyr, coords, 4).permute(0, 2, 3, 1)
    assert (o16[..., 324:] == 0).all()
    err16 = (o16[..., :324].float() - ref).abs().max().item()
    assert err16 <= 2.0 ** -10 * ref.abs().max().item() + 1e-5, err16
    taps = [torch.randn(b, h, w, 384, device=DEV) for _ in range(3)]
    cs = [coords + k * 0.3 for k in range(3)]
    d16 = ext_ops.corr_tap_reduce(cs, [t.to(H16) for t in taps], h, w, 4, 4, 1 / 16, False)
    d32 = ext_ops.corr_tap_reduce(cs, [t.to(torch.bfloat16) for t in taps], h, w, 4, 4, 1 / 16, False)
    # the two differ only by the taps' 16-bit rounding (fp16: 11 bits, bf16: 8 bits)
    rel = ((d16 - d32).norm() / d32.norm()).item()
    assert rel < 1e-2, rel
    # and the fp16 fold is the generic fp32 lookup backward of the fp16-rounded taps
    gp = [torch.zeros_like(p) for p in pyr]
    for cc, t in zip(cs, taps):
        ext_ops.corr_lookup_bwd_(gp, cc, t.to(H16).float().contiguous(), 4)
    dref = ext_ops.corr_pyr_grad_reduce(gp, 1 / 16)
    assert ((d16 - dref).norm() / dref.norm()).item() < 1e-5


def test_onthefly_lookup_nhwc_fp16_taps(ext_ops):
    """On-the-fly correlation under fp16 autocast: the fp32-accurate split forward writes fp16
    taps itself (no bf16 rounding + cast), within fp16 rounding of the fp32 all-pairs lookup."""
    from pytorch_raft_amd.models.corr import AlternateCorrBlock
    b, c, h, w = 2, 256, 16, 24
    g = torch.Generator(device='cpu').manual_seed(4)
    f1 = torch.randn(b, c, h, w, generator=g).to(DEV)
    f2 = torch.randn(b, c, h, w, generator=g).to(DEV)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    coords = (torch.stack([xs, ys])[None].repeat(b, 1, 1, 1) +
              2 * torch.randn(b, 2, h, w, generator=g)).to(DEV)
    blk = AlternateCorrBlock(f1, f2, radius=4, impl='hip', precision='fp32')
    out = blk.lookup_nhwc(coords, 384, H16)
    assert out.dtype == H16 and out.shape == (b, h, w, 384)
    assert (out[..., 324:] == 0).all()
    ref = ext_ops.corr_lookup_fwd(ext_ops.corr_build(f1, f2, 4), coords, 4).permute(0, 2, 3, 1)
    err = (out[..., :324].float() - ref).abs().max().item()
    assert err <= 2.0 ** -10 * ref.abs().max().item() + 1e-4, err
