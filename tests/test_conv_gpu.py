"""Implicit-GEMM MFMA conv kernel vs a plain PyTorch fp32 conv of the same bf16 operands."""
import pytest
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import conv as C

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _ref(x_nchw, w, b, pad):
    # fp32 reference on the bf16-rounded operands
    return F.conv2d(x_nchw.to(torch.bfloat16).float(), w.to(torch.bfloat16).float(), b, padding=pad)


@pytest.mark.parametrize('cin,cout,k,epi', [
    (256, 192, (3, 3), C.EPI_RELU_BF16),
    (384, 256, (1, 5), C.EPI_BF16),
    (384, 128, (5, 1), C.EPI_F32),
    (128, 576, (1, 1), C.EPI_F32),
    (256, 2, (3, 3), C.EPI_F32),
    (128, 126, (3, 3), C.EPI_RELU_BF16),
])
def test_conv_fwd_single_segment(ext_ops, cin, cout, k, epi):
    torch.manual_seed(0)
    B, H, W = 2, 13, 21
    x = torch.randn(B, cin, H, W, device=DEV)
    w = torch.randn(cout, cin, *k, device=DEV) / (cin * k[0] * k[1]) ** 0.5
    b = torch.randn(cout, device=DEV)
    pad = (k[0] // 2, k[1] // 2)
    ref = _ref(x, w, b, pad)
    if epi == C.EPI_RELU_BF16:
        ref = ref.relu()
    xb = C.nhwc(x)
    wpk = C.pack_weight(w, [cin], [cin])
    f32 = epi in (C.EPI_F32, C.EPI_ACC_F32)
    out = torch.zeros(B, H, W, cout + 6, device=DEV, dtype=torch.float32 if f32 else torch.bfloat16)
    C.conv_fwd([(xb, 0, cin)], wpk, b, k, pad, cout, epi, [out], [3])
    got = C.nchw(out[..., 3:3 + cout]).float()
    tol = 2e-2 if not f32 else 2e-3
    torch.testing.assert_close(got, ref, atol=tol * max(1.0, ref.abs().max().item()), rtol=tol)
    assert torch.all(out[..., :3] == 0) and torch.all(out[..., 3 + cout:] == 0)


def test_conv_fwd_multi_segment_padded(ext_ops):
    torch.manual_seed(1)
    B, H, W = 2, 9, 17
    # 324 real channels in a 384-wide buffer + a 64-channel second segment at an offset
    x1 = torch.randn(B, 324, H, W, device=DEV)
    x2 = torch.randn(B, 64, H, W, device=DEV)
    w = torch.randn(96, 388, 3, 3, device=DEV) / 60
    b = torch.randn(96, device=DEV)
    ref = _ref(torch.cat([x1, x2], 1), w, b, (1, 1))
    buf1 = torch.zeros(B, H, W, 384, device=DEV, dtype=torch.bfloat16)
    buf1[..., :324] = C.nhwc(x1)
    buf2 = torch.zeros(B, H, W, 128, device=DEV, dtype=torch.bfloat16)
    buf2[..., 32:96] = C.nhwc(x2)
    wpk = C.pack_weight(w, [324, 64], [384, 64])
    out = torch.empty(B, H, W, 96, device=DEV)
    C.conv_fwd([(buf1, 0, 384), (buf2, 32, 64)], wpk, b, (3, 3), (1, 1), 96, C.EPI_F32, [out], [0])
    torch.testing.assert_close(C.nchw(out), ref, atol=2e-3, rtol=2e-3)


def test_conv_fwd_small_cin(ext_ops):
    torch.manual_seed(2)
    B, H, W = 3, 11, 15
    x = torch.randn(B, 2, H, W, device=DEV) * 4
    w = torch.randn(128, 2, 7, 7, device=DEV) / 10
    b = torch.randn(128, device=DEV)
    ref = _ref(x, w, b, (3, 3)).relu()
    buf = torch.zeros(B, H, W, 8, device=DEV, dtype=torch.bfloat16)
    buf[..., :2] = C.nhwc(x)
    wpk = C.pack_weight_small(w)
    out = torch.empty(B, H, W, 128, device=DEV, dtype=torch.bfloat16)
    C.conv_fwd([(buf, 0, 8)], wpk, b, (7, 7), (3, 3), 128, C.EPI_RELU_BF16, [out], [0], cin_small=2)
    torch.testing.assert_close(C.nchw(out).float(), ref, atol=3e-2, rtol=2e-2)


def test_conv_gru_epilogues(ext_ops):
    torch.manual_seed(3)
    B, H, W, hd = 2, 10, 14, 128
    h = torch.randn(B, hd, H, W, device=DEV).tanh()
    x = torch.randn(B, 256, H, W, device=DEV)
    wzr = torch.randn(2 * hd, hd + 256, 1, 5, device=DEV) / 40
    bzr = torch.randn(2 * hd, device=DEV) * 0.1
    wq = torch.randn(hd, hd + 256, 1, 5, device=DEV) / 40
    bq = torch.randn(hd, device=DEV) * 0.1
    hb, xb = C.nhwc(h), C.nhwc(x)
    hr, xr = hb.float().permute(0, 3, 1, 2), xb.float().permute(0, 3, 1, 2)
    zr = torch.sigmoid(_ref(torch.cat([hr, xr], 1), wzr, bzr, (0, 2)))
    z, r = zr[:, :hd], zr[:, hd:]
    z_b, r_b = z.to(torch.bfloat16).float(), r.to(torch.bfloat16).float()
    rh = (r_b * hr).to(torch.bfloat16).float()
    q = torch.tanh(_ref(torch.cat([rh, xr], 1), wq, bq, (0, 2)))
    hn = hr + z_b * (q - hr)

    zbuf = torch.empty(B, H, W, hd, device=DEV, dtype=torch.bfloat16)
    rhbuf = torch.empty_like(zbuf)
    rbuf = torch.empty_like(zbuf)
    C.conv_fwd([(hb, 0, hd), (xb, 0, 256)], C.pack_weight(wzr, [hd, 256], [hd, 256]), bzr, (1, 5),
               (0, 2), 2 * hd, C.EPI_GRU_ZR, [zbuf, rhbuf, rbuf], [0, 0, 0], aux=[hb], aux_offs=[0],
               split=hd)
    torch.testing.assert_close(C.nchw(zbuf).float(), z, atol=1e-2, rtol=1e-2)
    torch.testing.assert_close(C.nchw(rbuf).float(), r, atol=1e-2, rtol=1e-2)
    hnew = torch.empty_like(zbuf)
    qbuf = torch.empty_like(zbuf)
    C.conv_fwd([(rhbuf, 0, hd), (xb, 0, 256)], C.pack_weight(wq, [hd, 256], [hd, 256]), bq, (1, 5),
               (0, 2), hd, C.EPI_GRU_Q, [hnew, qbuf], [0, 0], aux=[hb, zbuf], aux_offs=[0, 0])
    torch.testing.assert_close(C.nchw(qbuf).float(), q, atol=3e-2, rtol=3e-2)
    torch.testing.assert_close(C.nchw(hnew).float(), hn, atol=3e-2, rtol=3e-2)


def test_conv_dgrad_via_flipped_weights(ext_ops):
    torch.manual_seed(4)
    B, H, W = 2, 12, 16
    for cin, cout, k in [(256, 192, (3, 3)), (384, 128, (1, 5)), (384, 256, (5, 1))]:
        pad = (k[0] // 2, k[1] // 2)
        x = torch.randn(B, cin, H, W, device=DEV, requires_grad=True)
        w = (torch.randn(cout, cin, *k, device=DEV) / 30).to(torch.bfloat16).float()
        g = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).float()
        F.conv2d(x, w, None, padding=pad).backward(g)
        gb = C.nhwc(g)
        dx = torch.zeros(B, H, W, cin, device=DEV)
        C.conv_fwd([(gb, 0, cout)], C.pack_weight_dgrad(w, [cout], [cout]), None, k, pad, cin,
                   C.EPI_ACC_F32, [dx], [0])
        torch.testing.assert_close(C.nchw(dx), x.grad, atol=5e-3, rtol=5e-3)


@pytest.mark.parametrize('cin,cout,k,segs', [
    (256, 192, (3, 3), None),
    (384, 256, (1, 5), (128, 256)),
    (128, 576, (1, 1), None),
    (256, 2, (3, 3), None),
    (96, 126, (3, 3), None),
])
def test_conv_wgrad(ext_ops, cin, cout, k, segs):
    torch.manual_seed(5)
    B, H, W = 2, 11, 19
    pad = (k[0] // 2, k[1] // 2)
    x = torch.randn(B, cin, H, W, device=DEV).to(torch.bfloat16).float()
    w = torch.randn(cout, cin, *k, device=DEV, requires_grad=True)
    b = torch.zeros(cout, device=DEV, requires_grad=True)
    g = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).float()
    F.conv2d(x, w, b, padding=pad).backward(g)
    xb = C.nhwc(x)
    if segs is None:
        seg_list, real, padc = [(xb, 0, cin)], [cin], [cin]
    else:
        seg_list = [(C.nhwc(x[:, :segs[0]]), 0, segs[0]), (C.nhwc(x[:, segs[0]:]), 0, segs[1])]
        real = padc = list(segs)
    gb = torch.zeros(B, H, W, C.round_up(cout, 8), device=DEV, dtype=torch.bfloat16)
    gb[..., :cout] = C.nhwc(g)
    dw = torch.zeros(cout, k[0] * k[1] * cin, device=DEV)
    db = torch.zeros(cout, device=DEV)
    C.conv_wgrad(gb, 0, seg_list, k, pad, cout, dw, db)
    got = C.unpack_weight_grad(dw, cout, real, padc, k)
    scale = w.grad.abs().max().item()
    torch.testing.assert_close(got, w.grad, atol=2e-3 * scale, rtol=1e-3)
    torch.testing.assert_close(db, b.grad, atol=1e-3 * b.grad.abs().max().item(), rtol=1e-3)


def test_conv_wgrad_small_cin(ext_ops):
    torch.manual_seed(6)
    B, H, W = 2, 9, 13
    x = (torch.randn(B, 2, H, W, device=DEV) * 3).to(torch.bfloat16).float()
    w = torch.randn(128, 2, 7, 7, device=DEV, requires_grad=True)
    g = torch.randn(B, 128, H, W, device=DEV).to(torch.bfloat16).float()
    F.conv2d(x, w, None, padding=3).backward(g)
    buf = torch.zeros(B, H, W, 8, device=DEV, dtype=torch.bfloat16)
    buf[..., :2] = C.nhwc(x)
    dw = torch.zeros(128, 128, device=DEV)
    C.conv_wgrad(C.nhwc(g), 0, [(buf, 0, 8)], (7, 7), (3, 3), 128, dw, None, cin_small=2)
    got = C.unpack_weight_grad_small(dw, 128, 2, (7, 7))
    torch.testing.assert_close(got, w.grad, atol=2e-3 * w.grad.abs().max().item(), rtol=1e-3)


def test_conv_dgrad_relu_gated_bf16(ext_ops):
    """conv_dgrad_ with a bf16 output segment: the ReLU backward of the layer below is fused in."""
    torch.manual_seed(7)
    B, H, W, cin, cout, k = 2, 12, 16, 256, 192, (3, 3)
    pad = (1, 1)
    x = torch.randn(B, cin, H, W, device=DEV, requires_grad=True)
    w = (torch.randn(cout, cin, *k, device=DEV) / 30).to(torch.bfloat16).float()
    g = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).float()
    F.conv2d(x, w, None, padding=pad).backward(g)
    y = torch.randn(B, H, W, cin + 64, device=DEV).relu().to(torch.bfloat16)  # relu output, offset 32
    ref = x.grad * (y[..., 32:32 + cin].permute(0, 3, 1, 2).float() > 0)
    out = torch.full((B, H, W, cin + 16), 7.0, device=DEV, dtype=torch.bfloat16)
    wd = C.pack_weight_dgrad(w, [cout], [cout])
    torch.ops.raft_amd.conv_dgrad_([C.nhwc(g)], [0], [cout], wd, 3, 3, 1, 1, 0, 1.0, [out], [8],
                                   [cin], [cin], [0], [y], [32], [], [])
    torch.testing.assert_close(C.nchw(out[..., 8:8 + cin]).float(), ref, atol=2e-2, rtol=2e-2)
    assert torch.all(out[..., :8] == 7.0) and torch.all(out[..., 8 + cin:] == 7.0)


@pytest.mark.parametrize('cin,cout,k,segs,g_off,pps', [
    (256, 192, (3, 3), None, 0, None),
    (384, 256, (1, 5), (128, 128, 128), 0, 128),
    (128, 576, (1, 1), None, 0, None),
    (256, 2, (3, 3), None, 0, 64),
    (128, 64, (3, 3), None, 64, None),
])
def test_conv_wgrad_multi_items(ext_ops, cin, cout, k, segs, g_off, pps):
    """One launch summing the weight gradient of several (grad, input) items (GRU iterations)."""
    torch.manual_seed(7)
    B, H, W = 2, 11, 19
    n_items = 3
    pad = (k[0] // 2, k[1] // 2)
    w = torch.randn(cout, cin, *k, device=DEV, requires_grad=True)
    b = torch.zeros(cout, device=DEV, requires_grad=True)
    items = []
    for _ in range(n_items):
        x = torch.randn(B, cin, H, W, device=DEV).to(torch.bfloat16).float()
        g = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).float()
        F.conv2d(x, w, b, padding=pad).backward(g)
        gb = torch.zeros(B, H, W, g_off + C.round_up(cout, 8), device=DEV, dtype=torch.bfloat16)
        gb[..., g_off:g_off + cout] = C.nhwc(g)
        if segs is None:
            bufs = [C.nhwc(x)]
        else:
            bufs, o = [], 0
            for c in segs:
                bufs.append(C.nhwc(x[:, o:o + c]))
                o += c
        items.append((gb, bufs))
    seg_cnt = [cin] if segs is None else list(segs)
    dw = torch.zeros(cout, k[0] * k[1] * cin, device=DEV)
    db = torch.zeros(cout, device=DEV)
    C.conv_wgrad_multi(items, g_off, [0] * len(seg_cnt), seg_cnt, k, pad, cout, dw, db,
                       pix_per_split=pps)
    got = C.unpack_weight_grad(dw, cout, seg_cnt, seg_cnt, k)
    scale = w.grad.abs().max().item()
    torch.testing.assert_close(got, w.grad, atol=2e-3 * scale, rtol=1e-3)
    torch.testing.assert_close(db, b.grad, atol=1e-3 * b.grad.abs().max().item(), rtol=1e-3)


@pytest.mark.parametrize('cin,cout,k,segs,g_off,splits', [
    (256, 192, (3, 3), None, 0, 0),
    (384, 256, (1, 5), (128, 128, 128), 0, 0),
    (384, 256, (5, 1), (128, 256), 0, 3),
    (128, 576, (1, 1), None, 0, 0),
    (128, 64, (3, 3), None, 64, 1),
    (192, 126, (3, 3), (64, 128), 0, 0),
    (64, 80, (3, 3), None, 0, 0),
    (96, 64, (3, 3), None, 0, 0),        # 64-wide Cout tile, 32-channel Cin tail
    (96, 96, (3, 3), None, 0, 5),        # Cin tail at 128-wide Cout tiles
    (64, 48, (3, 3), None, 8, 0),
])
def test_conv_wgrad_taps(ext_ops, cin, cout, k, segs, g_off, splits):
    """Tap-fused weight gradient (halo tiles, all taps per workgroup, deterministic split reduce)
    vs the fp32 PyTorch conv weight/bias gradient, summed over 3 items."""
    torch.manual_seed(11)
    B, H, W = 2, 13, 21
    pad = (k[0] // 2, k[1] // 2)
    w = torch.randn(cout, cin, *k, device=DEV, requires_grad=True)
    b = torch.zeros(cout, device=DEV, requires_grad=True)
    items = []
    for _ in range(3):
        x = torch.randn(B, cin, H, W, device=DEV).to(torch.bfloat16).float()
        g = torch.randn(B, cout, H, W, device=DEV).to(torch.bfloat16).float()
        F.conv2d(x, w, b, padding=pad).backward(g)
        gb = torch.full((B, H, W, g_off + C.round_up(cout, 8)), 3.0, device=DEV,
                        dtype=torch.bfloat16)
        gb[..., g_off:g_off + cout] = C.nhwc(g)
        if cout % 8:  # channels past cout inside the last 8-wide chunk are ignored
            gb[..., g_off + cout:] = 5.0
        if segs is None:
            bufs = [C.nhwc(x)]
        else:
            bufs, o = [], 0
            for c in segs:
                bufs.append(C.nhwc(x[:, o:o + c]))
                o += c
        items.append((gb, bufs))
    seg_cnt = [cin] if segs is None else list(segs)
    dw = torch.ones(cout, k[0] * k[1] * cin, device=DEV)   # accumulates into existing values
    db = torch.ones(cout, device=DEV)
    C.conv_wgrad_taps(items, g_off, [0] * len(seg_cnt), seg_cnt, k, pad, cout, dw, db,
                      splits=splits)
    got = C.unpack_weight_grad(dw - 1.0, cout, seg_cnt, seg_cnt, k)
    scale = w.grad.abs().max().item()
    torch.testing.assert_close(got, w.grad, atol=2e-3 * scale, rtol=1e-3)
    torch.testing.assert_close(db - 1.0, b.grad, atol=1e-3 * b.grad.abs().max().item(), rtol=1e-3)
    # deterministic: a second run gives bit-identical results
    dw2 = torch.ones_like(dw)
    db2 = torch.ones_like(db)
    C.conv_wgrad_taps(items, g_off, [0] * len(seg_cnt), seg_cnt, k, pad, cout, dw2, db2,
                      splits=splits)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


HALO_CFGS = (30, 31, 32, 33)   # conv_igemm.hip kCfgs: the halo-tile kernel (conv_halo.h)
GATE_CFGS = HALO_CFGS


@pytest.mark.parametrize('cfg', HALO_CFGS)
@pytest.mark.parametrize('segs,cout,k,hw', [
    ([256], 192, (3, 3), (13, 21)),
    ([128, 128], 256, (1, 5), (13, 21)),
    ([128, 128], 128, (5, 1), (11, 62)),    # 5x1 at W = 62: the largest (16-piece) A image
    ([384], 256, (1, 1), (9, 17)),
    ([128], 126, (3, 3), (46, 62)),
])
def test_conv_halo_fwd(ext_ops, cfg, segs, cout, k, hw):
    """Halo-tile kernels forced for every tile shape: fwd vs an fp32 conv of the bf16 operands,
    across image / batch boundaries (rows whose shifted neighbour leaves the image read zeros)."""
    torch.manual_seed(5)
    B, (H, W) = 2, hw
    cin = sum(segs)
    xs = [torch.randn(B, c, H, W, device=DEV) for c in segs]
    w = torch.randn(cout, cin, *k, device=DEV) / (cin * k[0] * k[1]) ** 0.5
    b = torch.randn(cout, device=DEV)
    pad = (k[0] // 2, k[1] // 2)
    ref = _ref(torch.cat(xs, 1), w, b, pad)
    bufs = [C.nhwc(x) for x in xs]
    wpk = C.pack_weight(w, segs, segs)
    out = torch.zeros(B, H, W, cout + 2, device=DEV)
    torch.ops.raft_amd.conv_set_forced_cfg(cfg)
    try:
        C.conv_fwd([(t, 0, c) for t, c in zip(bufs, segs)], wpk, b, k, pad, cout, C.EPI_F32,
                   [out], [0])
        torch.cuda.synchronize()
    finally:
        torch.ops.raft_amd.conv_set_forced_cfg(-1)
    torch.testing.assert_close(C.nchw(out[..., :cout]), ref, atol=2e-3 * max(1.0, ref.abs().max().item()),
                               rtol=2e-3)
    assert torch.all(out[..., cout:] == 0)


@pytest.mark.parametrize('cfg', GATE_CFGS)
def test_conv_halo_gru_and_dgrad(ext_ops, cfg):
    """Halo kernels under the GRU gate epilogue (with a per-pixel bias map) and the multi-segment
    dgrad epilogue (fp32 store + accumulate), against the register / LDS-DMA kernels' results."""
    torch.manual_seed(6)
    B, H, W, hd = 2, 10, 14, 128
    h = C.nhwc(torch.randn(B, hd, H, W, device=DEV).tanh())
    x = C.nhwc(torch.randn(B, 128, H, W, device=DEV))
    wzr = torch.randn(2 * hd, 2 * hd, 1, 5, device=DEV) / 40
    bmap = torch.randn(B, H, W, 2 * hd, device=DEV) * 0.1
    wpk = C.pack_weight(wzr, [hd, 128], [hd, 128])
    g = C.nhwc(torch.randn(B, 2 * hd, H, W, device=DEV))
    wd = C.pack_weight_dgrad(wzr, [2 * hd], [2 * hd])
    zb = torch.zeros(2 * hd, device=DEV)

    def run():
        z, rh, r = (torch.empty(B, H, W, hd, device=DEV, dtype=torch.bfloat16) for _ in range(3))
        C.conv_fwd([(h, 0, hd), (x, 0, 128)], wpk, bmap, (1, 5), (0, 2), 2 * hd, C.EPI_GRU_ZR,
                   [z, rh, r], [0, 0, 0], aux=[h], aux_offs=[0], split=hd)
        dh = torch.randn(B, H, W, hd, device=DEV, generator=torch.Generator(DEV).manual_seed(7))
        dx = torch.empty(B, H, W, 128, device=DEV)
        torch.ops.raft_amd.conv_dgrad_(
            [g], [0], [2 * hd], wd, 1, 5, 0, 2, 0, 1.0, [dh, dx], [0, 0], [hd, 128], [hd, 128],
            [1, 0], [dh, dx], [0, 0], [], [])
        torch.cuda.synchronize()
        return z.float(), rh.float(), r.float(), dh, dx

    want = run()
    torch.ops.raft_amd.conv_set_forced_cfg(cfg)
    try:
        got = run()
    finally:
        torch.ops.raft_amd.conv_set_forced_cfg(-1)
    for name, a_, b_ in zip(('z', 'rh', 'r', 'dh', 'dx'), got, want):
        torch.testing.assert_close(a_, b_, atol=2e-2, rtol=1e-2, msg=lambda m: name + ': ' + m)
