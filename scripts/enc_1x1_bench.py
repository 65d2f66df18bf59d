"""Encoder convs that still run on MIOpen at chairs (`core/extractor.py:44-45,144`): the 1x1
stride-2 downsample convs, the 1x1 output conv (with bias) and, for reference, the 3x3 stride-2
convs. MIOpen forward / input gradient / weight gradient vs the same 1x1 conv as plain GEMMs on
the channels_last (pixels, channels) matrix (hipBLASLt), with the stride-2 gather / scatter.
usage: PYTHONPATH=. python scripts/enc_1x1_bench.py"""
import torch
import torch.nn.functional as F

from scripts.conv_bench import timeit

dev = torch.device('cuda')
bf = torch.bfloat16
CL = torch.channels_last


def gemm_fwd(x, w2, b, s):
    xs = x[:, :, ::s, ::s] if s > 1 else x
    n, c, h, wd = xs.shape
    x2 = xs.permute(0, 2, 3, 1).reshape(n * h * wd, c)
    y2 = F.linear(x2, w2, b)
    return y2.view(n, h, wd, -1).permute(0, 3, 1, 2)


def gemm_dgrad(gy, w2, s, xshape):
    n, co, h, wd = gy.shape
    g2 = gy.permute(0, 2, 3, 1).reshape(n * h * wd, co)
    dxs = (g2 @ w2).view(n, h, wd, -1).permute(0, 3, 1, 2)
    if s == 1:
        return dxs
    dx = torch.empty(xshape, device=gy.device, dtype=gy.dtype, memory_format=CL).zero_()
    dx[:, :, ::s, ::s] = dxs
    return dx


def gemm_wgrad(gy, x, s):
    xs = x[:, :, ::s, ::s] if s > 1 else x
    n, c, h, wd = xs.shape
    x2 = xs.permute(0, 2, 3, 1).reshape(n * h * wd, c)
    g2 = gy.permute(0, 2, 3, 1).reshape(n * h * wd, -1)
    return g2.t() @ x2, g2.sum(0, dtype=torch.float32)


for name, B, H, W, ci, co, k, s in [
        ('fnet.l2.down 1x1 s2', 24, 184, 248, 64, 96, 1, 2), ('cnet.l2.down 1x1 s2', 12, 184, 248, 64, 96, 1, 2),
        ('fnet.l3.down 1x1 s2', 24, 92, 124, 96, 128, 1, 2), ('cnet.l3.down 1x1 s2', 12, 92, 124, 96, 128, 1, 2),
        ('fnet.out 1x1', 24, 46, 62, 128, 256, 1, 1), ('cnet.out 1x1', 12, 46, 62, 128, 256, 1, 1),
        ('fnet.l2.conv1 3x3 s2', 24, 184, 248, 64, 96, 3, 2), ('cnet.l2.conv1 3x3 s2', 12, 184, 248, 64, 96, 3, 2),
        ('fnet.l3.conv1 3x3 s2', 24, 92, 124, 96, 128, 3, 2), ('cnet.l3.conv1 3x3 s2', 12, 92, 124, 96, 128, 3, 2)]:
    p = k // 2
    x = torch.randn(B, ci, H, W, device=dev).to(bf).contiguous(memory_format=CL)
    w = (torch.randn(co, ci, k, k, device=dev) / (k * k * ci) ** 0.5).to(bf).contiguous(memory_format=CL)
    b = torch.randn(co, device=dev).to(bf) if s == 1 else None
    y = F.conv2d(x, w, b, s, p)
    gy = torch.randn_like(y).contiguous(memory_format=CL)
    t_mf = timeit(lambda: F.conv2d(x, w, b, s, p), 20)
    t_md = timeit(lambda: torch.ops.aten.convolution_backward(
        gy, x, w, None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, False, False]), 20)
    t_mw = timeit(lambda: torch.ops.aten.convolution_backward(
        gy, x, w, [co] if b is not None else None, [s, s], [p, p], [1, 1], False, [0, 0], 1,
        [False, True, b is not None]), 20)
    line = f'{name:22s}: miopen fwd {t_mf:6.1f} dgrad {t_md:6.1f} wgrad {t_mw:6.1f} us'
    if k == 1:
        w2 = w.view(co, ci)
        t_gf = timeit(lambda: gemm_fwd(x, w2, b, s), 20)
        t_gd = timeit(lambda: gemm_dgrad(gy, w2, s, x.shape), 20)
        t_gw = timeit(lambda: gemm_wgrad(gy, x, s), 20)
        yr = F.conv2d(x.float(), w.float(), b.float() if b is not None else None, s, p)
        yg = gemm_fwd(x, w2, b, s).float()
        dxr, dwr, _ = torch.ops.aten.convolution_backward(
            gy.float(), x.float(), w.float(), None, [s, s], [p, p], [1, 1], False, [0, 0], 1, [True, True, False])
        dxg = gemm_dgrad(gy, w2, s, x.shape).float()
        dwg = gemm_wgrad(gy, x, s)[0].float().view_as(dwr)
        e = [(a - r).abs().max().item() / r.abs().max().item() for a, r in ((yg, yr), (dxg, dxr), (dwg, dwr))]
        line += (f' | gemm fwd {t_gf:6.1f} dgrad {t_gd:6.1f} wgrad {t_gw:6.1f} us'
                 f' (err {e[0]:.1e} {e[1]:.1e} {e[2]:.1e})')
    print(line, flush=True)
