"""Encoder stride-1 3x3 convs (the residual blocks, `core/extractor.py:22-23`): MIOpen NHWC bf16
forward / input gradient vs the update block's implicit-GEMM MFMA kernels on the same operands.
usage: PYTHONPATH=. python scripts/enc_conv_bench.py"""
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import _ext
from pytorch_raft_amd.ops import conv as C
from scripts.conv_bench import timeit

dev = torch.device('cuda')
ops = _ext.ops()
for name, B, H, W, c in [('fnet.l1', 24, 184, 248, 64), ('cnet.l1', 12, 184, 248, 64),
                         ('fnet.l3', 24, 46, 62, 128), ('cnet.l3', 12, 46, 62, 128)]:
    x = torch.randn(B, c, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(c, c, 3, 3, device=dev) / (9 * c) ** 0.5)
    wb = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(B, c, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    t_mf = timeit(lambda: F.conv2d(x, wb, None, 1, 1), 20)
    t_md = timeit(lambda: torch.ops.aten.convolution_backward(
        dy, x, wb, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False]), 20)
    xn, gn = x.permute(0, 2, 3, 1), dy.permute(0, 2, 3, 1)
    wpk = C.pack_weight(w, [c], [c])
    wd = C.pack_weight_dgrad(w, [c], [c])
    out = torch.empty(B, H, W, c, device=dev, dtype=torch.bfloat16)
    dx = torch.empty(B, H, W, c, device=dev, dtype=torch.bfloat16)
    fwd = lambda: C.conv_fwd([(xn, 0, c)], wpk, None, (3, 3), (1, 1), c, C.EPI_BF16, [out], [0])  # noqa
    dgr = lambda: ops.conv_dgrad_([gn], [0], [c], wd, 3, 3, 1, 1, 0, 1.0, [dx], [0], [c], [c], [0], [dx], [-1], [], [])  # noqa
    t_of, t_od = timeit(fwd, 20), timeit(dgr, 20)
    ref = F.conv2d(x.float(), wb.float(), None, 1, 1)
    err = (out.permute(0, 3, 1, 2).float() - ref).abs().max().item() / ref.abs().max().item()
    refd = torch.ops.aten.convolution_backward(dy.float(), x.float(), wb.float(), None, [1, 1], [1, 1], [1, 1],
                                               False, [0, 0], 1, [True, False, False])[0]
    errd = (dx.permute(0, 3, 1, 2).float() - refd).abs().max().item() / refd.abs().max().item()
    print(f'{name}: fwd miopen {t_mf:6.1f} ours {t_of:6.1f} us (err {err:.1e}) | dgrad miopen {t_md:6.1f} '
          f'ours {t_od:6.1f} us (err {errd:.1e})', flush=True)
