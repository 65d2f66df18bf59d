"""Split-bf16 fp32 conv (ops/conv_fp32.py) vs fp64 at the encoder's geometries: forward, input and
weight gradients, with the output gradient in NCHW and channels_last layout, autotuned and
heuristic kernel configs.  Prints one line per case (relative errors; ~1e-5 expected)."""
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import _ext, conv_fp32  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ops = _ext.ops()
    cases = [(64, 64, 3, 48, 64), (96, 96, 3, 24, 32), (128, 128, 3, 12, 16), (128, 256, 1, 12, 16),
             (64, 64, 3, 13, 21), (256, 192, 3, 13, 21)]
    for tune in (1, 0):
        ops.conv_set_autotune(tune)
        for cin, cout, k, h, w in cases:
            for layout in ('nchw', 'cl'):
                torch.manual_seed(0)
                x = torch.randn(3, cin, h, w, device='cuda', requires_grad=True)
                wt = (torch.randn(cout, cin, k, k, device='cuda') / (cin * k * k) ** 0.5).requires_grad_()
                bi = torch.randn(cout, device='cuda', requires_grad=True)
                g = torch.randn(3, cout, h, w, device='cuda')
                if layout == 'cl':
                    g = g.contiguous(memory_format=torch.channels_last)
                y = conv_fp32.conv2d(x, wt, bi, (k // 2, k // 2))
                dx, dw = torch.autograd.grad(y, (x, wt), g)
                xd, wd, bd = (t.detach().double().requires_grad_() for t in (x, wt, bi))
                yr = F.conv2d(xd, wd, bd, padding=k // 2)
                dxr, dwr = torch.autograd.grad(yr, (xd, wd), g.double())
                print('tune=%d %3d->%3d k%d %3dx%3d %-4s  y %.2e  dx %.2e  dw %.2e' % (
                    tune, cin, cout, k, h, w, layout, rel(y.double(), yr), rel(dx.double(), dxr),
                    rel(dw.double(), dwr)), flush=True)
    ops.conv_set_autotune(-1)


if __name__ == '__main__':
    main()
