"""Time the correlation fold (corr_tap_reduce: tap gradients of every iteration -> dense bf16 dC)
at the chairs training shape (B=12, 46x62, 4 levels, r=4, 12 iterations).  The kernel variant
follows RAFT_TAPRED (0 = union box, default; 1 = workgroup per pixel; 2 = wave per pixel); prints us per call
and a checksum so the variants can be compared bit for bit."""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import _ext  # noqa: E402


def main():
    ops = _ext.ops()
    b, h, w, iters = 12, 46, 62, 12
    g = torch.Generator(device='cpu').manual_seed(0)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    base = torch.stack([xs, ys])[None].repeat(b, 1, 1, 1)
    c = base + 4 * torch.randn(b, 2, h, w, generator=g)
    coords = []
    for _ in range(iters):   # windows drift per iteration as in training
        c = c + 0.7 * torch.randn(b, 2, h, w, generator=g)
        coords.append(c.clone().cuda())
    douts = [torch.randn(b, h, w, 384, generator=g).to(torch.bfloat16).cuda() for _ in range(iters)]
    for _ in range(3):
        out = ops.corr_tap_reduce(coords, douts, h, w, 4, 4, 1.0 / 16, True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    n = 10
    for _ in range(n):
        out = ops.corr_tap_reduce(coords, douts, h, w, 4, 4, 1.0 / 16, True)
    e1.record()
    torch.cuda.synchronize()
    print('corr_tap_reduce %.1f us/call  checksum %.6f' % (e0.elapsed_time(e1) * 1000 / n,
                                                           out.float().sum().item()), flush=True)


if __name__ == '__main__':
    main()
