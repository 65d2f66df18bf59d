"""Encoder norm kernels (encoder_norm.hip) on the chairs shapes: time per call of the forward
(statistics + finalize + apply) and backward (statistics + finalize + apply) passes, with the
bytes each moves and the achieved HBM bandwidth.  Plain = relu(norm(x)) (`core/extractor.py:
22-25`); block-end = relu(relu(norm(x)) + res), whose backward also reads the block output and
writes g (`core/extractor.py:47-56`).
usage: PYTHONPATH=. python scripts/norm_bench.py"""
import torch

from pytorch_raft_amd.ops import _ext
from scripts.conv_bench import timeit

dev = torch.device('cuda')
ops = _ext.ops()
CL = torch.channels_last
bf = torch.bfloat16


def t(*shape):
    return torch.randn(*shape, device=dev).to(bf).contiguous(memory_format=CL)


print('%-28s %9s %9s %9s %9s' % ('layer', 'fwd us', 'fwd TB/s', 'bwd us', 'bwd TB/s'))
for name, n, c, h, w, mode in [('fnet l1 (instance)', 24, 64, 184, 248, 0),
                               ('cnet l1 (batch)', 12, 64, 184, 248, 1),
                               ('fnet l2 (instance)', 24, 96, 92, 124, 0),
                               ('fnet l3 (instance)', 24, 128, 46, 62, 0)]:
    g = torch.ones(c, device=dev) if mode == 1 else None
    b = torch.zeros(c, device=dev) if mode == 1 else None
    rm = torch.zeros(c, device=dev) if mode == 1 else None
    rv = torch.ones(c, device=dev) if mode == 1 else None
    x, res, dy = t(n, c, h, w), t(n, c, h, w), t(n, c, h, w)
    y = torch.empty_like(x)
    dx, gout = torch.empty_like(x), torch.empty_like(x)
    dg = torch.empty(c, device=dev) if mode == 1 else None
    db = torch.empty(c, device=dev) if mode == 1 else None
    nb = x.numel() * 2
    for kind in ('plain', 'block-end'):
        r = res if kind == 'block-end' else None
        fwd = lambda: ops.norm_fwd_(x, mode, 1, g, b, None, rm, rv, 0.1, 1e-5, r, y, None)  # noqa
        mean, invstd = fwd()
        if kind == 'plain':
            bwd = lambda: ops.norm_bwd_(dy, x, None, mean, invstd, mode, 1, g, b, dg, db, None, dx)  # noqa
            fb, bb = 3 * nb, 5 * nb            # fwd: x twice (stats, apply) + y; bwd: (dy, x) x 2 + dx
        else:
            bwd = lambda: ops.norm_bwd_(dy, x, None, mean, invstd, mode, 1, g, b, dg, db, None, dx,  # noqa
                                        None, y, gout)
            fb = 4 * nb                        # + res
            bb = 7 * nb                        # stats: dy, x, y, gout; apply: gout, x, dx
        tf, tb = timeit(fwd, 20), timeit(bwd, 20)
        print('%-28s %9.1f %9.2f %9.1f %9.2f' % (name + ' ' + kind, tf, fb / tf / 1e6, tb, bb / tb / 1e6),
              flush=True)
