"""Flow warping (backward warp by a dense flow field): HIP kernel + torch grid_sample oracle.

``warp_image(x, flo, convention)``: output(p) = x(p + flo(p)), bilinear, zero padding.
``convention='reference'`` reproduces the reference demos exactly: coordinates normalised with
(W-1) / (H-1) but sampled with ``grid_sample``'s default ``align_corners=False``
(`demo_warp.py:45-49`), i.e. sample position (p + flo) * W/(W-1) - 0.5.  ``'exact'`` samples at
p + flo.  Differentiable w.r.t. both image and flow.
"""
import torch
import torch.nn.functional as F

from . import _ext


def _affine(convention, h, w):
    if convention == 'reference':
        return (w / max(w - 1, 1), -0.5, h / max(h - 1, 1), -0.5)
    if convention == 'exact':
        return (1.0, 0.0, 1.0, 0.0)
    raise ValueError(convention)


def torch_warp(x, flo, convention='reference'):
    b, c, h, w = x.shape
    ys, xs = torch.meshgrid(torch.arange(h, device=x.device, dtype=torch.float32),
                            torch.arange(w, device=x.device, dtype=torch.float32), indexing='ij')
    vx = xs[None] + flo[:, 0]
    vy = ys[None] + flo[:, 1]
    if convention == 'reference':
        gx = 2.0 * vx / max(w - 1, 1) - 1.0
        gy = 2.0 * vy / max(h - 1, 1) - 1.0
        return F.grid_sample(x, torch.stack([gx, gy], -1), align_corners=False)
    gx = 2.0 * vx / max(w - 1, 1) - 1.0
    gy = 2.0 * vy / max(h - 1, 1) - 1.0
    return F.grid_sample(x, torch.stack([gx, gy], -1), align_corners=True)


class _Warp(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, flo, sx, bx, sy, by):
        ctx.save_for_backward(x, flo)
        ctx.p = (sx, bx, sy, by)
        return _ext.ops().warp_fwd(x, flo, sx, bx, sy, by)

    @staticmethod
    def backward(ctx, dout):
        x, flo = ctx.saved_tensors
        dimg, dflow = _ext.ops().warp_bwd(x, flo, dout.contiguous().float(), *ctx.p)
        return dimg, dflow, None, None, None, None


def warp_image(x, flo, convention='reference', impl='auto'):
    if impl != 'torch' and _ext.device_ok(x) and _ext.gpu_path_enabled(required=(impl == 'hip')):
        h, w = x.shape[-2:]
        p = _affine(convention, h, w)
        return _Warp.apply(x.float().contiguous(), flo.float().contiguous(), *p)
    return torch_warp(x.float(), flo.float(), convention)
