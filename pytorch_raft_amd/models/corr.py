"""Correlation volume + multi-scale lookup.

Two user-visible classes with the reference's constructor / call signatures:

* ``CorrBlock(fmap1, fmap2, num_levels=4, radius=4)``  all-pairs 4D volume (`core/corr.py:12-60`).
* ``AlternateCorrBlock(fmap1, fmap2, num_levels=4, radius=4)``  memory-efficient on-the-fly
  correlation (`core/corr.py:63-91` + `alt_cuda_corr/`), here fully differentiable.

Both return ``corr`` of shape (B, L*(2r+1)^2, H, W), float32, channel = level*(2r+1)^2 + ix*(2r+1) + iy
with ix the x-offset index (x-offset-major, `SURVEY.md` §2.7 item 7).

Dispatch: on a GPU tensor with the native extension loaded every call goes to the hand-written
HIP kernels in ``pytorch_raft_amd/csrc/kernels/corr_*.hip`` (via ``pytorch_raft_amd.ops.corr``).
On CPU (or with ``impl='torch'``) the pure-PyTorch formulation below runs; it is also the numerics
oracle the GPU tests compare against.
"""
import math

import torch
import torch.nn.functional as F

from ..utils.utils import bilinear_sampler
from ..ops import corr as corr_ops
from ..ops import _ext


def _window_delta(r, device, dtype=torch.float32):
    """(2r+1, 2r+1, 2) offsets; first window axis offsets x, second offsets y."""
    lin = torch.arange(-r, r + 1, device=device, dtype=dtype)
    a, b = torch.meshgrid(lin, lin, indexing='ij')
    return torch.stack([a, b], dim=-1)


def torch_corr_volume(fmap1, fmap2):
    """(B, C, H, W) x 2 -> (B, H, W, 1, H, W) scaled by 1/sqrt(C)  (`core/corr.py:52-60`)."""
    b, c, h, w = fmap1.shape
    f1 = fmap1.reshape(b, c, h * w)
    f2 = fmap2.reshape(b, c, h * w)
    corr = torch.matmul(f1.transpose(1, 2), f2)
    return corr.view(b, h, w, 1, h, w) / math.sqrt(c)


def torch_corr_pyramid(fmap1, fmap2, num_levels):
    corr = torch_corr_volume(fmap1, fmap2)
    b, h1, w1, d, h2, w2 = corr.shape
    corr = corr.reshape(b * h1 * w1, d, h2, w2)
    pyr = [corr]
    for _ in range(num_levels - 1):
        corr = F.avg_pool2d(corr, 2, stride=2)
        pyr.append(corr)
    return pyr


def torch_corr_lookup(pyramid, coords, radius):
    """Pure-torch lookup on an all-pairs pyramid (`core/corr.py:29-50`)."""
    r = radius
    coords = coords.permute(0, 2, 3, 1)
    b, h1, w1, _ = coords.shape
    delta = _window_delta(r, coords.device).view(1, 2 * r + 1, 2 * r + 1, 2)
    out = []
    for lvl, corr in enumerate(pyramid):
        centroid = coords.reshape(b * h1 * w1, 1, 1, 2) / 2 ** lvl
        sampled = bilinear_sampler(corr, centroid + delta)
        out.append(sampled.view(b, h1, w1, -1))
    out = torch.cat(out, dim=-1)
    return out.permute(0, 3, 1, 2).contiguous().float()


def torch_onthefly_corr(fmap_pyramid2, fmap1, coords, radius):
    """Differentiable pure-torch on-the-fly correlation (oracle for the HIP alternate path).

    For every query pixel and level it gathers the (2r+2)^2 integer fmap2 positions around the
    centroid, dots them with fmap1 and blends the bilinear taps -- exactly the arithmetic of
    ``alt_cuda_corr`` forward (`alt_cuda_corr/correlation_kernel.cu:59-115`), with zero padding.
    Memory is O(HW * (2r+2)^2 * C) per level, so keep it to small shapes (tests / CPU).
    """
    r = radius
    b, c, h, w = fmap1.shape
    d = 2 * r + 1
    outs = []
    f1 = fmap1.permute(0, 2, 3, 1).reshape(b, h * w, c)
    for lvl, f2 in enumerate(fmap_pyramid2):
        hl, wl = f2.shape[-2:]
        cen = coords.permute(0, 2, 3, 1).reshape(b, h * w, 2) / 2 ** lvl
        x0 = torch.floor(cen[..., 0])
        y0 = torch.floor(cen[..., 1])
        fx = (cen[..., 0] - x0)[..., None, None]
        fy = (cen[..., 1] - y0)[..., None, None]
        off = torch.arange(-r, r + 2, device=fmap1.device, dtype=torch.float32)
        # integer sample grid (b, hw, d+1 [x], d+1 [y])
        xs = x0[..., None, None] + off.view(1, 1, -1, 1)
        ys = y0[..., None, None] + off.view(1, 1, 1, -1)
        xs = xs.expand(b, h * w, d + 1, d + 1)
        ys = ys.expand(b, h * w, d + 1, d + 1)
        inb = (xs >= 0) & (xs <= wl - 1) & (ys >= 0) & (ys <= hl - 1)
        idx = (ys.clamp(0, hl - 1) * wl + xs.clamp(0, wl - 1)).long()
        f2f = f2.reshape(b, c, hl * wl).permute(0, 2, 1)  # b, hwl, c
        g = torch.gather(f2f, 1, idx.reshape(b, -1, 1).expand(-1, -1, c))
        g = g.view(b, h * w, d + 1, d + 1, c)
        dots = (g * f1[:, :, None, None, :]).sum(-1) * inb.to(g.dtype)
        # bilinear taps: tap (ix, iy) blends integer corners (ix,iy),(ix+1,iy),(ix,iy+1),(ix+1,iy+1)
        taps = ((1 - fx) * (1 - fy) * dots[:, :, :-1, :-1] + fx * (1 - fy) * dots[:, :, 1:, :-1]
                + (1 - fx) * fy * dots[:, :, :-1, 1:] + fx * fy * dots[:, :, 1:, 1:])
        outs.append(taps.reshape(b, h * w, d * d))
    out = torch.cat(outs, dim=-1) / math.sqrt(c)
    return out.permute(0, 2, 1).reshape(b, -1, h, w).contiguous()


def _use_hip(t, impl):
    if impl == 'torch':
        return False
    if not _ext.device_ok(t):
        return False
    return corr_ops.available(required=(impl == 'hip'))


class CorrBlock:
    """All-pairs correlation pyramid with a (2r+1)^2 window lookup per level."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, impl='auto', precision='fp32',
                 nhwc_lookup=False):
        """``nhwc_lookup``: every lookup goes through ``lookup_nhwc`` (the fused update block),
        so the pyramid may be stored in bf16 under mixed precision."""
        self.num_levels = num_levels
        self.radius = radius
        self.hip = _use_hip(fmap1, impl)
        if self.hip:
            # precision='bf16' (mixed precision): bf16 fmaps (the encoder outputs, exact in bf16)
            # go to the bf16-MFMA build as they are; the pyramid and lookups stay fp32 and the
            # backward GEMMs take a bf16 dcorr.  fp32 fmaps use the exact-f32 MFMA build.
            if precision == 'bf16' and fmap1.dtype == torch.bfloat16 and fmap1.shape[1] % 16 == 0:
                f1, f2 = fmap1, fmap2
            else:
                f1, f2 = fmap1.float().contiguous(), fmap2.float().contiguous()
            self.volume = corr_ops.AllPairsVolume(
                f1, f2, num_levels, bf16_backward=(precision == 'bf16'),
                bf16_pyramid=bool(nhwc_lookup) and precision == 'bf16')
            self.corr_pyramid = None
        else:
            self.corr_pyramid = torch_corr_pyramid(fmap1.float(), fmap2.float(), num_levels)

    def __call__(self, coords):
        if self.hip:
            return self.volume.lookup(coords, self.radius)
        return torch_corr_lookup(self.corr_pyramid, coords, self.radius)

    def lookup_nhwc(self, coords, cbuf, dtype=torch.bfloat16):
        """(B,H,W,cbuf) zero-padded taps for the fused HIP update block, in its operand dtype
        (bf16, or fp16 under fp16 autocast: written from the fp32 pyramid)."""
        if self.hip:
            return self.volume.lookup_nhwc(coords, self.radius, cbuf, dtype)
        return _to_nhwc_padded(self(coords), cbuf, dtype)

    @staticmethod
    def corr(fmap1, fmap2):
        return torch_corr_volume(fmap1, fmap2)


def _to_nhwc_padded(corr, cbuf, dtype=torch.bfloat16):
    x = corr.permute(0, 2, 3, 1).to(dtype)
    if cbuf > x.shape[-1]:
        x = F.pad(x, (0, cbuf - x.shape[-1]))
    return x.contiguous()


class AlternateCorrBlock:
    """On-the-fly correlation: O(HW * r^2) memory instead of O((HW)^2); differentiable."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, impl='auto', precision='fp32',
                 nhwc_lookup=False):
        """``nhwc_lookup``: every lookup goes through ``lookup_nhwc`` (the fused update block),
        so the pyramid may be stored in bf16 under mixed precision."""
        self.num_levels = num_levels
        self.radius = radius
        self.hip = _use_hip(fmap1, impl)
        # only the levels that are used are built (reference builds one extra, `core/corr.py:69`)
        self.fmap1 = fmap1.float()
        pyr = [fmap2.float()]
        for _ in range(num_levels - 1):
            pyr.append(F.avg_pool2d(pyr[-1], 2, stride=2))
        self.pyramid2 = pyr
        if self.hip:
            self.volume = corr_ops.OnTheFlyVolume(self.fmap1, self.pyramid2, precision)

    def __call__(self, coords):
        if self.hip:
            return self.volume.lookup(coords, self.radius)
        return torch_onthefly_corr(self.pyramid2, self.fmap1, coords, self.radius)

    def lookup_nhwc(self, coords, cbuf, dtype=torch.bfloat16):
        """(B,H,W,cbuf) zero-padded taps for the fused HIP update block (bf16 MFMA taps; fp16
        taps under fp16 autocast, written as fp16 by the fp32-accurate split forward; dtype fp32:
        split-fp32 [hi | lo] taps of the fp32 on-the-fly lookup)."""
        if dtype == torch.float32:
            from ..ops.update_hip import split_nhwc
            return split_nhwc(self(coords), cbuf)
        if self.hip:
            out = self.volume.lookup_nhwc(coords, self.radius, cbuf, dtype)
            return out if out.dtype == dtype else out.to(dtype)
        return _to_nhwc_padded(self(coords), cbuf, dtype)
