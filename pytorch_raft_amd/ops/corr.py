"""Autograd wrappers around the HIP correlation kernels.

Design (MI355X-first, see `SURVEY.md` §7.4 item 3):

* ``AllPairsVolume`` builds the 4-level all-pairs pyramid with ONE fused MFMA kernel
  (csrc/kernels/corr_allpairs.hip) instead of bmm + 3 avg_pool2d (`core/corr.py:19-27,52-60`).
* The pyramid is produced by an autograd node that outputs a 0-d *token*; every per-iteration
  lookup consumes that token.  Lookup backward accumulates straight into ONE pyramid-gradient buffer
  owned by the volume (race-free RMW, csrc/kernels/corr_lookup.hip) and returns an empty token grad.
  Autograd runs the build node's backward only after all lookups' backward, at which point a single
  pass folds the pyramid gradient (avg-pool adjoint, 1/sqrt(C)) and two GEMMs produce d(fmap1),
  d(fmap2).  The reference instead allocates + zero-fills a dense plane-sized gradient per level per
  iteration inside grid_sample backward and lets autograd add them up.
* ``OnTheFlyVolume`` is the differentiable counterpart of the reference's forward-only
  ``alt_cuda_corr`` (csrc/kernels/corr_onthefly.hip: 8x8 query tiles, MFMA tile-GEMM against the
  tile's fmap2 bounding box) with the same token scheme for d(fmap1), d(fmap2 levels).
"""
import math
import os

import torch
import torch.nn.functional as F

from . import _ext


# RAFT_CORR_BWD_GEMM=0: the feature-map gradients of the all-pairs correlation on torch.bmm
# (hipBLASLt) instead of the MFMA kernels of corr_bwd.hip (bf16, and the split-bf16 passes of the
# fp32 correlation) -- A/B and tests
_NATIVE_BWD_GEMM = os.environ.get('RAFT_CORR_BWD_GEMM', '1') != '0'


def available(required=False):
    return _ext.gpu_path_enabled(required=required)


class _State:
    """Mutable holder shared between the build node and its lookups."""

    def __init__(self):
        self.grad = None
        self.grad_f1 = None
        self.windows = []
        self.taps = []       # (coords, bf16 NHWC lookup-output gradient) per iteration
        self.taps_split = False  # the taps are split-fp32 [hi | lo] rows (the fp32 schedule)
        self.radius = None
        self.bf16_bwd = False
        self.pyr_bf16 = False  # bf16 pyramid: NHWC (bf16-output) lookups only


def _nhwc_bf16(f):
    """(B,C,H,W) bf16 (channels_last memory, as the encoders produce it) -> (B,H,W,C) contiguous."""
    return f.permute(0, 2, 3, 1).contiguous()


class _AllPairsBuild(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, levels, state):
        ops = _ext.ops()
        ctx.nhwc = fmap1.dtype == torch.bfloat16
        if ctx.nhwc:
            # mixed precision: bf16 MFMA straight from the NHWC encoder outputs (no fp32 copy);
            # a bf16 pyramid when only the NHWC lookup (fused update block, bf16 output) reads it
            f1, f2 = _nhwc_bf16(fmap1), _nhwc_bf16(fmap2)
            pyr = ops.corr_build_bf16(f1, f2, levels, bool(state.pyr_bf16))
            ctx.save_for_backward(f1, f2)
        else:
            pyr = ops.corr_build(fmap1, fmap2, levels)
            ctx.save_for_backward(fmap1, fmap2)
        state.pyramid = pyr
        ctx.state = state
        ctx.shape = tuple(fmap1.shape)
        token = fmap1.new_zeros((), dtype=torch.float32)
        return token

    @staticmethod
    def backward(ctx, _dtoken):
        st = ctx.state
        fmap1, fmap2 = ctx.saved_tensors
        if st.grad is None and not st.taps:
            return None, None, None, None
        b, c, h, w = ctx.shape
        dcorr = None
        # mixed precision, tap path only: dcorr in bf16 and bf16 GEMMs (fp32 accumulation); the
        # fmaps are bf16 encoder outputs, so only the dcorr rounding differs from fp32
        bf16 = (st.bf16_bwd or ctx.nhwc) and st.grad is None and bool(st.taps)
        if st.grad is not None:
            dcorr = _ext.ops().corr_pyr_grad_reduce(st.grad, 1.0 / math.sqrt(c))  # (B, N, N)
        # mixed precision, tap path only: the fold writes dC with rows padded to 64 columns and
        # the two feature-map GEMMs run on the hand-written MFMA kernel (corr_bwd.hip)
        native_gemm = (ctx.nhwc and bf16 and dcorr is None and bool(st.taps) and c % 128 == 0
                       and _NATIVE_BWD_GEMM)
        # fp32 correlation (fp16 / fp32 schedules), tap path only: the fold writes dC as its
        # split-bf16 planes and the two GEMMs run as three-pass split MFMA kernels (fp32 output)
        split_gemm = (not ctx.nhwc and not bf16 and dcorr is None and bool(st.taps)
                      and c % 128 == 0 and _NATIVE_BWD_GEMM)
        if st.taps:
            dt = _ext.ops().corr_tap_reduce([x[0] for x in st.taps], [x[1] for x in st.taps],
                                            h, w, len(st.pyramid), st.radius, 1.0 / math.sqrt(c),
                                            bf16, 64 if (native_gemm or split_gemm) else 0,
                                            st.taps_split, split_gemm)
            dcorr = dt if dcorr is None else dcorr + dt
        st.grad = None
        st.taps = []
        st.pyramid = None
        if native_gemm:
            g1, g2 = _ext.ops().corr_bwd_fmaps(dcorr, fmap1, fmap2)
            return g1.permute(0, 3, 1, 2), g2.permute(0, 3, 1, 2), None, None
        if split_gemm:
            # fp32 (B, H, W, C) gradients, returned as channels_last-strided (B, C, H, W) views
            g1, g2 = _ext.ops().corr_bwd_fmaps_split(dcorr, fmap1, fmap2)
            return g1.permute(0, 3, 1, 2), g2.permute(0, 3, 1, 2), None, None
        if ctx.nhwc:
            # (B,N,C) operands: dF1 = dC F2, dF2 = dC^T F1 -> NHWC results, returned as
            # channels_last (B,C,H,W) bf16 like the encoder outputs they flow back into
            dcorr = dcorr.to(torch.bfloat16)
            f1n = fmap1.view(b, h * w, c)
            f2n = fmap2.view(b, h * w, c)
            g1 = torch.bmm(dcorr, f2n).view(b, h, w, c).permute(0, 3, 1, 2)
            g2 = torch.bmm(dcorr.transpose(1, 2), f1n).view(b, h, w, c).permute(0, 3, 1, 2)
            return g1, g2, None, None
        f1 = fmap1.view(b, c, h * w)
        f2 = fmap2.view(b, c, h * w)
        if bf16:
            f1 = f1.to(torch.bfloat16)
            f2 = f2.to(torch.bfloat16)
        # dF1 = F2 dC^T, dF2 = F1 dC  (library GEMMs)
        g1 = torch.bmm(f2, dcorr.transpose(1, 2)).view(b, c, h, w)
        g2 = torch.bmm(f1, dcorr).view(b, c, h, w)
        return g1.float(), g2.float(), None, None


class _AllPairsLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, radius, state):
        out = _ext.ops().corr_lookup_fwd(state.pyramid, coords, radius)
        ctx.state = state
        ctx.radius = radius
        ctx.save_for_backward(coords)
        return out

    @staticmethod
    def backward(ctx, dout):
        st = ctx.state
        (coords,) = ctx.saved_tensors
        if st.grad is None:
            st.grad = [torch.zeros_like(p) for p in st.pyramid]
        _ext.ops().corr_lookup_bwd_(st.grad, coords, dout.contiguous().float(), ctx.radius)
        return None, None, None, None


class _AllPairsLookupNHWC(torch.autograd.Function):
    """Lookup writing bf16 taps into a zero-padded NHWC (B,H,W,cbuf) buffer: the direct input of
    the fused update block's first 1x1 conv (no NCHW->NHWC transpose, no fp32->bf16 cast kernel)."""

    @staticmethod
    def forward(ctx, token, coords, radius, state, cbuf, dtype=torch.bfloat16):
        b, _, h, w = coords.shape
        # the tile kernel writes every channel of each pixel row, padding included; fp16 taps
        # (fp16 autocast) come from an fp32 pyramid; dtype fp32 (the fp32 schedule): split
        # [hi | lo] bf16 taps, 2 cbuf channels (ops/update_hip.py's split-fp32 operands)
        spl = dtype == torch.float32
        out = torch.empty(b, h, w, 2 * cbuf if spl else cbuf, device=coords.device,
                          dtype=torch.bfloat16 if spl else dtype)
        _ext.ops().corr_lookup_nhwc_(state.pyramid, coords, radius, out, spl)
        ctx.state = state
        ctx.radius = radius
        ctx.spl = spl
        ctx.save_for_backward(coords)
        return out

    @staticmethod
    def backward(ctx, dout):
        st = ctx.state
        (coords,) = ctx.saved_tensors
        b, _, h, w = coords.shape
        levels = len(st.pyramid)
        spl = ctx.spl
        # split taps enter the fold twice (hi and lo rows): at most 16 iterations per fold
        if (_window_reduce_fits(h, w, levels) and len(st.taps) < (16 if spl else 32)
                and dout.shape[-1] % 8 == 0 and (not st.taps or st.taps_split == spl)
                and (not spl or dout.dtype == torch.bfloat16)):
            # keep the iteration's 16-bit tap gradient (bf16, or fp16 under fp16 autocast); all
            # iterations are folded into dcorr once per step straight from these rows
            # (corr_tap_reduce)
            td = dout.dtype if dout.dtype in (torch.bfloat16, torch.float16) else torch.bfloat16
            st.taps.append((coords, dout.to(td).contiguous()))
            st.taps_split = spl
            st.radius = ctx.radius
        else:
            if st.grad is None:
                st.grad = [torch.zeros_like(p) for p in st.pyramid]
            if spl:   # split-encoded fp32 tap gradient
                c = dout.shape[-1] // 2
                dout = dout[..., :c].float() + dout[..., c:].float()
            _ext.ops().corr_lookup_bwd_(st.grad, coords, dout.float().contiguous(), ctx.radius)
        return None, None, None, None, None, None


def _window_reduce_fits(h, w, levels):
    tot, hh, ww = 0, h, w
    for _ in range(levels):
        tot += hh * ww
        hh, ww = hh // 2, ww // 2
    return tot * 4 <= 64 * 1024


class AllPairsVolume:
    def __init__(self, fmap1, fmap2, num_levels=4, bf16_backward=False, bf16_pyramid=False):
        self.state = _State()
        self.state.bf16_bwd = bool(bf16_backward)
        # the window lookup writes bf16 taps anyway: a bf16 pyramid halves the bytes its
        # per-iteration gathers pull (~0.5 GB fp32 volume at chairs / batch 12)
        self.state.pyr_bf16 = bool(bf16_pyramid) and fmap1.dtype == torch.bfloat16
        self.levels = num_levels
        # bf16 encoder outputs are channels_last: kept as they are, so _nhwc_bf16's permute is
        # already contiguous (a plain .contiguous() here made an NCHW copy that _nhwc_bf16 then
        # permuted back: two full copies of each fmap per step)
        if fmap1.dtype == torch.bfloat16:
            fmap1 = fmap1.contiguous(memory_format=torch.channels_last)
            fmap2 = fmap2.contiguous(memory_format=torch.channels_last)
        else:
            fmap1, fmap2 = fmap1.contiguous(), fmap2.contiguous()
        self.token = _AllPairsBuild.apply(fmap1, fmap2, num_levels, self.state)

    @property
    def pyramid(self):
        return self.state.pyramid

    def lookup(self, coords, radius):
        if self.state.pyr_bf16:
            raise RuntimeError('bf16 pyramid: only the NHWC lookup (lookup_nhwc) reads it')
        return _AllPairsLookup.apply(self.token, coords.contiguous().float(), radius, self.state)

    def lookup_nhwc(self, coords, radius, cbuf, dtype=torch.bfloat16):
        """(B,H,W,cbuf) taps in ``dtype`` (bf16 / fp16); dtype fp32: split-fp32 [hi | lo] bf16
        taps (B,H,W,2 cbuf) from the fp32 pyramid."""
        if dtype != torch.bfloat16 and self.state.pyr_bf16:
            raise RuntimeError('bf16 pyramid: the NHWC lookup writes bf16 taps')
        return _AllPairsLookupNHWC.apply(self.token, coords.contiguous().float(), radius, self.state,
                                         cbuf, dtype)


def _pool_nhwc(x):
    # avg-pool 2x2 (floor) on an NHWC tensor via the NCHW view, returned NHWC-contiguous
    return F.avg_pool2d(x.permute(0, 3, 1, 2), 2, stride=2).permute(0, 2, 3, 1).contiguous()


class _OTFBuild(torch.autograd.Function):
    """fmap1 (B,C,H,W), pyramid of fmap2 (list) -> token; keeps NHWC bf16 MFMA operands in
    ``state`` (converted once per step, not per lookup as `core/corr.py:82-83` does)."""

    @staticmethod
    def forward(ctx, fmap1, *args):
        state = args[-1]
        f2_levels = args[:-1]
        f1 = fmap1.permute(0, 2, 3, 1)
        f2 = [f.permute(0, 2, 3, 1) for f in f2_levels]
        state.f1 = f1.to(torch.bfloat16).contiguous()
        state.f2 = [f.to(torch.bfloat16).contiguous() for f in f2]
        state.lo = []
        if state.precision == 'fp32':
            # x = hi + lo with both parts bf16: the kernel's 3-MFMA split product is fp32-accurate
            state.lo = [(f1 - state.f1.float()).to(torch.bfloat16).contiguous()]
            state.lo += [(f - h.float()).to(torch.bfloat16).contiguous() for f, h in zip(f2, state.f2)]
        ctx.state = state
        ctx.nlev = len(f2_levels)
        return fmap1.new_zeros(())

    @staticmethod
    def backward(ctx, _dtoken):
        st = ctx.state
        if st.windows:
            _otf_alloc_grads(st)
            _ext.ops().corr_otf_window_bwd_(st.f1, st.f2, [w[0] for w in st.windows],
                                            [w[1] for w in st.windows], st.grad_f1, st.grad,
                                            st.radius)
            st.windows = []
        if st.grad is None:
            return (None,) * (ctx.nlev + 2)
        g1 = st.grad_f1.permute(0, 3, 1, 2)
        g2 = [g.permute(0, 3, 1, 2) for g in st.grad]
        st.grad = st.grad_f1 = None
        st.f1 = st.f2 = st.lo = None
        return (g1, *g2, None)


def _otf_alloc_grads(st):
    if st.grad is None:
        st.grad = [torch.zeros(f.shape, device=f.device, dtype=torch.float32) for f in st.f2]
        st.grad_f1 = torch.zeros(st.f1.shape, device=st.f1.device, dtype=torch.float32)


def _otf_backward(st, coords, dout, radius):
    _otf_alloc_grads(st)
    if dout.dtype not in (torch.float32, torch.bfloat16):
        dout = dout.float()
    dout = dout.contiguous()
    ops = _ext.ops()
    ops.corr_otf_bwd_(st.f1, st.f2, coords, dout, st.grad_f1, st.grad, radius)
    if st.precision == 'fp32' and st.lo:
        # fp32-accurate backward (the reference's alt_cuda_corr backward is fp32): with the window
        # gradient dS = dS_hi + dS_lo and F = F_hi + F_lo (bf16 parts), dF1 = dS F2 and
        # dF2 = dS^T F1 are the three bf16 products hi*hi (above) + lo(dS)*hi + hi*lo(F), each a
        # pass of the same MFMA kernel accumulating into the gradients (~2^-16 relative; the
        # dropped lo*lo term is ~2^-18)
        ops.corr_otf_bwd_(st.f1, st.f2, coords, dout, st.grad_f1, st.grad, radius, 1)
        ops.corr_otf_bwd_(st.lo[0], st.lo[1:], coords, dout, st.grad_f1, st.grad, radius)


class _OTFLookup(torch.autograd.Function):
    @staticmethod
    def forward(ctx, token, coords, radius, state):
        b, _, h, w = coords.shape
        nc = len(state.f2) * (2 * radius + 1) ** 2
        out = torch.empty(b, h, w, nc, device=coords.device, dtype=torch.float32)
        _ext.ops().corr_otf_fwd_(state.f1, state.f2, coords, radius, out, state.lo)
        ctx.state = state
        ctx.radius = radius
        ctx.save_for_backward(coords)
        return out.permute(0, 3, 1, 2)  # NCHW-shaped, channels_last strides

    @staticmethod
    def backward(ctx, dout):
        (coords,) = ctx.saved_tensors
        _otf_backward(ctx.state, coords, dout.float().permute(0, 2, 3, 1), ctx.radius)
        return None, None, None, None


class _OTFLookupNHWC(torch.autograd.Function):
    """bf16 taps straight into the zero-padded (B,H,W,cbuf) input of the fused update block; fp16
    taps (fp16 autocast) from the fp32-accurate split forward, stored as fp16 by the kernel."""

    @staticmethod
    def forward(ctx, token, coords, radius, state, cbuf, dtype=torch.bfloat16):
        b, _, h, w = coords.shape
        dt = torch.float16 if (dtype == torch.float16 and state.lo) else torch.bfloat16
        out = torch.empty(b, h, w, cbuf, device=coords.device, dtype=dt)
        _ext.ops().corr_otf_fwd_(state.f1, state.f2, coords, radius, out, state.lo)
        ctx.state = state
        ctx.radius = radius
        ctx.save_for_backward(coords)
        return out

    @staticmethod
    def backward(ctx, dout):
        st = ctx.state
        (coords,) = ctx.saved_tensors
        if len(st.windows) < 32 and dout.shape[-1] % 8 == 0:
            # the iteration's bf16 tap gradient is kept; the MFMA box GEMMs + dF2 atomics then run
            # ONCE per step over all iterations (build node backward) instead of once per
            # iteration, forming each pixel's window gradients from the taps in LDS
            # (fp16 tap gradients are rounded to bf16 here: the backward's MFMA operand type)
            st.windows.append((coords, dout.to(torch.bfloat16).contiguous()))
            st.radius = ctx.radius
        else:
            _otf_backward(st, coords, dout, ctx.radius)
        return None, None, None, None, None, None


class OnTheFlyVolume:
    """precision: 'bf16' (MFMA operands bf16, fp32 accumulation) or 'fp32' (split-bf16 forward
    AND backward, ~2^-16 relative error: three bf16 products per product, fp32 accumulation)."""

    def __init__(self, fmap1, fmap2_pyramid, precision='fp32'):
        assert precision in ('bf16', 'fp32'), precision
        self.state = _State()
        self.state.precision = precision
        self.token = _OTFBuild.apply(fmap1.contiguous(), *fmap2_pyramid, self.state)

    def lookup(self, coords, radius):
        return _OTFLookup.apply(self.token, coords.contiguous().float(), radius, self.state)

    def lookup_nhwc(self, coords, radius, cbuf, dtype=torch.bfloat16):
        return _OTFLookupNHWC.apply(self.token, coords.contiguous().float(), radius, self.state,
                                    cbuf, dtype)
