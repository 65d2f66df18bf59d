"""fp32 convolutions (update block + stride-1 encoder convs) on the bf16 MFMA kernels (split-bf16,
3 products).

The reference's paper schedule trains in fp32 (`train_standard.sh`, no `--mixed_precision`):
every update-block conv (`core/update.py`) is then an fp32 NCHW conv.  gfx950's matrix cores
have no fast fp32 path (the fp32 MFMA rate is 1/8 of bf16), so an fp32 operand is carried as
an exact-to-2^-16 pair ``x = x_hi + x_lo`` of bf16 values and the conv as three bf16 products

    conv(x, w) ~= conv(x_hi, w_hi) + conv(x_lo, w_hi) + conv(x_hi, w_lo)      (fp32 accumulation)

(the dropped ``x_lo * w_lo`` term and the bf16 rounding of the residuals are ~2^-16 relative,
the same scheme the fp32 correlation kernels use).  The three products are ONE launch of the
implicit-GEMM conv kernel: the input buffer is NHWC ``[x_hi | x_lo]`` (each half padded to a
multiple of 64 channels), read as the virtual concat ``[x_hi, x_lo, x_hi]`` against packed
weights ``[w_hi, w_hi, w_lo]``.  The input gradient is the same construction on the split
output gradient and the flipped / transposed weights; the weight gradient is two launches of the
weight-gradient kernel (``g_hi x [x_hi | x_lo]`` and ``g_lo x x_hi``).

Used by :class:`pytorch_raft_amd.models.update.MfmaConv2d` (every update-block conv; convf1's 2
input channels ride in a 64-channel slot) while an fp32 model runs on a GPU, so the decode of an
fp32 step has no MIOpen call left and is captured in the training hipGraph like the bf16 one;
bf16 autocast takes the fused update block.
"""
import contextlib
import os

import torch

from . import _ext
from . import conv as C

_ACTIVE = {'on': False}
# RAFT_FP32_MFMA=0: fp32 models keep MIOpen fp32 convs in the update block (A/B measurements)
_ENV_ON = os.environ.get('RAFT_FP32_MFMA', '1') != '0'


# packed [w_hi | w_hi | w_lo] weights of the current decode (forward and adjoint), keyed by the
# parameter storage and version: the 12 iterations share them.  One dict per decode
# (``enabled()`` scope), referenced by that decode's autograd nodes: it lives until their
# backward has run and the graph is freed, never across decodes (no stale pack can be served
# to a later tensor that reuses a freed weight's storage).


@contextlib.contextmanager
def enabled(on=True):
    """Route MfmaConv2d modules through the split-bf16 MFMA conv inside the block (one decode)."""
    prev = _ACTIVE['on'], _ACTIVE.get('packed'), _ACTIVE.get('mods')
    _ACTIVE['on'] = bool(on)
    _ACTIVE['packed'] = {}
    _ACTIVE['mods'] = {}   # module -> _ModState of this decode (weight token, deferred wgrad)
    try:
        yield
    finally:
        _ACTIVE['on'], _ACTIVE['packed'], _ACTIVE['mods'] = prev


def active_for(x, weight):
    return (_ACTIVE['on'] and _ENV_ON and x.is_cuda and x.dtype == torch.float32 and
            weight.dtype == torch.float32 and x.dim() == 4 and not torch.is_autocast_enabled())


def fits(x, cout):
    """The split operands ([hi | lo] bf16 NHWC, 2 x the 64-padded channels) and the fp32 output
    stay inside the kernels' 32-bit buffer-descriptor range; larger calls keep MIOpen."""
    b, cin, h, w = x.shape
    pix = b * h * w
    return (pix * 4 * max(C.round_up(cin, 64), C.round_up(cout, 64)) < 2 ** 31 and
            pix * 4 * cout < 2 ** 31)


def _split_nhwc_torch(x, cpad):
    """Reference formulation of :func:`_split_nhwc` (CPU tensors; the kernel's oracle)."""
    b, c, h, w = x.shape
    xn = x.permute(0, 2, 3, 1)
    hi = xn.to(torch.bfloat16)
    buf = torch.zeros(b, h, w, 2 * cpad, device=x.device, dtype=torch.bfloat16)
    buf[..., :c] = hi
    buf[..., cpad:cpad + c] = (xn - hi.float()).to(torch.bfloat16)
    return buf


def _split_nhwc(x, cpad):
    """(B, C, H, W) fp32 (any strides) -> (B, H, W, 2 cpad) bf16 [hi | lo] (zero padded): on the
    GPU ONE pass of the split_hilo kernel (LDS-tiled transpose when x is NCHW)."""
    if not x.is_cuda:
        return _split_nhwc_torch(x, cpad)
    b, c, h, w = x.shape
    buf = torch.empty(b, h, w, 2 * cpad, device=x.device, dtype=torch.bfloat16)
    _ext.ops().split_hilo_(x, buf)
    return buf


# Split operands handed over by their producers (the encoders' fp32 norm kernels write a conv's
# input, or a conv output's gradient, also as the [hi | lo] pair): tensor -> split buffer, taken
# once by the consuming split conv.  An entry holds its tensor, so no other tensor can reuse its
# storage while it waits (matching by storage address, layout and version is then exact).  Each
# encoder pass starts by clearing it (encoder.py:_encoder_body): an encoder pass on another
# thread can only make a consumer fall back to its own split_hilo pass, never hand it a wrong
# operand.
_HANDOFF = {}


def _hkey(t):
    return (t.data_ptr(), t.device.index, tuple(t.shape), tuple(t.stride()))


def offer_split(t, buf):
    _HANDOFF[_hkey(t)] = (t, t._version, buf)


def clear_handoff():
    _HANDOFF.clear()


def _take_split(t, cpad):
    """The split pair of ``t`` offered by its producer, else one split_hilo pass."""
    e = _HANDOFF.pop(_hkey(t), None) if _HANDOFF else None
    if e is not None and e[1] == t._version and e[2].shape[-1] == 2 * cpad:
        return e[2]
    return _split_nhwc(t, cpad)


def _pack3(w, cpad):
    """(Cout, Cin, kh, kw) fp32 -> packed [w_hi | w_hi | w_lo] over three cpad-wide segments."""
    cin = w.shape[1]
    wh = w.to(torch.bfloat16).float()
    w3 = torch.cat([wh, wh, w - wh], dim=1)
    return C.pack_weight(w3, [cin] * 3, [cpad] * 3)


def _wgrad(gs, g_off, xs, offs, cnts, k, pad, cout, dw):
    """dw += weight gradient: the tap-fused kernel (the fused block's) where it applies (1x1,
    3x3, 1x5, 5x1), the tile kernel otherwise (convf1's 7x7)."""
    if C._taps_ok(offs, cnts, k):
        C.conv_wgrad_multi([(gs, [xs] * len(offs))], g_off, offs, cnts, k, pad, cout, dw)
    else:
        C.conv_wgrad(gs, g_off, [(xs, o, c) for o, c in zip(offs, cnts)], k, pad, cout, dw)


def _packed(cache, weight, cpad, adjoint):
    key = (weight.data_ptr(), weight._version, tuple(weight.shape), cpad, adjoint)
    w = cache.get(key)
    if w is None:
        src = weight.detach()
        if adjoint:
            src = src.flip(2, 3).transpose(0, 1).contiguous()   # (Cin, Cout, kh, kw)
        w = cache[key] = _pack3(src, cpad)
    return w


_PREPACK_PLANS = {}


def _prepack_plan(shapes):
    """Gather codes of every split-packed weight ([w_hi | w_hi | w_lo] per tap, forward and
    adjoint, as _pack3 lays them out) of convs with ``shapes``: built once per geometry by running
    the packing on element-id tensors (float64 ids, 0 = zero padding); ids past the weights'
    total are the same elements' residual halves (gather sources n..2n-1)."""
    if shapes in _PREPACK_PLANS:
        return _PREPACK_PLANS[shapes]
    numels = [co * ci * kh * kw for co, ci, kh, kw in shapes]
    total = sum(numels)
    parts, views, off = [], [], 0
    for (co, ci, kh, kw), n in zip(shapes, numels):
        ids = torch.arange(n, dtype=torch.float64).view(co, ci, kh, kw) + off + 1
        off += n
        for adjoint in (False, True):
            src = ids.flip(2, 3).transpose(0, 1) if adjoint else ids
            seg = src.shape[1]
            cpad = C.round_up(seg, 64)
            w3 = torch.cat([src, src, src + total], dim=1)   # [hi | hi | lo]
            t = C.pack_weight(w3, [seg] * 3, [cpad] * 3, dtype=torch.float64)
            views.append((adjoint, cpad, tuple(t.shape)))
            parts.append(t.reshape(-1))
    e = torch.cat(parts).round().long() - 1
    e[e < 0] = 2 * total                                    # zero padding -> the zero slot
    plan = (C.gather_index(e, numels + numels), views)
    _PREPACK_PLANS[shapes] = plan
    return plan


def prepack(pairs):
    """Split-pack the weights of several fp32 convs in ONE gather launch into the current scope's
    pack cache (what :func:`_packed` would build per conv with ~10 small kernels, forward and
    adjoint).  ``pairs`` = [(weight as the convs will see it, fp32 contiguous source of the
    same values)]; at most GATHER_MAX / 2 convs per launch."""
    cache = _ACTIVE.get('packed')
    if cache is None or not pairs:
        return
    half = C.GATHER_MAX // 2
    for i in range(0, len(pairs), half):
        chunk = pairs[i:i + half]
        shapes = tuple(tuple(w.shape) for w, _ in chunk)
        dev = chunk[0][1].device
        code, views = _prepack_plan(shapes)
        if code.device != dev:
            code = code.to(dev)
            _PREPACK_PLANS[shapes] = (code, views)
        srcs = [src for _, src in chunk]
        out = torch.empty(code.numel(), device=dev, dtype=torch.bfloat16)
        C.gather_cast(srcs + srcs, code, out, lo_from=len(srcs))
        off = 0
        for j, (adjoint, cpad, shape) in enumerate(views):
            w = chunk[j // 2][0]
            n = shape[0] * shape[1]
            cache[(w.data_ptr(), w._version, tuple(w.shape), cpad, adjoint)] = out[off:off + n].view(shape)
            off += n


class _ModState:
    """One MfmaConv2d module within one decode: its detached parameters, their split packs, and
    the (split output gradient, split input) pairs of every call, whose weight / bias gradients
    are computed in ONE batched launch pair when the module's token node runs (after the last
    call's backward) instead of per iteration."""

    def __init__(self, weight, bias, pad, cache):
        self.weight = weight.detach()
        self.bias = None if bias is None else bias.detach()
        self.pad = pad
        self.cache = cache
        self.items = []
        self.tok = None


class _WeightSink(torch.autograd.Function):
    """Token standing for a module's weight and bias in the decode: every call takes it as input
    (returning no gradient for it), so its backward runs once, after all of them."""

    @staticmethod
    def forward(ctx, st, weight, bias):
        ctx.st = st
        ctx.has_bias = bias is not None
        return weight.new_zeros(())

    @staticmethod
    def backward(ctx, _g):
        st = ctx.st
        dw, db = _flush_wgrad(st)
        st.items = []
        return None, dw, (db if ctx.has_bias else None)


def _flush_wgrad(st):
    cout, cin, kh, kw = st.weight.shape
    dev = st.weight.device
    if not st.items:
        return torch.zeros_like(st.weight), torch.zeros(cout, device=dev)
    k = kh * kw
    cp = st.items[0][1].shape[-1] // 2
    cop = st.items[0][0].shape[-1] // 2
    d1 = torch.zeros(cout, k * 2 * cp, device=dev)    # g_hi x [x_hi | x_lo]
    d2 = torch.zeros(cout, k * cp, device=dev)        # g_lo x x_hi
    db = torch.zeros(cout, device=dev)                # sum(g_hi) + sum(g_lo)
    if C._taps_ok([0, cp], [cp, cp], (kh, kw)):
        for i in range(0, len(st.items), C.MAX_WG_ITEMS):
            chunk = st.items[i:i + C.MAX_WG_ITEMS]
            C.conv_wgrad_multi([(gs, [xs, xs]) for gs, xs in chunk], 0, [0, cp], [cp, cp], (kh, kw),
                               st.pad, cout, d1, db)
            C.conv_wgrad_multi([(gs, [xs]) for gs, xs in chunk], cop, [0], [cp], (kh, kw), st.pad,
                               cout, d2, db)
    else:  # convf1's 7x7 over a 64-channel slot: the tile kernel, per item
        for gs, xs in st.items:
            C.conv_wgrad(gs, 0, [(xs, 0, cp), (xs, cp, cp)], (kh, kw), st.pad, cout, d1, db)
            C.conv_wgrad(gs, cop, [(xs, 0, cp)], (kh, kw), st.pad, cout, d2, db)
    g1 = C.unpack_weight_grad(d1, cout, [cin, cin], [cp, cp], (kh, kw))
    dw = g1[:, :cin] + g1[:, cin:] + C.unpack_weight_grad(d2, cout, [cin], [cp], (kh, kw))
    return dw, db


def _split_conv_fwd(x, weight, bias, pad, cache):
    b, cin, h, w = x.shape
    cout, _, kh, kw = weight.shape
    cp = C.round_up(cin, 64)
    xs = _split_nhwc(x, cp)
    # NHWC fp32 output (row-contiguous epilogue stores), handed on as a channels_last tensor: the
    # next conv's split then reads it channel-contiguous
    out = torch.empty(b, cout, h, w, device=x.device, dtype=torch.float32,
                      memory_format=torch.channels_last)
    C.conv_fwd([(xs, 0, cp), (xs, cp, cp), (xs, 0, cp)], _packed(cache, weight, cp, False),
               None if bias is None else bias.contiguous(), (kh, kw), pad, cout,
               C.EPI_F32, [out.permute(0, 2, 3, 1)], [0])
    return out, xs


class _SplitConvTok(torch.autograd.Function):
    """Split-bf16 conv of one call: forward, input gradient here; the weight / bias gradient is
    deferred to the module's token node (_WeightSink)."""

    @staticmethod
    def forward(ctx, x, tok, st):
        out, xs = _split_conv_fwd(x, st.weight, st.bias, st.pad, st.cache)
        ctx.save_for_backward(xs)
        ctx.st = st
        ctx.cin = x.shape[1]
        return out   # not a view: the update block applies in-place ReLUs to it

    @staticmethod
    def backward(ctx, g):
        (xs,) = ctx.saved_tensors
        st = ctx.st
        b, cout, h, w = g.shape
        cin = ctx.cin
        _, _, kh, kw = st.weight.shape
        cop = C.round_up(cout, 64)
        gs = _split_nhwc(g, cop)
        st.items.append((gs, xs))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(b, cin, h, w, device=g.device, dtype=torch.float32,
                             memory_format=torch.channels_last)
            C.conv_fwd([(gs, 0, cop), (gs, cop, cop), (gs, 0, cop)], _packed(st.cache, st.weight, cop, True),
                       None, (kh, kw), st.pad, cin, C.EPI_F32, [dx.permute(0, 2, 3, 1)], [0])
        return dx, None, None


def module_conv2d(mod, x):
    """MfmaConv2d forward while the split path is active: per decode, a module's calls share one
    weight token (batched weight gradients) and its packed split weights."""
    _ext.gpu_path_enabled(required=True)
    pad = tuple(int(p) for p in mod.padding)
    cache = _ACTIVE.get('packed')
    cache = {} if cache is None else cache
    need_w = mod.weight.requires_grad or (mod.bias is not None and mod.bias.requires_grad)
    if not (torch.is_grad_enabled() and (need_w or x.requires_grad)):
        return _split_conv_fwd(x, mod.weight.detach(), None if mod.bias is None else mod.bias.detach(),
                               pad, cache)[0]
    mods = _ACTIVE.get('mods')
    if mods is None:   # outside an enabled() scope (tests): a token per call
        mods = {}
    st = mods.get(id(mod))
    if st is None:
        st = mods[id(mod)] = _ModState(mod.weight, mod.bias, pad, cache)
        st.tok = _WeightSink.apply(st, mod.weight, mod.bias)
    return _SplitConvTok.apply(x, st.tok, st)


class _SplitConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, pad):
        b, cin, h, w = x.shape
        cout, _, kh, kw = weight.shape
        cp = C.round_up(cin, 64)
        xs = _take_split(x, cp)
        # NHWC fp32 output (row-contiguous epilogue stores), handed on as a channels_last tensor:
        # the next conv's split then reads it channel-contiguous
        out = torch.empty(b, cout, h, w, device=x.device, dtype=torch.float32,
                          memory_format=torch.channels_last)
        cache = _ACTIVE.get('packed')
        cache = {} if cache is None else cache
        ctx.packed = cache
        C.conv_fwd([(xs, 0, cp), (xs, cp, cp), (xs, 0, cp)], _packed(cache, weight, cp, False),
                   None if bias is None else bias.contiguous(), (kh, kw), pad, cout,
                   C.EPI_F32, [out.permute(0, 2, 3, 1)], [0])
        ctx.save_for_backward(xs, weight)
        ctx.pad, ctx.cin, ctx.has_bias = pad, cin, bias is not None
        return out   # not a view: the update block applies in-place ReLUs to it

    @staticmethod
    def backward(ctx, g):
        xs, weight = ctx.saved_tensors
        b, cout, h, w = g.shape
        cin, pad = ctx.cin, ctx.pad
        _, _, kh, kw = weight.shape
        cp = xs.shape[-1] // 2
        cop = C.round_up(cout, 64)
        gs = _take_split(g, cop)
        dx = dw = db = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(b, cin, h, w, device=g.device, dtype=torch.float32,
                             memory_format=torch.channels_last)
            C.conv_fwd([(gs, 0, cop), (gs, cop, cop), (gs, 0, cop)], _packed(ctx.packed, weight, cop, True), None,
                       (kh, kw), pad, cin, C.EPI_F32, [dx.permute(0, 2, 3, 1)], [0])
        if ctx.needs_input_grad[1] and C._taps_ok([0], [cp], (kh, kw)):
            # ONE tap-fused launch of the three products g_hi x_hi + g_lo x_hi + g_hi x_lo
            # (split=True, the fused decode's split weight gradient)
            dwp = torch.zeros(cout, kh * kw * cp, device=g.device)
            C.conv_wgrad_multi([(gs, [xs])], 0, [0], [cp], (kh, kw), pad, cout, dwp, None, split=True)
            dw = C.unpack_weight_grad(dwp, cout, [cin], [cp], (kh, kw))
        elif ctx.needs_input_grad[1]:
            k = kh * kw
            d1 = torch.zeros(cout, k * 2 * cp, device=g.device)    # g_hi x [x_hi | x_lo]
            _wgrad(gs, 0, xs, [0, cp], [cp, cp], (kh, kw), pad, cout, d1)
            d2 = torch.zeros(cout, k * cp, device=g.device)        # g_lo x x_hi
            _wgrad(gs, cop, xs, [0], [cp], (kh, kw), pad, cout, d2)
            g1 = C.unpack_weight_grad(d1, cout, [cin, cin], [cp, cp], (kh, kw))
            dw = g1[:, :cin] + g1[:, cin:] + C.unpack_weight_grad(d2, cout, [cin], [cp], (kh, kw))
        if ctx.has_bias and ctx.needs_input_grad[2]:
            # the fp32 gradient's exact sum (the encoders fold their conv biases into the norms:
            # only bias-carrying calls pay this reduce)
            db = g.sum((0, 2, 3))
        return dx, dw, db, None


def conv2d(x, weight, bias, padding):
    """fp32 conv2d (stride 1, 'same'-style padding) on the split-bf16 MFMA kernels."""
    _ext.gpu_path_enabled(required=True)
    return _SplitConv.apply(x, weight, bias, tuple(int(p) for p in padding))
