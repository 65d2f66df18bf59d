"""Channels-last bf16 fast path of the RAFT encoders (fnet / cnet) on MI355X.

Reference: `core/extractor.py:6-56` (ResidualBlock), `:60-116` (BottleneckBlock), `:118-267`
(BasicEncoder / SmallEncoder forward).  Module tree, parameters and buffers are the nn.Module ones
(checkpoint layout untouched); only the execution differs:

* convolutions run as MIOpen NHWC bf16 convs (channels_last activations and weights -- no
  NCHW<->NHWC transposes) WITHOUT their bias; the bias is folded into the following norm
  (csrc/kernels/encoder_norm.hip), where it cancels for training-mode statistics and shifts the
  eval-mode (frozen) BatchNorm.  Its gradient is computed exactly from the norm's backward sums;
* every norm + ReLU is one autograd node with a hand-written forward (stats, finalize, apply) and
  backward (sums, finalize, apply), replacing InstanceNorm-as-batch_norm, clamp, add and the
  per-conv bias-gradient reductions of the eager graph;
* the residual add + ReLU is one node.

Used automatically by ``_Encoder.forward`` on the GPU under bf16 or fp16 autocast
(``fast_path_ok``; the reference's ``--mixed_precision`` is fp16 autocast, `core/raft.py:99`):
activations, weights and weight gradients are in the autocast dtype, statistics and accumulation
in fp32.  An fp32 model (the reference's default schedule) takes the same path in fp32 -- the
stride-1 convs as split-bf16 MFMA convs (ops/conv_fp32.py), the strided ones on MIOpen fp32, the
norm / ReLU / residual nodes on the fp32 instantiations of the same kernels -- instead of the
eager NCHW modules (ATen instance norm on channels_last tensors, separate ReLU / add kernels).
"""
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _ext

MODE_INSTANCE, MODE_BATCH_TRAIN, MODE_BATCH_EVAL, MODE_NONE = range(4)
_DTYPES = (torch.bfloat16, torch.float16)
# RAFT_FP32_ENC_FAST=0: an fp32 model's encoders run the eager modules (split convs per module)
_FP32_FAST = os.environ.get('RAFT_FP32_ENC_FAST', '1') != '0'


def _norm_mode(norm):
    if isinstance(norm, nn.InstanceNorm2d):
        if norm.affine or norm.track_running_stats:
            return None
        return MODE_INSTANCE
    if isinstance(norm, nn.BatchNorm2d):
        if norm.training or not norm.track_running_stats:
            return MODE_BATCH_TRAIN
        return MODE_BATCH_EVAL
    if isinstance(norm, nn.Sequential) and len(norm) == 0:
        return MODE_NONE
    return None


def _split_buf(t, pad):
    """Empty split-pair buffer (N, H, W, 2 pad) bf16 for the fp32 tensor t, or None."""
    if not pad or t.dtype != torch.float32:
        return None
    n, _, h, w = t.shape
    return torch.empty(n, h, w, 2 * pad, device=t.device, dtype=torch.bfloat16)


def _offer(t, buf):
    if buf is not None:
        from . import conv_fp32
        conv_fp32.offer_split(t, buf)


def _split_pads(x, conv):
    """(input, output-gradient) split-operand widths -- the 64-padded channel counts -- of conv
    applied to x when that call runs as ONE split conv (fp32 schedule, stride-1 'same' geometry,
    no image chunking), else (0, 0): then nothing is handed over."""
    if conv is None or x.dtype != torch.float32 or not _split_ok(x, conv):
        return 0, 0
    n, _, h, w = x.shape
    per = max(x[0].numel(), conv.out_channels * h * w) * x.element_size()
    if n > 1 and n * per > _CONV_BYTES:
        return 0, 0
    return _kslot(conv.in_channels), _kslot(conv.out_channels)


class _NormAct(torch.autograd.Function):
    """y = act(norm(x + conv_bias)) on channels_last bf16 / fp16; x is the bias-free conv output."""

    @staticmethod
    def forward(ctx, x, gamma, beta, cbias, norm, mode, relu, holder=None, sp=(0, 0), tst=None):
        # tst: (per-tile statistics, tiles per image) of x from its producing conv (conv_enc64's
        # epilogue) -- the norm then runs no statistics pass over x
        # sp = (ysp, gsp): fp32 schedule, the consuming / producing conv is a split conv -- y
        # (its input) and dx (its output gradient) are also written as the split pair
        # (2 x the 64-padded channels) and handed over (conv_fp32.offer_split)
        y = torch.empty_like(x, memory_format=torch.channels_last)
        ys = _split_buf(y, sp[0])
        rm = rv = None
        momentum = 0.1
        eps = 1e-5
        if isinstance(norm, (nn.BatchNorm2d, nn.InstanceNorm2d)):
            eps = norm.eps
        if mode in (MODE_BATCH_TRAIN, MODE_BATCH_EVAL) and norm.track_running_stats:
            rm, rv = norm.running_mean, norm.running_var
            if mode == MODE_BATCH_TRAIN:
                # num_batches_tracked: incremented for every batch norm of the encoder at once
                # (one multi-tensor add in encoder_forward)
                momentum = norm.momentum if norm.momentum is not None else \
                    1.0 / float(norm.num_batches_tracked.item())
        mean, invstd = _ext.ops().norm_fwd_(x, mode, int(relu), gamma, beta, cbias, rm, rv,
                                            float(momentum), float(eps), None, y, ys,
                                            *(tst if tst is not None else (None, 0)))
        _offer(y, ys)
        ctx.gsp = sp[1]
        # y is not kept (the backward recomputes the ReLU mask from x) unless an identity-residual
        # consumer stashes its gradient in `holder` (the stem output feeding layer1): the stash
        # is then added where the ReLU mask is applied, in the statistics pass (no add kernel)
        ctx.holder = holder
        ctx.save_for_backward(x, mean, invstd, gamma, beta, y if holder is not None else None)
        ctx.mode = mode
        ctx.relu = relu
        ctx.has = (gamma is not None, beta is not None, cbias is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mean, invstd, gamma, beta, y = ctx.saved_tensors
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        c = x.shape[1]
        dev = x.device
        # written (not accumulated) by the finalize kernel: no zero fill
        dg = torch.empty(c, device=dev) if ctx.has[0] else None
        db = torch.empty(c, device=dev) if ctx.has[1] else None
        dc = torch.empty(c, device=dev) if ctx.has[2] else None
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dxs = _split_buf(dx, ctx.gsp)
        stash = ctx.holder.pop('g', None) if ctx.holder is not None else None
        if stash is not None and ctx.relu:
            # g = (dy + stash) [y > 0] formed in the statistics pass (y = relu(norm(x)): the
            # recomputed mask from x is the same one)
            g = torch.empty_like(x, memory_format=torch.channels_last)
            _ext.ops().norm_bwd_(dy, x, None, mean, invstd, ctx.mode, 1, gamma, beta, dg, db, dc,
                                 dx, stash, y, g, dxs)
        else:
            if stash is not None:
                dy = dy + stash
            _ext.ops().norm_bwd_(dy, x, None, mean, invstd, ctx.mode, int(ctx.relu), gamma, beta,
                                 dg, db, dc, dx, None, None, None, dxs)
        _offer(dx, dxs)
        return dx, dg, db, dc, None, None, None, None, None, None


class _NormActAddRelu(torch.autograd.Function):
    """out = relu(relu(norm(x + conv_bias)) + res): the second conv of a residual block, its norm,
    ReLU, the residual add and the block-end ReLU as ONE node -- the apply pass adds the residual,
    so the branch output is never written (`core/extractor.py:47-56`)."""

    @staticmethod
    def forward(ctx, x, gamma, beta, cbias, res, norm, mode, holder, res_holder, sp=(0, 0),
                tst=None):
        out = torch.empty_like(x, memory_format=torch.channels_last)
        outs = _split_buf(out, sp[0])   # see _NormAct: the block output's split pair
        ctx.gsp = sp[1]
        ctx.holder = holder          # receives the NEXT block's residual gradient (see backward)
        ctx.res_holder = res_holder  # this block's residual comes from such a block: stash into it
        rm = rv = None
        momentum = 0.1
        eps = 1e-5
        if isinstance(norm, (nn.BatchNorm2d, nn.InstanceNorm2d)):
            eps = norm.eps
        if mode in (MODE_BATCH_TRAIN, MODE_BATCH_EVAL) and norm.track_running_stats:
            rm, rv = norm.running_mean, norm.running_var
            if mode == MODE_BATCH_TRAIN:
                # num_batches_tracked: incremented for every batch norm of the encoder at once
                # (one multi-tensor add in encoder_forward)
                momentum = norm.momentum if norm.momentum is not None else \
                    1.0 / float(norm.num_batches_tracked.item())
        res = res.contiguous(memory_format=torch.channels_last)
        mean, invstd = _ext.ops().norm_fwd_(x, mode, 1, gamma, beta, cbias, rm, rv, float(momentum),
                                            float(eps), res, out, outs,
                                            *(tst if tst is not None else (None, 0)))
        _offer(out, outs)
        ctx.save_for_backward(x, out, mean, invstd, gamma, beta)
        ctx.mode = mode
        ctx.has = (gamma is not None, beta is not None, cbias is not None)
        return out

    @staticmethod
    def backward(ctx, dout):
        x, out, mean, invstd, gamma, beta = ctx.saved_tensors
        dout = dout.to(out.dtype).contiguous(memory_format=torch.channels_last)
        g = torch.empty_like(out, memory_format=torch.channels_last)
        # an identity-residual consumer of this block's output left its gradient in the stash
        # instead of handing it to autograd: it is added where the block-end ReLU mask is applied
        # (no bf16 add kernel).  It always runs first -- this node waits for every consumer of
        # its output.
        stash = ctx.holder.pop('g', None)
        c = x.shape[1]
        dev = x.device
        dg = torch.empty(c, device=dev) if ctx.has[0] else None
        db = torch.empty(c, device=dev) if ctx.has[1] else None
        dc = torch.empty(c, device=dev) if ctx.has[2] else None
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dxs = _split_buf(dx, ctx.gsp)
        # block-end ReLU fused into the norm backward's statistics pass: g = (dout [+ stash]) *
        # [out > 0] is formed there and stored once (it is also the residual's gradient)
        _ext.ops().norm_bwd_(dout, x, None, mean, invstd, ctx.mode, 1, gamma, beta, dg, db, dc, dx,
                             stash, out, g, dxs)
        _offer(dx, dxs)
        gres = g
        if ctx.res_holder is not None:
            ctx.res_holder['g'] = g
            gres = None
        return dx, dg, db, dc, gres, None, None, None, None, None, None


class _StashGrad(torch.autograd.Function):
    """Identity whose input gradient goes into the producer's stash (``holder``) instead of
    autograd: a downsample block's input feeds its stride-2 conv1 AND its downsample conv, and
    the two input gradients would otherwise be summed by an add kernel before the producing
    block's norm backward, which adds the stash in its statistics pass anyway."""

    @staticmethod
    def forward(ctx, x, holder):
        ctx.holder = holder
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        g = g.contiguous(memory_format=torch.channels_last)
        prev = ctx.holder.get('g')
        ctx.holder['g'] = g if prev is None else prev + g
        return None, None


class _AddRelu(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b):
        a = a.contiguous(memory_format=torch.channels_last)
        b = b.contiguous(memory_format=torch.channels_last)
        out = torch.empty_like(a, memory_format=torch.channels_last)
        _ext.ops().add_relu_(a, b, out)
        ctx.save_for_backward(out)
        return out

    @staticmethod
    def backward(ctx, dout):
        (out,) = ctx.saved_tensors
        dout = dout.to(out.dtype).contiguous(memory_format=torch.channels_last)
        g = torch.empty_like(out, memory_format=torch.channels_last)
        _ext.ops().relu_mask_(dout, out, g)
        return g, g


class _ContextAct(torch.autograd.Function):
    """net, inp = tanh / relu of the context encoder's two channel halves (`core/raft.py:111-113`)
    in one native pass, each as its own contiguous NHWC tensor (returned as NCHW views) -- the
    fused update block's operand layout, so no split / activation / layout-copy kernels."""

    @staticmethod
    def forward(ctx, cnet, hdim):
        b, c, hh, ww = cnet.shape
        h = torch.empty(b, hh, ww, hdim, device=cnet.device, dtype=cnet.dtype)
        x = torch.empty(b, hh, ww, c - hdim, device=cnet.device, dtype=cnet.dtype)
        _ext.ops().ctx_act_(cnet, hdim, h, x)
        ctx.save_for_backward(h, x)
        ctx.set_materialize_grads(False)
        return h.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2)

    @staticmethod
    def backward(ctx, gh, gx):
        h, x = ctx.saved_tensors
        b, hh, ww, hd = h.shape
        gin = torch.empty(b, hd + x.shape[-1], hh, ww, device=h.device, dtype=h.dtype,
                          memory_format=torch.channels_last)
        nhwc = (lambda g: None if g is None else g.to(h.dtype).permute(0, 2, 3, 1).contiguous())
        _ext.ops().ctx_act_bwd_(nhwc(gh), nhwc(gx), h, x, gin)
        return gin, None


def context_act(cnet, hdim):
    """(tanh(cnet[:, :hdim]), relu(cnet[:, hdim:])) by the native kernel when cnet is a 16-bit
    channels_last GPU tensor the kernel takes; None otherwise (the caller runs the eager ops)."""
    c = cnet.shape[1]
    if not (cnet.is_cuda and cnet.dtype in (torch.bfloat16, torch.float16) and cnet.dim() == 4
            and cnet.is_contiguous(memory_format=torch.channels_last) and c % 8 == 0 and c <= 256
            and hdim % 8 == 0 and 0 < hdim < c and _ext.device_ok(cnet)
            and _ext.gpu_path_enabled(required=False)):
        return None
    return _ContextAct.apply(cnet, hdim)


class _CastWeightsCL(torch.autograd.Function):
    """All conv weights of an encoder -> 16-bit (bf16 / fp16: the autocast dtype) channels_last
    views of ONE buffer, and back.

    Per conv, ``weight.to(bf16).contiguous(channels_last)`` and the backward cast of its bf16
    gradient are 2-3 tiny kernels each (~100 launches per step for both encoders).  Here the
    forward is ONE native permuting gather + cast over the weights in place (gather_cast_) and
    the backward one inverse gather + cast over the per-conv gradients, with
    the index maps built once per weight geometry.  The same gather also lays out, for every
    native stride-1 3x3 conv, the ADJOINT weight (flipped taps, Cin <-> Cout: the input-gradient
    conv's packed [ci][tap * co' + o] operand) and -- when Cin is not a multiple of 64 (the 96-
    channel convs) -- a forward pack with 64-aligned K slots [co][tap * ci' + c] whose padded
    entries read a zero element; the backward then runs no per-conv flip / transpose / pad
    kernels.  Those extra outputs carry no gradient."""

    @staticmethod
    def forward(ctx, maps, dt, *ws):
        perm, inv, shapes, extra = maps
        # one gather + cast launch over the weights in place (csrc/kernels/gather.hip)
        packed = torch.empty(perm.numel(), device=ws[0].device, dtype=dt)
        from . import conv as C
        C.gather_cast([w.detach().float().contiguous() for w in ws], perm, packed)
        outs, off = [], 0
        for (co, ci, kh, kw) in shapes:
            n = co * ci * kh * kw
            outs.append(packed[off:off + n].view(co, kh, kw, ci).permute(0, 3, 1, 2))
            off += n
        ext = []
        for _, rows, cols in extra:
            ext.append(packed[off:off + rows * cols].view(rows, cols))
            off += rows * cols
        ctx.maps = maps
        ctx.dt = dt
        ctx.mark_non_differentiable(*ext)
        # the extra packs never get a gradient: no zero-filled stand-ins for them (13 fills of a
        # BasicEncoder's packs per backward); a weight without one is zero-filled below
        ctx.set_materialize_grads(False)
        return tuple(outs) + tuple(ext)

    @staticmethod
    def backward(ctx, *gs):
        perm, inv, shapes, extra = ctx.maps
        parts = []
        for g, (co, ci, kh, kw) in zip(gs[:len(shapes)], shapes):
            if g is None:
                g = torch.zeros(co, ci, kh, kw, device=perm.device, dtype=ctx.dt)
            # (co, kh, kw, ci) memory order: a view of a channels_last gradient
            parts.append(g.to(ctx.dt).permute(0, 2, 3, 1).contiguous())
        # fp32 parameter-layout gradients of every weight: ONE inverse gather + cast launch
        flat = torch.empty(inv.numel(), device=perm.device)
        from . import conv as C
        C.gather_cast(parts, inv, flat)
        grads, off = [], 0
        for (co, ci, kh, kw) in shapes:
            n = co * ci * kh * kw
            grads.append(flat[off:off + n].view(co, ci, kh, kw))
            off += n
        return (None, None, *grads)


_MAPS = {}


def _kslot(c):
    return (c + 63) // 64 * 64


def _native_geom(conv):
    """Static geometry of a conv the native 3x3 path can run (the input-dependent checks come
    at call time, ``_conv_native_ok``): stride-1 'same' 3x3 with 32-multiple channel counts."""
    return (conv.kernel_size == (3, 3) and conv.stride == (1, 1) and conv.padding == (1, 1)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.in_channels % 32 == 0
            and conv.out_channels % 32 == 0 and conv.out_channels <= 1024
            and conv.in_channels <= 1024)


def _cast_maps(shapes, device, native=()):
    key = (tuple(shapes), str(device), tuple(native))
    if key not in _MAPS:
        perm, off, offs = [], 0, []
        for (co, ci, kh, kw) in shapes:
            n = co * ci * kh * kw
            # packed (co, kh, kw, ci) position -> flat NCHW (co, ci, kh, kw) element
            perm.append(torch.arange(n).view(co, ci, kh, kw).permute(0, 2, 3, 1).reshape(-1) + off)
            offs.append(off)
            off += n
        n_fwd = off
        zero = n_fwd  # index of the appended zero element
        extra = []    # ('adj' | 'fwd', rows, cols) per extra output, in output order
        for j in native:
            co, ci, kh, kw = shapes[j]
            idx = torch.arange(co * ci * kh * kw).view(co, ci, kh, kw) + offs[j]
            # adjoint W'[c][tap'][o] = W[o][c][flip(tap')]: packed (ci, kh, kw, co'), o >= co zero
            adj = idx.flip(2, 3).permute(1, 2, 3, 0)
            cop = _kslot(co)
            if cop > co:
                adj = torch.cat([adj, torch.full((ci, kh, kw, cop - co), zero)], 3)
            perm.append(adj.reshape(-1))
            extra.append(('adj', ci, kh * kw * cop))
        for j in native:
            co, ci, kh, kw = shapes[j]
            cip = _kslot(ci)
            if cip == ci:
                continue  # the channels_last weight IS the packed forward operand
            idx = torch.arange(co * ci * kh * kw).view(co, ci, kh, kw).permute(0, 2, 3, 1) + offs[j]
            fwd = torch.cat([idx, torch.full((co, kh, kw, cip - ci), zero)], 3)
            perm.append(fwd.reshape(-1))
            extra.append(('fwd', co, kh * kw * cip))
        perm = torch.cat(perm)
        inv = torch.empty(n_fwd, dtype=torch.long)
        inv[perm[:n_fwd]] = torch.arange(n_fwd)
        # forward: (weight, offset) codes of the native gather; backward: flat inverse permutation
        from . import conv as C
        numels = [co * ci * kh * kw for (co, ci, kh, kw) in shapes]
        code = C.gather_index(perm, numels)
        inv_code = C.gather_index(inv, numels)   # packed position -> (weight, offset)
        _MAPS[key] = (code.to(device), inv_code.to(device), list(shapes), tuple(extra))
    return _MAPS[key]


def cast_conv_weights(convs, dt=torch.bfloat16):
    """({conv: 16-bit channels_last weight}, {conv: packed adjoint weight}, {conv: packed forward
    weight with 64-aligned K slots, when Cin % 64 != 0}) for a list of nn.Conv2d, one batched cast
    node; ``dt`` = bf16 or fp16 (fp32: channels_last fp32 weights only -- the split convs pack
    their own operands)."""
    ws = [c.weight for c in convs]
    native = () if dt == torch.float32 else tuple(j for j, c in enumerate(convs) if _native_geom(c))
    maps = _cast_maps([tuple(w.shape) for w in ws], ws[0].device, native)
    outs = _CastWeightsCL.apply(maps, dt, *ws)
    ext = outs[len(convs):]
    adj = {convs[j]: ext[k] for k, j in enumerate(native)}
    fwd, k = {}, len(native)
    for j in native:
        if _kslot(convs[j].in_channels) != convs[j].in_channels:
            fwd[convs[j]] = ext[k]
            k += 1
    return dict(zip(convs, outs[:len(convs)])), adj, fwd


class _Head1x1(torch.autograd.Function):
    """The encoders' final 1x1 conv (`core/extractor.py:185`, 128 -> 256 with bias) on the
    MFMA implicit-GEMM kernels of the update block (NHWC bf16 / fp16, fp32 accumulation): forward with
    the bias epilogue, input gradient by the same kernel on the transposed weight, weight / bias
    gradient by the split-K wgrad kernel.  Replaces MIOpen's 1x1 solvers, one of which produced
    inf weight gradients under hipGraph replay (profiles/r2/graph_cmp_cnet_conv2.log)."""

    @staticmethod
    def forward(ctx, x, weight, bias):
        from . import conv as C
        B, cin, H, W = x.shape
        cout = weight.shape[0]
        xn = x.permute(0, 2, 3, 1)                     # channels_last memory: a view, no copy
        if not xn.is_contiguous():
            xn = xn.contiguous()
        w2 = weight.reshape(cout, cin)
        wpk = C.pack_weight(weight, [cin], [cin], dtype=x.dtype)   # (Npad, cin) 16-bit
        out = torch.empty(B, H, W, cout, device=x.device, dtype=x.dtype)
        C.conv_fwd([(xn, 0, cin)], wpk, bias.float().contiguous(), (1, 1), (0, 0), cout,
                   C.EPI_BF16, [out], [0])
        ctx.save_for_backward(xn, w2)
        return out.permute(0, 3, 1, 2)                  # (B, cout, H, W), channels_last strides

    @staticmethod
    def backward(ctx, dy):
        from . import conv as C
        xn, w2 = ctx.saved_tensors
        B, H, W, cin = xn.shape
        cout = w2.shape[0]
        dt = xn.dtype
        g = dy.permute(0, 2, 3, 1).to(dt).contiguous()   # (B, H, W, cout)
        dx = torch.empty(B, H, W, cin, device=xn.device, dtype=dt)
        wd = C.pack_weight(w2.t().contiguous().view(cin, cout, 1, 1), [cout], [cout], dtype=dt)
        _ext.ops().conv_dgrad_([g], [0], [cout], wd, 1, 1, 0, 0, 0, 1.0, [dx], [0], [cin], [cin],
                               [0], [dx], [-1], [], [])
        dw = torch.zeros(cout, cin, device=xn.device)
        db = torch.zeros(cout, device=xn.device)
        if dt == torch.float16:
            # the tile kernel (conv_wgrad.hip) is bf16-only; the tap-fused one takes fp16
            C.conv_wgrad_taps([(g, [xn])], 0, [0], [cin], (1, 1), (0, 0), cout, dw, db)
        else:
            C.conv_wgrad(g, 0, [(xn, 0, cin)], (1, 1), (0, 0), cout, dw, db)
        return dx.permute(0, 3, 1, 2), dw.view(cout, cin, 1, 1), db


def _head_ok(x, conv, dt=torch.bfloat16):
    return (conv.kernel_size == (1, 1) and conv.stride == (1, 1) and conv.bias is not None
            and conv.in_channels % 64 == 0 and conv.out_channels % 32 == 0 and x.is_cuda
            and _HEAD_NATIVE and dt in _DTYPES)


_HEAD_NATIVE = os.environ.get('RAFT_ENCODER_HEAD_NATIVE', '1') != '0'


class _Conv3x3WgradNative(torch.autograd.Function):
    """Stride-1 3x3 "same" encoder conv (the residual blocks' stride-1 convs, `core/extractor.py
    :22-23`): forward and input gradient on MIOpen, weight gradient on the tap-fused MFMA kernel
    (csrc/kernels/conv_wgrad_taps.hip -- one workgroup per Cout x 64-Cin slab owns all 9 taps over
    8x8-pixel halo tiles).  Replaces MIOpen's backward-weights solvers and their zero-fill / cast
    passes (SubTensorOp kernels) for these convs."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return F.conv2d(x, w, None, 1, 1)

    @staticmethod
    def backward(ctx, dy):
        from . import conv as C
        x, w = ctx.saved_tensors
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = torch.ops.aten.convolution_backward(
                dy, x, w, None, [1, 1], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]
        if ctx.needs_input_grad[1]:
            co, ci = w.shape[:2]
            # 16-bit stored straight by the split reduce (no zero fill, no cast kernel)
            dwp = torch.empty(co, 9 * ci, device=x.device, dtype=x.dtype)
            C.conv_wgrad_taps([(dy.permute(0, 2, 3, 1), [x.permute(0, 2, 3, 1)])], 0, [0], [ci],
                              (3, 3), (1, 1), co, dwp, None)
            # packed (co, kh, kw, ci) -> (co, ci, kh, kw) with channels_last strides (= w's)
            dw = dwp.view(co, 3, 3, ci).permute(0, 3, 1, 2)
        return dx, dw


_WGRAD_NATIVE = os.environ.get('RAFT_ENCODER_WGRAD_NATIVE', '1') != '0'


_ENC64 = os.environ.get('RAFT_ENC64', '1') != '0'


# RAFT_ENC64_STATS=1: the norm after a conv_enc64 conv takes its statistics from the conv's
# epilogue instead of running its own statistics pass (A/B; see README)
_ENC64_STATS = os.environ.get('RAFT_ENC64_STATS', '0') == '1'


def _enc64_tiles(h, w):
    return ((h + 7) // 8) * ((w + 15) // 16)


def _conv3x3_nhwc(xn, wpk, ci, co, sink=None):
    """NHWC 16-bit stride-1 3x3 conv with a packed [co][tap * ci' + c] weight (ci' = ci rounded up
    to 64; the K slot past ci reads zeros): 64 -> 64 channels on the persistent 2-D halo-tile
    kernel (conv_enc64.hip), anything else on the implicit GEMM.  ``sink`` (dict): the 64 -> 64
    kernel also reduces its output into per-tile norm statistics, left in sink['tst'] as
    (tensor, tiles per image) for the norm that follows."""
    from . import conv as C
    B, H, W, _ = xn.shape
    out = torch.empty(B, H, W, co, device=xn.device, dtype=xn.dtype)
    if _ENC64 and ci == 64 and co == 64:
        part = None
        if sink is not None and _ENC64_STATS:
            tiles = _enc64_tiles(H, W)
            part = torch.empty(B * tiles, 4, 64, device=xn.device, dtype=torch.float32)
            sink['tst'] = (part, tiles)
        _ext.ops().conv_enc64_(xn, wpk, out, part)
    else:
        C.conv_fwd([(xn, 0, _kslot(ci))], wpk, None, (3, 3), (1, 1), co, C.EPI_BF16, [out], [0],
                   bn=32)
    return out


def _conv3x3_native_fwd(x, w, wf=None, sink=None):
    ci, co = x.shape[1], w.shape[0]
    xn = x.permute(0, 2, 3, 1)                     # channels_last memory: a view
    if wf is None:
        wf = w.permute(0, 2, 3, 1).reshape(co, 9 * ci)
        if _kslot(ci) != ci:
            wf = torch.nn.functional.pad(wf.view(co, 9, ci), (0, _kslot(ci) - ci)).reshape(co, -1)
    return _conv3x3_nhwc(xn, wf, ci, co, sink).permute(0, 3, 1, 2)


class _Conv3x3Native(torch.autograd.Function):
    """Stride-1 3x3 "same" encoder conv with 64-multiple channel counts (`core/extractor.py:22-23`:
    layer1's 64-channel and layer3's 128-channel residual convs) entirely on the MFMA kernels:
    forward = the update block's implicit-GEMM conv (bf16 epilogue), input gradient = the same
    kernel on the flipped / transposed weight, weight gradient = the tap-fused kernel.  MIOpen
    took 1.6-4.5x longer per call on these shapes (profiles/r3/enc_conv_miopen_vs_mfma.txt) and
    zero-filled every input-gradient buffer before its solver ran (SubTensorOpWithScalar1d).

    The channels_last bf16 weight (co, kh, kw, ci in memory) IS the kernels' packed layout
    [co][tap * ci + c]: the forward packs nothing."""

    @staticmethod
    def forward(ctx, x, w, wd=None, wf=None, sink=None):
        ctx.save_for_backward(x, w, wd)
        return _conv3x3_native_fwd(x, w, wf, sink)

    @staticmethod
    def backward(ctx, dy):
        from . import conv as C
        x, w, wd = ctx.saved_tensors
        co, ci = w.shape[:2]
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        gn = dy.permute(0, 2, 3, 1)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            B, _, H, W = x.shape
            if wd is None:
                # adjoint weight W'[c][tap'][o] = W[o][c][flip(tap')], in the kernels' packed
                # layout (normally laid out by the batched weight cast, _CastWeightsCL)
                wd = C.pack_weight(w.flip(2, 3).transpose(0, 1), [co], [_kslot(co)], npad_mult=1,
                                   dtype=x.dtype)
            if _ENC64 and ci == 64 and co == 64:
                dx = _conv3x3_nhwc(gn, wd, co, ci).permute(0, 3, 1, 2)
            else:
                dxn = torch.empty(B, H, W, ci, device=x.device, dtype=x.dtype)
                _ext.ops().conv_dgrad_([gn], [0], [_kslot(co)], wd, 3, 3, 1, 1, 0, 1.0, [dxn], [0],
                                       [ci], [ci], [0], [dxn], [-1], [], [])
                dx = dxn.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[1]:
            dwp = torch.empty(co, 9 * ci, device=x.device, dtype=x.dtype)
            C.conv_wgrad_taps([(gn, [x.permute(0, 2, 3, 1)])], 0, [0], [ci], (3, 3), (1, 1), co,
                              dwp, None)
            dw = dwp.view(co, 3, 3, ci).permute(0, 3, 1, 2)
        return dx, dw, None, None, None


# RAFT_STEM_NATIVE=0: the encoders' 7x7 stride-2 stem conv on MIOpen instead of stem_conv.hip
_STEM_NATIVE = os.environ.get('RAFT_STEM_NATIVE', '1') != '0'


def _stem_ok(x, conv, w):
    """The encoders' stem (`core/extractor.py:129,165`: 7x7, stride 2, pad 3, 3 -> 64 / 32) on the
    MFMA stem kernels: 16-bit channels_last input and weight."""
    return (_STEM_NATIVE and conv.kernel_size == (7, 7) and conv.stride == (2, 2)
            and conv.padding == (3, 3) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.in_channels == 3 and conv.out_channels in (32, 64) and x.is_cuda
            and x.dtype in _DTYPES and w.dtype == x.dtype
            and x.is_contiguous(memory_format=torch.channels_last)
            and w.is_contiguous(memory_format=torch.channels_last))


def _stem_fwd(x, w):
    b, _, h, wd = x.shape
    out = torch.empty(b, (h - 1) // 2 + 1, (wd - 1) // 2 + 1, w.shape[0], device=x.device,
                      dtype=x.dtype)
    # channels_last memory: (B, H, W, 3) and (C, 7, 7, 3) are contiguous views
    _ext.ops().stem_conv_fwd_(x.permute(0, 2, 3, 1), w.permute(0, 2, 3, 1), out)
    return out.permute(0, 3, 1, 2)


class _StemConv(torch.autograd.Function):
    """Stem conv on stem_conv.hip: forward and weight gradient on MFMA (MIOpen: ~100 us forward +
    ~134 us weight gradient per call at chairs, plus a zero fill); the input gradient -- never
    needed for images -- falls back to ATen."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return _stem_fwd(x, w)

    @staticmethod
    def backward(ctx, dy):
        x, w = ctx.saved_tensors
        dx = dw = None
        dy = dy.to(x.dtype).contiguous(memory_format=torch.channels_last)
        if ctx.needs_input_grad[1]:
            dw = _ext.ops().stem_conv_wgrad(x.permute(0, 2, 3, 1), dy.permute(0, 2, 3, 1))
            dw = dw.permute(0, 3, 1, 2)
        if ctx.needs_input_grad[0]:
            dx = torch.nn.grad.conv2d_input(x.shape, w, dy, stride=2, padding=3)
        return dx, dw


_CONV_NATIVE = os.environ.get('RAFT_ENCODER_CONV_NATIVE', '1') != '0'


def _conv_native_ok(x, conv):
    # 32-multiple channel counts: a 96-channel operand runs in a 128-channel K slot (the kernels
    # read the missing channels as zeros; the packed weights are zero there)
    return (_CONV_NATIVE and _wgrad_native_ok(x, conv) and _native_geom(conv))


def _wgrad_native_ok(x, conv):
    return (_WGRAD_NATIVE and conv.kernel_size == (3, 3) and conv.stride == (1, 1)
            and conv.padding == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.in_channels % 32 == 0 and conv.out_channels % 8 == 0
            and conv.in_channels <= 1024 and x.is_cuda and x.dtype in _DTYPES
            and x.is_contiguous(memory_format=torch.channels_last)
            and x.numel() * 2 < 2 ** 31 and x.shape[0] * x.shape[2] * x.shape[3] * conv.out_channels * 2 < 2 ** 31)


# int32 byte-offset range of MIOpen's kernels and of our buffer descriptors
_CONV_BYTES = int(os.environ.get('RAFT_CONV_CHUNK_BYTES', str(2 ** 31 - 1)))


def _conv(ps, x, conv, with_bias=False, sink=None):
    """One encoder conv; batches whose input or output passes 2 GiB run as equal image chunks
    (a conv is per-image; the batch norm that couples the images runs on the whole batch, so a
    training-mode batch-norm encoder -- the chairs stage -- no longer caps the per-GPU batch)."""
    n, _, h, w = x.shape
    sh, sw = conv.stride
    ho = (h + 2 * conv.padding[0] - conv.dilation[0] * (conv.kernel_size[0] - 1) - 1) // sh + 1
    wo = (w + 2 * conv.padding[1] - conv.dilation[1] * (conv.kernel_size[1] - 1) - 1) // sw + 1
    per = max(x[0].numel(), conv.out_channels * ho * wo) * x.element_size()
    if n > 1 and n * per > _CONV_BYTES:
        k = max(1, _CONV_BYTES // per)
        parts = -(-n // k)
        size = -(-n // parts)   # equal chunks: the same kernel choices for every chunk
        outs = [_conv_one(ps, c, conv, with_bias) for c in torch.split(x, size, dim=0)]
        return torch.cat(outs, dim=0).contiguous(memory_format=torch.channels_last)
    return _conv_one(ps, x, conv, with_bias, sink)


def _split_geom(conv):
    k = conv.kernel_size
    return (conv.stride == (1, 1) and conv.dilation == (1, 1) and conv.groups == 1
            and conv.padding == (k[0] // 2, k[1] // 2))


def _split_ok(x, conv):
    """fp32 stride-1 'same' conv on the split-bf16 MFMA kernels (ops/conv_fp32.py)."""
    from . import conv_fp32
    return x.dtype == torch.float32 and _split_geom(conv) and conv_fp32.fits(x, conv.out_channels)


def _conv_one(ps, x, conv, with_bias=False, sink=None):
    w = ps.weights.get(conv)
    if w is None:
        w = conv.weight.to(x.dtype).contiguous(memory_format=torch.channels_last)
    if x.dtype == torch.float32:
        # fp32 schedule: split-bf16 MFMA for the stride-1 convs, MIOpen fp32 for the strided ones
        b = conv.bias if (with_bias and conv.bias is not None) else None
        if _split_ok(x, conv):
            from . import conv_fp32
            return conv_fp32.conv2d(x, w, b, conv.padding)
        return F.conv2d(x, w, b, conv.stride, conv.padding, conv.dilation, conv.groups)
    if not with_bias and _conv_native_ok(x, conv) and w.is_contiguous(memory_format=torch.channels_last):
        if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
            return _Conv3x3Native.apply(x, w, ps.adjoint.get(conv), ps.fwdpack.get(conv), sink)
        return _conv3x3_native_fwd(x, w, ps.fwdpack.get(conv), sink)
    if not with_bias and _stem_ok(x, conv, w):
        if torch.is_grad_enabled() and (x.requires_grad or w.requires_grad):
            return _StemConv.apply(x, w)
        return _stem_fwd(x, w)
    if not with_bias and _wgrad_native_ok(x, conv) and torch.is_grad_enabled() and \
            (x.requires_grad or w.requires_grad):
        return _Conv3x3WgradNative.apply(x, w)
    b = conv.bias.to(x.dtype) if (with_bias and conv.bias is not None) else None
    return F.conv2d(x, w, b, conv.stride, conv.padding, conv.dilation, conv.groups)


def conv_norm_act(ps, x, conv, norm, relu=True, holder=None, consumer=None):
    """``consumer``: the conv that reads this output (fp32 schedule: when both are split convs
    the norm kernels also write the split operands, see _NormAct)."""
    mode = _norm_mode(norm)
    # training statistics: the 64 -> 64 conv kernel reduces its own output (no stats pass)
    sink = {} if mode in (MODE_INSTANCE, MODE_BATCH_TRAIN) else None
    y = _conv(ps, x, conv, sink=sink)
    y = y.contiguous(memory_format=torch.channels_last)
    gamma = beta = None
    if mode in (MODE_BATCH_TRAIN, MODE_BATCH_EVAL) and norm.affine:
        gamma, beta = norm.weight, norm.bias
    sp = (_split_pads(y, consumer)[0], _split_pads(x, conv)[1])
    out = _NormAct.apply(y, gamma, beta, conv.bias, norm, mode, relu, holder, sp,
                         sink.get('tst') if sink else None)
    if holder is not None:
        ps.holders[id(out)] = (out, holder)
    return out


def residual_block(ps, blk, x, consumer=None):
    """`core/extractor.py:47-56` on the fast path (conv2 + norm2 + ReLU + add + ReLU fused);
    ``consumer``: the conv reading the block output (see conv_norm_act)."""
    y = conv_norm_act(ps, x, blk.conv1, blk.norm1, consumer=blk.conv2)
    if blk.downsample is not None:
        xd = x
        prod = ps.holders.get(id(x)) if _STASH else None
        if prod is not None and prod[0] is x:
            xd = _StashGrad.apply(x, prod[1])   # its gradient joins the producer's stash
        x = conv_norm_act(ps, xd, blk.downsample[0], blk.downsample[1], relu=False)
    mode = _norm_mode(blk.norm2)
    sink = {} if mode in (MODE_INSTANCE, MODE_BATCH_TRAIN) else None
    y2 = _conv(ps, y, blk.conv2, sink=sink).contiguous(memory_format=torch.channels_last)
    gamma = beta = None
    if mode in (MODE_BATCH_TRAIN, MODE_BATCH_EVAL) and blk.norm2.affine:
        gamma, beta = blk.norm2.weight, blk.norm2.bias
    # identity shortcut from a previous fused block: its gradient goes through that block's stash
    res_holder = ps.holders.get(id(x)) if (blk.downsample is None and _STASH) else None
    if res_holder is not None and res_holder[0] is not x:
        res_holder = None
    holder = {}
    sp = (_split_pads(y2, consumer)[0], _split_pads(y, blk.conv2)[1])
    out = _NormActAddRelu.apply(y2, gamma, beta, blk.conv2.bias, x, blk.norm2, mode, holder,
                                res_holder[1] if res_holder is not None else None, sp,
                                sink.get('tst') if sink else None)
    ps.holders[id(out)] = (out, holder)
    return out


# _Pass.holders: id(block output) -> (output, its gradient stash), for ONE encoder forward.
# Restriction of the stash: the identity-residual gradient of a fused block's output reaches its
# producer through the stash, not through autograd, so a tensor hook on an intermediate block
# output, or ``autograd.grad(..., inputs=[block_out])``, sees the gradient WITHOUT the shortcut
# term.  Parameter gradients and the encoder-input gradient are exact (the producer node always
# runs after all consumers of its output).  ``RAFT_ENCODER_STASH=0`` in the environment keeps
# the shortcut gradient in the autograd graph when intermediate activation gradients are needed.
_STASH = os.environ.get('RAFT_ENCODER_STASH', '1') != '0'


def bottleneck_block(ps, blk, x, consumer=None):
    """`core/extractor.py:105-116` on the fast path."""
    y = conv_norm_act(ps, x, blk.conv1, blk.norm1)
    y = conv_norm_act(ps, y, blk.conv2, blk.norm2)
    y = conv_norm_act(ps, y, blk.conv3, blk.norm3)
    if blk.downsample is not None:
        x = conv_norm_act(ps, x, blk.downsample[0], blk.downsample[1], relu=False)
    return _AddRelu.apply(x, y)


def fast_path_ok(enc, x):
    """GPU + native library + bf16 / fp16 autocast + supported norms; otherwise the eager path runs.
    ``enc.allow_native = False`` (set by RAFT for ``corr_impl='torch'``, the stock-ops baseline)
    forces the eager MIOpen / ATen encoder."""
    if not getattr(enc, 'allow_native', True):
        return False
    if not (isinstance(x, torch.Tensor) and x.is_cuda and _ext.device_ok(x)):
        return False
    if torch.is_autocast_enabled('cuda'):
        if torch.get_autocast_dtype('cuda') not in _DTYPES:
            return False
    else:
        # fp32 model: inside the encoders' split-conv scope (RAFT.encode, conv_fp32.enabled)
        from . import conv_fp32
        if not (_FP32_FAST and x.dtype == torch.float32 and conv_fp32._ACTIVE['on']
                and conv_fp32._ENV_ON):
            return False
    if enc.training and enc.dropout is not None:
        return False
    if not _ext.gpu_path_enabled(required=False):
        return False
    for m in enc.modules():
        if isinstance(m, (nn.GroupNorm,)):
            return False
        if isinstance(m, nn.InstanceNorm2d) and _norm_mode(m) is None:
            return False
    return True


class _Pass:
    """State of ONE encoder forward: the batched 16-bit weight casts and the residual-gradient
    stashes.  Passed down explicitly (no module globals), so encoder forwards running
    concurrently on two streams or threads, or re-entrantly, cannot see each other's state."""

    def __init__(self, weights, adjoint, fwdpack):
        self.weights = weights   # conv -> 16-bit channels_last weight
        self.adjoint = adjoint   # conv -> packed adjoint weight (native 3x3 convs)
        self.fwdpack = fwdpack   # conv -> packed forward weight, 64-aligned K slots (Cin 96)
        self.holders = {}        # id(block output) -> (output, its gradient stash)


def encoder_forward(enc, x):
    """`core/extractor.py:168-192` (both encoders): returns channels_last features in the
    autocast dtype (bf16 / fp16), or fp32 for an fp32 model."""
    dt = torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else torch.float32
    with torch.autocast('cuda', enabled=False):
        convs = [m for m in enc.modules() if isinstance(m, nn.Conv2d)]
        if _head_ok(x, enc.conv2, dt):
            convs = [c for c in convs if c is not enc.conv2]  # runs on _Head1x1 (fp32 weight)
        counters = [m.num_batches_tracked for m in enc.modules()
                    if isinstance(m, nn.BatchNorm2d) and _norm_mode(m) == MODE_BATCH_TRAIN
                    and m.track_running_stats and m.num_batches_tracked is not None]
        if counters:
            with torch.no_grad():
                torch._foreach_add_(counters, 1)
        ps = _Pass(*cast_conv_weights(convs, dt))
        if dt == torch.float32:
            # fp32 schedule: every split-conv's [w_hi | w_hi | w_lo] packs (forward and adjoint)
            # in one gather launch instead of ~10 small kernels per conv and direction
            from . import conv_fp32
            conv_fp32.prepack([(ps.weights[c], c.weight.detach().float().contiguous())
                               for c in convs if c in ps.weights and _split_geom(c)])
        return _encoder_body(ps, enc, x, dt)


def _encoder_body(ps, enc, x, dt=torch.bfloat16):
    x = x.to(dt).contiguous(memory_format=torch.channels_last)
    block_fn = residual_block if enc.block.__name__ == 'ResidualBlock' else bottleneck_block
    blocks = [blk for layer in (enc.layer1, enc.layer2, enc.layer3) for blk in layer]
    # the conv reading each block's output: the next block's conv1 when nothing else does (a
    # downsample conv reads it too); the head after the last block
    nxt = [b.conv1 if (block_fn is residual_block and b.downsample is None) else None
           for b in blocks[1:]] + [None if _head_ok(x, enc.conv2, dt) else enc.conv2]
    first = blocks[0].conv1 if (block_fn is residual_block and blocks[0].downsample is None) else None
    if dt == torch.float32:
        from . import conv_fp32
        conv_fp32.clear_handoff()   # nothing left over from an earlier pass
    # the stem output's identity-residual gradient (layer1's first block) goes to its stash
    x = conv_norm_act(ps, x, enc.conv1, enc.norm1, holder={} if _STASH else None, consumer=first)
    for blk, consumer in zip(blocks, nxt):
        x = block_fn(ps, blk, x, consumer)
    if _head_ok(x, enc.conv2, dt):
        return _Head1x1.apply(x, enc.conv2.weight, enc.conv2.bias)
    x = _conv(ps, x, enc.conv2, with_bias=True)
    return x
