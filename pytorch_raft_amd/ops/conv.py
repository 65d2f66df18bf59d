"""NHWC bf16 implicit-GEMM convolution on MFMA (csrc/kernels/conv_igemm.hip, conv_wgrad.hip).

Activation convention: a *buffer* is a contiguous (B, H, W, C) bf16 tensor; a *segment* is a channel
slice ``(buffer, offset, count)``.  A conv reads the virtual concatenation of up to three segments
(torch.cat never materialises) and writes its result into a channel slice of an output buffer.

Weights stay in the nn.Conv2d modules (checkpoint layout untouched) and are re-packed once per
optimizer step (``pack_weight``) to the kernel layout [Npad][KH*KW][CinPad] bf16, where each input
segment's real channels are placed at its padded offset (e.g. the 324 correlation channels live in
a 384-channel buffer whose tail is zero).  Segment widths are multiples of 64 = the kernel's K step.
"""
import os

import torch
import torch.nn.functional as F

from . import _ext

(EPI_BF16, EPI_RELU_BF16, EPI_F32, EPI_ACC_F32, EPI_GRU_ZR, EPI_GRU_Q, EPI_DGRAD,
 EPI_F32_NCHW) = range(8)
# split-fp32 flag OR-ed into an epilogue id (launchers.h EPI_SPL): the fp32 schedule's operands as
# bf16 [hi | lo] pair buffers, three bf16 products per conv (``split_weight``)
EPI_SPL = 32


def split_weight(wp, taps):
    """Packed fp32 weight (Npad, taps * cin) -> the split-fp32 operand (Npad, taps * 3 cin) bf16:
    per tap [w_hi | w_hi | w_lo] against the split convs' K thirds [x_hi | x_lo | x_hi]."""
    n, k = wp.shape
    w = wp.float().view(n, taps, k // taps)
    hi = w.to(torch.bfloat16)
    lo = (w - hi.float()).to(torch.bfloat16)
    return torch.cat([hi, hi, lo], 2).reshape(n, 3 * k).contiguous()


GATHER_MAX = 62   # sources of one gather_cast_ launch (csrc/kernels/gather.hip)


def gather_index(flat_ids, numels):
    """int64 element ids into the concatenation of tensors with ``numels`` elements (id ==
    sum(numels): the zero padding slot) -> gather_cast_'s int32 (source << 26 | offset) codes."""
    assert len(numels) <= GATHER_MAX and max(numels) <= 1 << 26
    starts = torch.tensor([0] + list(numels), dtype=torch.long).cumsum(0)
    ids = flat_ids.to(torch.long)
    k = torch.searchsorted(starts, ids, right=True) - 1     # source holding each id
    zero = ids >= starts[-1]
    off = ids - starts[k.clamp(max=len(numels) - 1)]
    code = (k << 26) | off
    code[zero] = 63 << 26
    return code.to(torch.int32)


def gather_cast(srcs, code, out, lo_from=-1):
    """out[i] = srcs[k][off] cast to out.dtype for code[i] = k << 26 | off (k = 63: zero);
    sources k >= lo_from (>= 0) give the split-fp32 residual v - bf16(v) instead (bf16 out):
    the native one-launch gather on the GPU; the same values by torch ops on the CPU (tests)."""
    if out.device.type == 'cuda':
        _ext.ops().gather_cast_(list(srcs), code, out, int(lo_from))
        return out
    c = code.long() & 0xFFFFFFFF
    k, off = c >> 26, c & ((1 << 26) - 1)
    starts = torch.tensor([0] + [int(t.numel()) for t in srcs], dtype=torch.long).cumsum(0)
    flat = torch.cat([t.reshape(-1).float() for t in srcs] + [torch.zeros(1)])
    if lo_from >= 0:
        lo = flat[starts[lo_from]:starts[-1]]
        flat[starts[lo_from]:starts[-1]] = lo - lo.to(torch.bfloat16).float()
    pos = torch.where(k == 63, starts[-1], starts[k.clamp(max=len(srcs) - 1)] + off)
    out.copy_(flat[pos])
    return out


def round_up(x, m):
    return (x + m - 1) // m * m


def pick_bn(cout):
    if cout <= 32:
        return 32
    if cout % 128 == 0 or cout == 126:
        return 128
    return 64


def pack_weight(w, seg_real, seg_pad, npad_mult=128, dtype=torch.bfloat16):
    """(Cout, Cin, KH, KW) -> (Npad, KH*KW*sum(seg_pad)) bf16.

    ``seg_real[i]`` input channels of the module map to a ``seg_pad[i]``-wide slot in the packed K.
    """
    cout, cin, kh, kw = w.shape
    assert sum(seg_real) == cin, (seg_real, cin)
    parts = []
    off = 0
    for r, p in zip(seg_real, seg_pad):
        part = w[:, off:off + r]
        if p > r:
            part = F.pad(part, (0, 0, 0, 0, 0, p - r))
        parts.append(part)
        off += r
    wp = torch.cat(parts, dim=1)                      # (Cout, CinPad, KH, KW)
    wp = wp.permute(0, 2, 3, 1).reshape(cout, -1)     # (Cout, KH*KW*CinPad), k = tap*CinPad + c
    npad = round_up(cout, npad_mult)
    if npad > cout:
        wp = F.pad(wp, (0, 0, 0, npad - cout))
    return wp.to(dtype).contiguous()


def pack_weight_small(w, npad_mult=128, dtype=torch.bfloat16):
    """Dense-K packing for tiny Cin: k = tap*Cin + c, padded to a multiple of 64 (one K step)."""
    cout, cin, kh, kw = w.shape
    wp = w.permute(0, 2, 3, 1).reshape(cout, kh * kw * cin)
    kp = round_up(kh * kw * cin, 64)
    wp = F.pad(wp, (0, kp - kh * kw * cin, 0, round_up(cout, npad_mult) - cout))
    return wp.to(dtype).contiguous()


def pack_weight_dgrad(w, out_real, out_pad, npad_mult=128):
    """Weights of the adjoint conv: W'[ci][tap'][co] = W[co][ci][flip(tap')]; the adjoint's input
    segments are the forward output channels (real ``out_real`` in ``out_pad`` slots)."""
    wt = w.flip(2, 3).transpose(0, 1).contiguous()   # (Cin, Cout, KH, KW)
    return pack_weight(wt, out_real, out_pad, npad_mult)


def conv_fwd(segs, wpk, bias, ksize, pad, cout, epi, outs, out_offs, aux=(), aux_offs=(),
             scale=1.0, split=0, cin_small=0, bn=None):
    """Launch the implicit-GEMM conv.  ``segs`` = [(buffer, offset, count)], ``outs`` buffers.

    The kernels address every operand through a 32-bit buffer descriptor (range-checked loads
    give the zero padding for free), so one launch covers < 2 GiB per buffer; larger batches
    (e.g. Sintel-size inference at batch 512+) are issued as batch slices."""
    limit = 1 << 31
    bmap = bias is not None and bias.dim() == 4   # per-pixel bias map (GRU epilogues)
    big = max(t.numel() * t.element_size() for t in [s[0] for s in segs] + list(outs) + list(aux)
              + ([bias] if bmap else []))
    if big >= limit:
        b = segs[0][0].shape[0]
        step = max(1, (limit - 1) * b // big)
        for b0 in range(0, b, step):
            sl = slice(b0, min(b, b0 + step))
            conv_fwd([(t[sl], o, c) for t, o, c in segs], wpk, bias[sl] if bmap else bias, ksize, pad, cout, epi,
                     [t[sl] for t in outs], out_offs, [t[sl] for t in aux], aux_offs, scale,
                     split, cin_small, bn)
        return
    ops = _ext.ops()
    ins = [s[0] for s in segs]
    ops.conv_fwd_(ins, [int(s[1]) for s in segs], [int(s[2]) for s in segs], wpk, bias,
                  int(ksize[0]), int(ksize[1]), int(pad[0]), int(pad[1]), int(cout), int(cin_small),
                  int(epi), int(bn or pick_bn(cout)), float(scale), int(split), list(outs),
                  [int(o) for o in out_offs], list(aux), [int(o) for o in aux_offs])


def nhwc(x, dtype=torch.bfloat16):
    """NCHW tensor -> contiguous (B, H, W, C) buffer."""
    return x.permute(0, 2, 3, 1).to(dtype).contiguous()


def nchw(x):
    return x.permute(0, 3, 1, 2)


def conv_wgrad(g, g_off, segs, ksize, pad, cout, dw, db=None, cin_small=0, pix_per_split=None):
    """dw (cout, kpad) fp32 += weight gradient in packed-K layout; db (cout) fp32 += bias grad.

    ``g`` is the bf16 NHWC gradient w.r.t. the conv's pre-activation output (channels
    [g_off, g_off+cout)); ``segs`` the forward input segments.
    """
    ops = _ext.ops()
    if pix_per_split is None:
        p = g.shape[0] * g.shape[1] * g.shape[2]
        # ~one full round of workgroups (256 CUs x 2 resident): split-K partials are combined
        # with fp32 atomics, whose count grows with the number of splits
        tiles = max(1, (cout + 127) // 128) * max(1, (dw.shape[1] + 127) // 128)
        splits = max(1, min(p // 128, (512 + tiles - 1) // tiles))
        pix_per_split = round_up((p + splits - 1) // splits, 64)
    ops.conv_wgrad_(g, int(g_off), [s[0] for s in segs], [int(s[1]) for s in segs],
                    [int(s[2]) for s in segs], int(ksize[0]), int(ksize[1]), int(pad[0]),
                    int(pad[1]), int(cout), int(cin_small), dw, db, int(pix_per_split))


MAX_WG_ITEMS = 32
# max partial tiles (items x K-splits) reduced into one weight-gradient tile by fp32 atomics
_WG_FANIN = int(os.environ.get('RAFT_WG_FANIN', '48'))


# weight-gradient kernel of the fused update blocks: 'taps' = tap-fused (conv_wgrad_taps.hip, one
# workgroup per (128 Cout x 64 Cin) owns every tap, halo tiles in LDS), 'tile' = packed-K tiles
_WG_IMPL = os.environ.get('RAFT_WGRAD_IMPL', 'taps')
_TAP_KERNELS = {(1, 1), (1, 5), (5, 1), (3, 3)}


def _taps_ok(in_off, in_cnt, ksize):
    return (_WG_IMPL == 'taps' and tuple(ksize) in _TAP_KERNELS
            and all(c % 64 == 0 for c in in_cnt) and all(o % 8 == 0 for o in in_off)
            and sum(int(c) for c in in_cnt) // 64 <= 16)


def conv_wgrad_taps(items, g_off, in_off, in_cnt, ksize, pad, cout, dw, db=None, splits=0,
                    split=False):
    """Tap-fused variant of :func:`conv_wgrad_multi` (segments must be multiples of 64 channels).
    Partial tiles of the ``splits`` chunk ranges are reduced deterministically (no atomics).
    ``split``: split-fp32 [hi | lo] operands (three products per item, at most 10 items)."""
    ins = [b for _, bufs in items for b in bufs]
    _ext.ops().conv_wgrad_taps_([g for g, _ in items], int(g_off), ins, [int(o) for o in in_off],
                                [int(c) for c in in_cnt], int(ksize[0]), int(ksize[1]),
                                int(pad[0]), int(pad[1]), int(cout), dw, db, int(splits),
                                bool(split))


def conv_wgrad_multi(items, g_off, in_off, in_cnt, ksize, pad, cout, dw, db=None,
                     pix_per_split=None, split=False):
    """dw / db += the weight / bias gradient summed over ``items`` = [(g, [input buffers])] of one
    conv geometry (the GRU iterations of a step), in ONE launch.  Segment i of every item is
    channels [in_off[i], in_off[i] + in_cnt[i]) of that item's i-th buffer."""
    ops = _ext.ops()
    n = len(items)
    assert 1 <= n <= MAX_WG_ITEMS
    if split or (pix_per_split is None and _taps_ok(in_off, in_cnt, ksize)):
        # split fp32: the tap-fused kernel only (three products per item)
        assert not split or n * 3 <= MAX_WG_ITEMS, 'split wgrad: at most 10 items per launch'
        ins = [b for _, bufs in items for b in bufs]
        ops.conv_wgrad_taps_([g for g, _ in items], int(g_off), ins, [int(o) for o in in_off],
                             [int(c) for c in in_cnt], int(ksize[0]), int(ksize[1]), int(pad[0]),
                             int(pad[1]), int(cout), dw, db, 0, bool(split))
        return
    if pix_per_split is None:
        g0 = items[0][0]
        p = g0.shape[0] * g0.shape[1] * g0.shape[2]
        tiles = max(1, (cout + 127) // 128) * max(1, (dw.shape[1] + 127) // 128)
        # >= ~3 resident rounds of workgroups over all items; each split's partial tile leaves
        # the chip as fp32 atomics, so no more splits than that -- and at most ~48 partial tiles
        # land on the same dw tile (a 768-way same-address atomic pile-up made the K=128 convf1
        # weight gradient 20x slower than its MFMA work)
        per_item = max(1, (768 + tiles * n - 1) // (tiles * n))
        per_item = max(1, min(per_item, _WG_FANIN // n))
        pix_per_split = round_up((p + per_item - 1) // per_item, 64)
    ins = [b for _, bufs in items for b in bufs]
    ops.conv_wgrad_multi_([g for g, _ in items], int(g_off), ins, [int(o) for o in in_off],
                          [int(c) for c in in_cnt], int(ksize[0]), int(ksize[1]), int(pad[0]),
                          int(pad[1]), int(cout), dw, db, int(pix_per_split))


def unpack_weight_grad(dw, cout, cin_real_segs, cin_pad_segs, ksize):
    """(cout, KH*KW*CinPad) packed gradient -> (Cout, Cin, KH, KW) module layout."""
    kh, kw = ksize
    cin_pad = sum(cin_pad_segs)
    g = dw.view(cout, kh, kw, cin_pad).permute(0, 3, 1, 2)
    parts = []
    off = 0
    for r, p in zip(cin_real_segs, cin_pad_segs):
        parts.append(g[:, off:off + r])
        off += p
    return torch.cat(parts, dim=1) if len(parts) > 1 else parts[0].contiguous()


def unpack_weight_grad_small(dw, cout, cin, ksize):
    kh, kw = ksize
    return dw[:, :kh * kw * cin].reshape(cout, kh, kw, cin).permute(0, 3, 1, 2).contiguous()
