"""Fused HIP update block for RAFT (full model): motion encoder + SepConvGRU + flow/mask heads.

Reference: `core/update.py:79-136` (BasicMotionEncoder, SepConvGRU, FlowHead, mask head) executed
once per GRU iteration under autocast.  Eager PyTorch runs ~110 ATen ops per iteration forward and
~280 forward+backward (cat, cast, conv, bias-grad reductions, sigmoid/tanh/mul/add and their
adjoints); on MI355X the step is dominated by per-kernel overhead rather than FLOPs.

This module runs one iteration as ONE autograd node built from the hand-written gfx950 kernels:

forward (12 MFMA implicit-GEMM convs + 1 prep kernel, NHWC bf16, fp32 accumulation)::

    corr(384, from the lookup kernel) -c1(1x1,relu)-> c1(256) -c2(3x3,relu)-> cf[0:192]
    flow -patch-> 7x7x2 im2col(128) -f1(as 1x1, relu)-> f1(128) -f2(3x3,relu)-> cf[192:256]
    cf -conv(3x3,relu)-> mf[0:126] ; mf[126:128] = flow
    [h | inp | mf] -zr1(1x5, sigmoid epilogue)-> z1, r1, r1*h
    [r1*h | inp | mf] -q1(1x5, tanh + GRU-update epilogue)-> h1, q1         (same for 5x1 -> h2)
    h2 -head(3x3, relu; flow_head.conv1 | mask.0 fused N=512)-> fm(512)
    fm[0:256] -fh2(3x3, VALU dot2 kernel)-> delta (fp32, NCHW)
    fm[256:512] -mask.2(1x1, x0.25)-> mask (NHWC bf16)

backward: bf16 pre-activation gradients from fused elementwise kernels (relu / GRU gate algebra),
dgrad = the same conv kernel on flipped/transposed weights writing fp32 gradients into channel
slices (virtual concat outputs, store or accumulate), wgrad = the split-K MFMA kernel with
transposing LDS reads accumulating into per-step fp32 packed weight-gradient buffers.

Weights are packed once per forward pass by ``_UpdateWeights`` whose backward (run by autograd
after every iteration's backward) unpacks the accumulated packed gradients into the nn.Conv2d
``.grad`` tensors -- the checkpoint layout is unchanged.
"""
import os

import torch

from . import _ext
from . import conv as C
from ..utils.utils import coords_grid

HD = 128  # hidden / context width of the full model
CORR_BUF = 384  # lookup taps (4 x 81 = 324) zero-padded to a multiple of the conv K step (64)


class _LayerSpec:
    """Geometry of one conv of the fused block."""

    def __init__(self, name, cout, ksize, in_real, in_pad, small=False, relu=False, scale=1.0,
                 patch=False, row_pad=None, adj_pad=None, adj_off=0, in_sel=None, no_bias=False):
        self.name = name
        # in_sel: [(start, count)] input-channel ranges of the module weight this conv uses (one
        # module conv split over two fused convs); no_bias: the module bias belongs to the other
        self.in_sel = in_sel
        self.no_bias = no_bias
        # row_pad: per source module, its output rows are zero-padded to this many (a hidden width
        # of 96 carried in 128-channel buffers); adj_pad / adj_off: K width of the adjoint (dgrad)
        # conv's input segment and where this layer's output channels sit inside it (the adjoint
        # input must be a multiple of 64 channels wide)
        self.row_pad = row_pad
        self.adj_pad = adj_pad
        self.adj_off = adj_off
        # patch: the conv runs as a 1x1 conv over a tap-major im2col patch buffer whose K order is
        # the dense-K packing of the small-Cin weight (convf1: 7x7x2 -> 98 of 128 channels)
        self.patch = patch
        self.cout = cout
        self.k = ksize
        self.pad = (ksize[0] // 2, ksize[1] // 2)
        self.in_real = in_real
        self.in_pad = in_pad
        self.small = small
        self.relu = relu
        self.scale = scale


_HM = [(0, HD), (2 * HD, 128)]   # [h | mf] channels of a ConvGRU conv's module weight
_CTX = [(HD, HD)]                # its context (inp) channels

SPECS = [
    _LayerSpec('c1', 256, (1, 1), [324], [CORR_BUF]),
    _LayerSpec('c2', 192, (3, 3), [256], [256]),
    _LayerSpec('f1', 128, (7, 7), [2], [8], small=True, patch=True),
    _LayerSpec('f2', 64, (3, 3), [128], [128]),
    _LayerSpec('conv', 126, (3, 3), [256], [256]),
    # ConvGRU convs over [h | inp | mf]: the per-iteration conv reads [h | mf] only; the context
    # part (inp: the same tensor in every iteration) is the '<name>i' conv, run ONCE per forward
    # into a per-pixel fp32 bias map, and once per backward on the iterations' summed
    # pre-activation gradients (linearity: sum_t conv_T(g_t) = conv_T(sum_t g_t))
    _LayerSpec('zr1', 256, (1, 5), [128, 128], [128, 128], in_sel=_HM, no_bias=True),
    _LayerSpec('q1', 128, (1, 5), [128, 128], [128, 128], in_sel=_HM, no_bias=True),
    _LayerSpec('zr2', 256, (5, 1), [128, 128], [128, 128], in_sel=_HM, no_bias=True),
    _LayerSpec('q2', 128, (5, 1), [128, 128], [128, 128], in_sel=_HM, no_bias=True),
    _LayerSpec('head', 512, (3, 3), [128], [128]),
    _LayerSpec('fh2', 2, (3, 3), [256], [256]),
    _LayerSpec('m2', 576, (1, 1), [256], [256], scale=0.25),
    _LayerSpec('zr1i', 256, (1, 5), [128], [128], in_sel=_CTX),
    _LayerSpec('q1i', 128, (1, 5), [128], [128], in_sel=_CTX),
    _LayerSpec('zr2i', 256, (5, 1), [128], [128], in_sel=_CTX),
    _LayerSpec('q2i', 128, (5, 1), [128], [128], in_sel=_CTX),
]
GRU_CONVS = ('zr1', 'q1', 'zr2', 'q2')
SPEC = {s.name: s for s in SPECS}


class Design:
    """A fused update block: its layer specs and where their parameters live in the module."""

    def __init__(self, specs, module_params):
        self.specs = specs
        self.spec = {s.name: s for s in specs}
        self.module_params = module_params

    def flat_params(self, ub):
        """Module parameters in spec order, each once (a module conv may feed two specs)."""
        mp = self.module_params(ub)
        out, seen = [], set()
        for s in self.specs:
            for w, b in mp[s.name]:
                if id(w) in seen:
                    continue
                seen.add(id(w))
                out += [w, b]
        return out


def module_params(ub):
    """(weight, bias) tensors of each fused layer, in SPECS order, from a BasicUpdateBlock."""
    e, g, fh, mk = ub.encoder, ub.gru, ub.flow_head, ub.mask
    return {
        'c1': [(e.convc1.weight, e.convc1.bias)],
        'c2': [(e.convc2.weight, e.convc2.bias)],
        'f1': [(e.convf1.weight, e.convf1.bias)],
        'f2': [(e.convf2.weight, e.convf2.bias)],
        'conv': [(e.conv.weight, e.conv.bias)],
        'zr1': [(g.convz1.weight, g.convz1.bias), (g.convr1.weight, g.convr1.bias)],
        'q1': [(g.convq1.weight, g.convq1.bias)],
        'zr2': [(g.convz2.weight, g.convz2.bias), (g.convr2.weight, g.convr2.bias)],
        'q2': [(g.convq2.weight, g.convq2.bias)],
        'head': [(fh.conv1.weight, fh.conv1.bias), (mk[0].weight, mk[0].bias)],
        'fh2': [(fh.conv2.weight, fh.conv2.bias)],
        'm2': [(mk[2].weight, mk[2].bias)],
        'zr1i': [(g.convz1.weight, g.convz1.bias), (g.convr1.weight, g.convr1.bias)],
        'q1i': [(g.convq1.weight, g.convq1.bias)],
        'zr2i': [(g.convz2.weight, g.convz2.bias), (g.convr2.weight, g.convr2.bias)],
        'q2i': [(g.convq2.weight, g.convq2.bias)],
    }


FULL = Design(SPECS, module_params)


def flat_params(ub, design=FULL):
    return design.flat_params(ub)


def _pack_layers(params_by_layer, need_grad, dtype, design=FULL, spl=False):
    """Kernel-layout weights of every fused conv: ({name: forward [Npad][K]}, {name: adjoint
    [Npad'][K']}, {name: bias}, {extra tables}).  Runs on real parameters or on index tensors
    (``_PackPlan``).  Extras: flow_head.conv2's bf16 pair tables for its VALU kernels, forward
    [t][o][c] and adjoint [t][c][o].  ``spl`` (the fp32 schedule): flow_head.conv2 runs on the
    MFMA conv kernels too, so its adjoint is packed (64-wide K slot of its 2 output channels)."""
    w_out, wd_out, b_out, x_out = {}, {}, {}, {}
    w_mod = {}   # per layer: the module weight as the fused conv sees it (in_sel / row_pad applied)
    F_ = torch.nn.functional
    for s in design.specs:
        ws = [w for w, _ in params_by_layer[s.name]]
        bs = [b for _, b in params_by_layer[s.name]]
        if s.in_sel is not None:
            ws = [torch.cat([w[:, a:a + n] for a, n in s.in_sel], 1) for w in ws]
        if s.no_bias:
            bs = [torch.zeros_like(b) for b in bs]
        if s.row_pad is not None:
            ws = [F_.pad(w, (0, 0, 0, 0, 0, 0, 0, s.row_pad - w.shape[0])) for w in ws]
            bs = [F_.pad(b, (0, s.row_pad - b.shape[0])) for b in bs]
        w = ws[0] if len(ws) == 1 else torch.cat(ws, 0)
        w_mod[s.name] = w
        b_out[s.name] = bs[0] if len(bs) == 1 else torch.cat(bs, 0)
        if s.small:
            w_out[s.name] = C.pack_weight_small(w, dtype=dtype)
        else:
            w_out[s.name] = C.pack_weight(w, s.in_real, s.in_pad, dtype=dtype)
        no_adj = design is FULL and s.name in _NO_ADJOINT and not (spl and s.name == 'fh2')
        if need_grad and not s.patch and not no_adj:
            # adjoint conv: inputs = this layer's output channels, outputs = its inputs
            cout_pad = s.adj_pad or C.round_up(s.cout, 32)
            if spl and s.name == 'fh2':
                cout_pad = 64
            wt = w
            if cout_pad > s.cout:
                wt = F_.pad(w, (0, 0, 0, 0, 0, 0, s.adj_off, cout_pad - s.cout - s.adj_off))
            wt = wt.flip(2, 3).transpose(0, 1).contiguous()  # (Cin, CoutPad, kh, kw)
            if sum(s.in_pad) > sum(s.in_real):
                # padded input slots become zero output rows of the adjoint
                parts, off = [], 0
                for r, p in zip(s.in_real, s.in_pad):
                    part = wt[off:off + r]
                    if p > r:
                        part = torch.nn.functional.pad(part, (0, 0, 0, 0, 0, 0, 0, p - r))
                    parts.append(part)
                    off += r
                wt = torch.cat(parts, 0)
            wd_out[s.name] = C.pack_weight(wt, [cout_pad], [cout_pad], dtype=dtype)
        if design is FULL and s.name == 'fh2':
            x_out['fh2f'] = w.permute(2, 3, 0, 1).reshape(18, 256).to(dtype)
            x_out['fh2d'] = w.permute(2, 3, 1, 0).reshape(9, 512).to(dtype)
    if need_grad and design is FULL:
        for tag in ('1', '2'):
            x_out['zrq' + tag] = _zrq_adjoint(w_mod['zr' + tag], w_mod['q' + tag], dtype)
    return w_out, wd_out, b_out, x_out


# layers whose plain adjoint is never packed: fh2 runs on its own VALU kernels, the z|r convs'
# input gradient is part of the combined z|r + q adjoint (_zrq_adjoint)
_NO_ADJOINT = ('fh2', 'zr1', 'zr2')


def _zrq_adjoint(w_zr, w_q, dtype):
    """Input gradient of a GRU half-step's z|r conv AND the motion-feature part of its q conv as
    ONE conv: inputs [d pre-z|r (256) | d pre-q (128)], outputs [dh (128) | d mf (128)].  The q
    conv reads [r*h | mf]; the gradient of r*h takes the gate path (OSeg gate 2), so the dh rows
    are zero over the d pre-q columns and their output tiles run only the K prefix of d pre-z|r
    (OSeg.kcin).  d mf gets both convs' contributions in one fp32 MFMA accumulation: no
    read-modify-write pass of the fp32 motion-feature gradient between the two convs
    (`core/update.py:45-60`)."""
    a_zr = w_zr.flip(2, 3).transpose(0, 1)             # (256 [h | mf], 256 [z | r], kh, kw)
    a_q = w_q.flip(2, 3).transpose(0, 1).clone()        # (256 [rh | mf], 128, kh, kw)
    a_q[:HD] = 0                                        # 0 = padding in the index-tensor plans
    wt = torch.cat([a_zr, a_q], 1).contiguous()         # (256, 384, kh, kw)
    return C.pack_weight(wt, [3 * HD], [3 * HD], dtype=dtype)


class _PackPlan:
    """Index maps that turn the 24 update-block parameters into every packed weight (forward and
    adjoint, bf16) with ONE gather + cast, and the packed fp32 weight/bias gradients back into
    the parameters' layout with one gather -- instead of ~100 small pad / permute / flip / cat /
    cast kernels per training step.  Built once per parameter geometry by running the packing
    code on index tensors (float64 holds the element ids exactly; 0 marks zero padding)."""

    def __init__(self, ub, need_grad, device, design=FULL, spl=False):
        SPECS = design.specs
        module_params = design.module_params
        params = design.flat_params(ub)
        self.numels = [p.numel() for p in params]
        self.shapes = [tuple(p.shape) for p in params]
        total = sum(self.numels)
        ids, off = [], 0
        for p in params:
            ids.append((torch.arange(p.numel(), dtype=torch.float64) + off + 1).view(p.shape))
            off += p.numel()
        idmap = {id(p): t for p, t in zip(params, ids)}
        by_layer = {s.name: [(idmap[id(w)], idmap[id(b)]) for w, b in module_params(ub)[s.name]]
                    for s in SPECS}
        w_idx, wd_idx, b_idx, x_idx = _pack_layers(by_layer, need_grad, torch.float64, design, spl)
        # gather index: element id - 1; padding (id 0) -> the zero slot appended after the params
        self.views = []       # (kind, name, shape) in gather order
        parts = []
        for kind, d in (('w', w_idx), ('wd', wd_idx), ('x', x_idx)):
            for name in [s.name for s in SPECS] + sorted(x_idx):
                if name in d:
                    t = d[name]
                    self.views.append((kind, name, tuple(t.shape)))
                    parts.append(t.reshape(-1))
        gidx = torch.cat(parts).round().long() - 1
        gidx[gidx < 0] = total
        # (parameter, offset) codes of the native gather: the parameters are read in place
        widx = C.gather_index(gidx, self.numels)
        if spl:
            widx, self.views = self._split_codes(widx, design)
        self.widx = widx.to(device)
        self.bshapes = [(s.name, b_idx[s.name].numel()) for s in SPECS]
        bidx = torch.cat([b_idx[s.name].reshape(-1) for s in SPECS]).round().long() - 1
        bidx[bidx < 0] = total   # padded rows (row_pad) read the zero slot
        self.bidx = C.gather_index(bidx, self.numels).to(device)
        self.kpad = {s.name: w_idx[s.name].shape[1] for s in SPECS}
        # gradient buffer: per layer dw (cout, kpad) then db (cout), concatenated in SPECS order;
        # uidx[e] = the buffer position holding parameter element e's gradient
        uidx = torch.full((total,), -1, dtype=torch.long)
        self.dw_views = []
        pos = 0
        for s in SPECS:
            ids_w = w_idx[s.name][:s.cout].round().long() - 1        # (cout, kpad)
            n = ids_w.numel()
            m = ids_w.reshape(-1) >= 0
            uidx[ids_w.reshape(-1)[m]] = torch.arange(pos, pos + n)[m]
            self.dw_views.append((s.name, 'w', pos, (s.cout, self.kpad[s.name])))
            pos += n
            ids_b = b_idx[s.name].round().long() - 1
            mb = ids_b >= 0   # padded output rows (row_pad) have no parameter
            uidx[ids_b[mb]] = torch.arange(pos, pos + s.cout)[mb]
            self.dw_views.append((s.name, 'b', pos, (s.cout,)))
            pos += s.cout
        assert (uidx >= 0).all(), 'every parameter element must have a gradient slot'
        self.dw_total = pos
        self.uidx = C.gather_index(uidx, [pos]).to(device)   # single source: the gradient buffer


    def _split_codes(self, widx, design):
        """The fp32 schedule's packs straight from the parameters: per tap [w_hi | w_hi | w_lo]
        (C.split_weight's layout) with the w_lo codes on the residual sources n..2n-1 of the
        gather (lo_from = n); the VALU flow-head tables stay plain bf16 casts."""
        n_src = len(self.numels)
        c = widx.long() & 0xFFFFFFFF
        parts, views, off = [], [], 0
        for kind, name, shape in self.views:
            n = shape[0] * shape[1]
            cv = c[off:off + n].view(shape)
            off += n
            if name in ('fh2f', 'fh2d'):
                parts.append(cv.reshape(-1))
                views.append((kind, name, shape))
                continue
            t = _taps_of(design, kind, name)
            cv3 = cv.view(shape[0], t, shape[1] // t)
            lo = torch.where((cv3 >> 26) == 63, cv3, cv3 + (n_src << 26))
            parts.append(torch.cat([cv3, cv3, lo], 2).reshape(-1))
            views.append((kind, name, (shape[0], 3 * shape[1])))
        sc = torch.cat(parts)
        sc = torch.where(sc >= 2 ** 31, sc - 2 ** 32, sc)   # uint32 codes as int32
        return sc.to(torch.int32), views


def _plan(ub, need_grad, device, design=FULL, spl=False):
    key = (need_grad, str(device), tuple(tuple(p.shape) for p in design.flat_params(ub)), spl)
    cache = ub.__dict__.setdefault('_raft_pack_plans', {})
    if key not in cache:
        cache[key] = _PackPlan(ub, need_grad, device, design, spl)
    return cache[key]


def _taps_of(design, kind, name):
    """Filter taps of a packed weight view (its K = taps x input channels)."""
    if kind == 'x':
        return design.spec['zr' + name[-1]].k[0] * design.spec['zr' + name[-1]].k[1] \
            if name.startswith('zrq') else 1
    s = design.spec[name]
    if kind == 'w' and s.patch:
        return 1
    return s.k[0] * s.k[1]


class _Packed:
    """Per-step packed weights (bf16, fp16, or -- dtype fp32, the fp32 schedule -- split-fp32
    [w_hi | w_hi | w_lo] bf16 per tap) + packed fp32 gradient accumulators."""

    def defer_wgrad(self, name, g, g_off, segs):
        self.pending.setdefault(name, []).append((g, g_off, segs))

    def __init__(self, ub, params, device, need_grad, design=FULL, dtype=torch.bfloat16):
        self.design = design
        self.dtype = dtype   # operand dtype: bf16, fp16 autocast, or fp32 (split bf16 pairs)
        self.spl = dtype == torch.float32
        self.w = {}
        self.wd = {}
        self.x = {}
        self.b = {}
        self.dw = {}
        self.db = {}
        self.pending = {}  # conv name -> [(g, g_off, segs)] awaiting the batched weight gradient
        self.fh2_items = []  # (fp32 delta gradient, head activations) per iteration
        self.ctx = None      # GRU conv -> bf16 (B,H,W,cout) context bias map (see ctx_maps)
        self.ctx_key = None
        self.device = device
        plan = self.plan = _plan(ub, need_grad, device, design, self.spl)
        self.kpad = plan.kpad
        with torch.no_grad():
            srcs = [p.detach().float().contiguous() for p in params]
            # every kernel-layout weight in ONE gather + cast launch (csrc/kernels/gather.hip);
            # fp32 schedule: straight into the split [w_hi | w_hi | w_lo] packs (residual
            # halves from the second copy of the sources)
            packed = torch.empty(plan.widx.numel(), device=device,
                                 dtype=torch.bfloat16 if self.spl else dtype)
            if self.spl:
                C.gather_cast(srcs + srcs, plan.widx, packed, lo_from=len(srcs))
            else:
                C.gather_cast(srcs, plan.widx, packed)
            off = 0
            for kind, name, shape in plan.views:
                n = shape[0] * shape[1]
                {'w': self.w, 'wd': self.wd, 'x': self.x}[kind][name] = packed[off:off + n].view(shape)
                off += n
            bias = torch.empty(plan.bidx.numel(), device=device)
            C.gather_cast(srcs, plan.bidx, bias)
            off = 0
            for name, n in plan.bshapes:
                self.b[name] = bias[off:off + n]
                off += n
            # 256 -> 2 conv: dedicated VALU kernels read bf16 pair tables
            if design is FULL:
                self.fh2_wf, self.fh2_wd = self.x['fh2f'], self.x['fh2d']
            self.b32 = self.b['fh2']
            if need_grad:
                self.dwflat = torch.zeros(plan.dw_total, device=device)
                for name, kind, pos, shape in plan.dw_views:
                    n = shape[0] * (shape[1] if len(shape) > 1 else 1)
                    (self.dw if kind == 'w' else self.db)[name] = \
                        self.dwflat[pos:pos + n].view(shape)


def _flush_wgrad(pk):
    """Weight gradients of every deferred (conv, iteration) item: one multi-item launch per conv
    (the weights are shared by all iterations; convf1 as a 1x1 conv over its patch buffers),
    the flow-head conv2 by its own VALU kernel (split fp32: by the tap-fused MFMA kernel, three
    products per item, so at most MAX_WG_ITEMS / 3 items per launch)."""
    spl = pk.spl
    for name, items in pk.pending.items():
        s = pk.design.spec[name]
        dw, db = pk.dw[name], pk.db[name]
        k, pad, small = ((1, 1), (0, 0), False) if s.patch else (s.k, s.pad, s.small)
        same = all(it[1] == items[0][1] and [(o, c) for _, o, c in it[2]] ==
                   [(o, c) for _, o, c in items[0][2]] for it in items)
        cnts = [c for _, _, c in items[0][2]]
        offs = [o for _, o, _ in items[0][2]]
        batched = C._taps_ok(offs, cnts, k) or not any(c % 128 for c in cnts)
        if spl:
            assert same and not small, 'split wgrad items must share one layout'
            g_off = items[0][1]
            in_off = [o for _, o, _ in items[0][2]]
            in_cnt = [c for _, _, c in items[0][2]]
            per = C.MAX_WG_ITEMS // 3
            for i in range(0, len(items), per):
                chunk = items[i:i + per]
                C.conv_wgrad_multi([(g, [b for b, _, _ in segs]) for g, _, segs in chunk], g_off,
                                   in_off, in_cnt, k, pad, s.cout, dw, db, split=True)
            continue
        if small or not same or not batched:
            for g, g_off, segs in items:
                C.conv_wgrad(g, g_off, segs, k, pad, s.cout, dw, db, cin_small=2 if small else 0)
            continue
        g_off = items[0][1]
        in_off = [o for _, o, _ in items[0][2]]
        in_cnt = [c for _, _, c in items[0][2]]
        for i in range(0, len(items), C.MAX_WG_ITEMS):
            chunk = items[i:i + C.MAX_WG_ITEMS]
            C.conv_wgrad_multi([(g, [b for b, _, _ in segs]) for g, _, segs in chunk], g_off,
                               in_off, in_cnt, k, pad, s.cout, dw, db)
    pk.pending = {}
    items = pk.fh2_items
    for i in range(0, len(items), 32):
        chunk = items[i:i + 32]
        g0 = chunk[0][0]
        units = len(chunk) * g0.shape[0] * ((g0.shape[2] + 7) // 8)
        # one partial [dw | db] row per workgroup, summed here (deterministic, no atomics)
        part = torch.empty(min(units, 512), 2 * 9 * 256 + 2, device=g0.device)
        _ext.ops().fh2_wgrad_([g for g, _ in chunk], [x for _, x in chunk], part)
        ps = part.sum(0)
        pk.dw['fh2'].add_(ps[:2 * 9 * 256].view(2, 9 * 256))
        pk.db['fh2'].add_(ps[2 * 9 * 256:])
    pk.fh2_items = []


class _State:
    def __init__(self):
        self.packed = None
        self.overlap = False
        self.params = []
        self.n_iter = 0        # iterations issued through this block (forward order)
        self.next_bwd = None   # iteration whose backward must run next (strictly n_iter-1 .. 0)
        self.dh_carry = None   # fp32 gradient of the next-to-run iteration's output state
        self.zero_h = None     # bf16 scalar zero, broadcast as the stand-in h gradient
        self.dinp_acc = None   # fp32 gradient w.r.t. the context input, summed over iterations
        self.ctx_g = {}        # GRU conv -> its pre-activation gradients of the iterations run
        self.design = FULL
        self.dtype = torch.bfloat16  # operand dtype (fp16 under fp16 autocast, fp32 split pairs)


class _UpdateWeights(torch.autograd.Function):
    @staticmethod
    def forward(ctx, state, *params):
        state.packed = _Packed(state.ub, params, params[0].device, need_grad=state.need_grad,
                               design=state.design, dtype=state.dtype)
        ctx.state = state
        ctx.n = len(params)
        return params[0].new_zeros(())

    @staticmethod
    def backward(ctx, _tok):
        st = ctx.state
        if st.dinp_acc is not None or st.ctx_g:
            # the context gradient is handed to autograd by iteration 0's backward; a partial
            # backward (autograd.grad over a subset of the iterations) would silently drop it
            raise RuntimeError('fused update block: the backward must run through every GRU '
                               'iteration down to iteration 0 (partial autograd.grad over the '
                               'iterations is not supported; use update_impl="torch")')
        pk = st.packed
        st.packed = None
        if st.overlap and pk.device.type == 'cuda':
            return _backward_overlapped(st, pk, ctx.n)
        _flush_wgrad(pk)
        return (None, *_unpack_grads(pk))


def _unpack_grads(pk):
    """Packed fp32 gradients -> one tensor per parameter (module layout), one gather."""
    for s in pk.design.specs:
        if s.scale != 1.0:
            pk.dw[s.name].mul_(s.scale)
            pk.db[s.name].mul_(s.scale)
    plan = pk.plan
    g = torch.empty(plan.uidx.numel(), device=pk.dwflat.device)
    C.gather_cast([pk.dwflat], plan.uidx, g)
    grads, off = [], 0
    for n, shape in zip(plan.numels, plan.shapes):
        grads.append(g[off:off + n].view(shape))
        off += n
    return grads


# ---------------------------------------------------------------- wgrad / encoder-backward overlap
# The batched weight gradients (~15 % of a training step, MFMA-bound) depend on nothing the rest
# of the backward produces, while the encoder backward that follows them (MIOpen convs + norm
# passes) is mostly memory-bound.  With overlap enabled (set_wgrad_overlap; the trainer turns it
# on) the flush runs on a side HIP stream concurrently with the rest of the backward, and the
# update-block parameter gradients are written into ``.grad`` by an end-of-backward callback
# after the main stream has joined the side stream -- so every consumer (optimizer, clip, RCCL
# bucket sync, which launches never-hooked buckets in ``finish``) sees finished gradients.
# Off by default: a plain autograd.grad() caller must get the gradients as return values.
_OVERLAP = False
_SIDE = {}


def set_wgrad_overlap(enabled):
    global _OVERLAP
    _OVERLAP = bool(enabled)


def _side_stream(dev):
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def _backward_overlapped(st, pk, n):
    dev = pk.device
    main = torch.cuda.current_stream(dev)
    side = _side_stream(dev)
    side.wait_stream(main)
    # everything the side stream reads was allocated on the main stream: keep it from being
    # recycled by main-stream allocations until the side stream is done with it
    for items in pk.pending.values():
        for g, _, segs in items:
            g.record_stream(side)
            for buf, _, _ in segs:
                buf.record_stream(side)
    for g, x in pk.fh2_items:
        g.record_stream(side)
        x.record_stream(side)
    pk.dwflat.record_stream(side)
    params = st.params
    with torch.cuda.stream(side):
        _flush_wgrad(pk)
        # .grad is assigned directly (no AccumulateGrad): match each parameter's strides, as
        # AccumulateGrad's layout contract would (fused optimizers require it)
        grads = [g if g.stride() == prm.stride() else torch.empty_like(prm).copy_(g)
                 for prm, g in zip(params, _unpack_grads(pk))]

    def _join():
        main.wait_stream(side)
        with torch.no_grad():
            for prm, g in zip(params, grads):
                if not prm.requires_grad:
                    continue
                g.record_stream(main)
                if prm.grad is None:
                    prm.grad = g
                else:
                    prm.grad.add_(g)

    torch.autograd.Variable._execution_engine.queue_callback(_join)
    return (None,) * (1 + n)


# ---------------------------------------------------------------- independent branches
# Each conv of an iteration is small (34k pixels at batch 12) and latency-bound, so two
# independent chains run concurrently on a second HIP stream and fill the CUs the other leaves
# idle: forward -- motion encoder flow branch (f1 -> f2) || correlation branch (c1 -> c2), mask
# conv m2 || flow-head conv fh2; backward -- m2 dgrad || fh2 dgrad, f2 dgrad || c2 -> c1 dgrad.
# Every buffer the branch touches is allocated on the main stream before the fork and stays
# referenced until after the join, so the caching allocator never hands it out while the branch
# runs.  Captured into the training hipGraph as parallel branches.
# OFF by default (RAFT_UPDATE_BRANCHES=1 enables it): measured 381-383 vs 397-398 pairs/s
# without -- co-running convs slow each other more than the overlap gains (kernel sum per step
# 31.0 -> 33.0 ms: the XCD-local tile order and L2 reuse of each conv are lost when two grids
# share the XCDs).  Round 6 re-check with the persisted tile table: 471.3 / 475.1 vs 476.0 / 478.3
# pairs/s (profiles/r6/r6i/ab_*.log) -- still off.
_BRANCHES = os.environ.get('RAFT_UPDATE_BRANCHES', '0') == '1'
# ConvGRU gate backward (gru_q_bwd / gru_zr_bwd) fused into the dgrad epilogues (OSeg.gate);
# RAFT_GRU_GATES_FUSED=0 runs the separate elementwise kernels
_GATES_FUSED = os.environ.get('RAFT_GRU_GATES_FUSED', '1') != '0'
_BRANCH = {}


class _Branch:
    def __init__(self, dev):
        self.side = None
        if _BRANCHES and dev.type == 'cuda':
            key = dev.index if dev.index is not None else torch.cuda.current_device()
            if key not in _BRANCH:
                _BRANCH[key] = torch.cuda.Stream(device=dev)
            self.side = _BRANCH[key]
            self.main = torch.cuda.current_stream(dev)
            self.side.wait_stream(self.main)

    def __enter__(self):
        if self.side is not None:
            self._ctx = torch.cuda.stream(self.side)
            self._ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.side is not None:
            self._ctx.__exit__(*exc)
        return False

    def join(self):
        if self.side is not None:
            self.main.wait_stream(self.side)


def _bf16(shape, dev, dt=torch.bfloat16):
    """16-bit activation buffer: bf16, or fp16 under fp16 autocast (the operand dtype of a step);
    dt fp32 (the fp32 schedule): a bf16 [hi | lo] pair buffer of twice the channels, the value
    being hi + lo (split fp32, ~2^-16 relative)."""
    if dt == torch.float32:
        return torch.empty(*shape[:-1], 2 * shape[-1], device=dev, dtype=torch.bfloat16)
    return torch.empty(*shape, device=dev, dtype=dt)


def _to_split(x32, buf=None):
    """fp32 (B,C,H,W) tensor of any strides (an NHWC tensor as .permute(0, 3, 1, 2)) -> split
    bf16 NHWC [hi | lo] (B,H,W,2C) (csrc/kernels/update_ew.hip split_hilo_kernel)."""
    b, c, h, w = x32.shape
    if buf is None:
        buf = torch.empty(b, h, w, 2 * c, device=x32.device, dtype=torch.bfloat16)
    _ext.ops().split_hilo_(x32, buf)
    return buf


def _from_split(xs):
    """split bf16 NHWC [hi | lo] (B,H,W,2C) -> fp32 NHWC (B,H,W,C)."""
    c = xs.shape[-1] // 2
    return xs[..., :c].float() + xs[..., c:].float()


class _SplitNHWC(torch.autograd.Function):
    """fp32 (B,C,H,W) -> split-fp32 NHWC operand (B,H,W,2 cpad) bf16 [hi | lo], channels past C
    zero; the gradient arrives split-encoded the same way and leaves as fp32 (B,C,H,W)."""

    @staticmethod
    def forward(ctx, x, cpad):
        b, c, h, w = x.shape
        ctx.c = c
        buf = torch.empty(b, h, w, 2 * cpad, device=x.device, dtype=torch.bfloat16)
        return _to_split(x.float(), buf)

    @staticmethod
    def backward(ctx, gs):
        g = _from_split(gs)[..., :ctx.c]
        return g.permute(0, 3, 1, 2), None


def split_nhwc(x, cpad=None):
    """Autograd-aware fp32 (B,C,H,W) -> split-fp32 NHWC operand of the fused update block's
    fp32 schedule (``HipUpdateBlock(dtype=torch.float32)``)."""
    return _SplitNHWC.apply(x, cpad or x.shape[1])


def _f32(shape, dev, zero=False):
    return (torch.zeros if zero else torch.empty)(*shape, device=dev, dtype=torch.float32)


# RAFT_CTX_BF16=0: fp32 context maps (A/B; bf16 halves the maps' per-iteration reads -- 1.5 KB per
# pixel and iteration -- at the rounding the GRU pre-activations see anyway)
_CTX_BF16 = os.environ.get('RAFT_CTX_BF16', '1') != '0'


def ctx_maps(pk, inp):
    """Context part of the four ConvGRU convs, conv(inp, W_inp) + bias as bf16 (fp32 with
    RAFT_CTX_BF16=0) (B,H,W,cout) maps -- computed once per forward pass (the iterations share
    ``inp``) and added by the iterations' GRU epilogues."""
    key = (inp.data_ptr(), tuple(inp.shape), inp._version)
    if pk.ctx is not None:
        if key != pk.ctx_key:
            raise RuntimeError('fused update block: every iteration of a forward pass must take '
                               'the same context tensor')
        return pk.ctx
    B, H, W, _ = inp.shape
    pk.ctx = {}
    c16 = _CTX_BF16 and not pk.spl   # split fp32: fp32 maps
    for name in GRU_CONVS:
        s = SPEC[name + 'i']
        m = torch.empty(B, H, W, s.cout, device=inp.device,
                        dtype=inp.dtype if c16 else torch.float32)
        C.conv_fwd([(inp, 0, HD)], pk.w[s.name], pk.b[s.name], s.k, s.pad, s.cout,
                   (C.EPI_BF16 if c16 else C.EPI_F32) | (C.EPI_SPL if pk.spl else 0), [m], [0])
        pk.ctx[name] = m
    pk.ctx_key = key
    return pk.ctx


def _sum_bf16(gs, spl=False):
    """bf16 sum (fp32 accumulation) of same-shape bf16 tensors (split fp32 pairs: the hi and lo
    halves summed in fp32, then recombined and re-split)."""
    ops = _ext.ops()
    n = _ext.SUM_MAX
    if spl:
        acc = torch.empty(gs[0].shape, device=gs[0].device, dtype=torch.float32)
        for i in range(0, len(gs), n):
            ops.sum_bf16_(gs[i:i + n], acc if i else None, acc)
        return _to_split(_from_split(acc).permute(0, 3, 1, 2))
    out = torch.empty_like(gs[0])
    if len(gs) <= n:
        ops.sum_bf16_(gs, None, out)
        return out
    carry = torch.empty(gs[0].shape, device=gs[0].device, dtype=torch.float32)
    ops.sum_bf16_(gs[:n], None, carry)
    for i in range(n, len(gs), n):
        ops.sum_bf16_(gs[i:i + n], carry, out if i + n >= len(gs) else carry)
    return out


def _iter_forward(pk, h, inp, corr, flow, need_mask=True, coords=None):
    """Forward of one fused iteration; returns (h2, delta, mask, saved tensors, upd).

    ``need_mask=False`` (inference iterations whose flow is not upsampled) computes only the
    flow-head half of the fused head conv and skips the mask conv: ~20 % of the iteration.
    ``coords`` (the iteration's detached coords1, (B,2,H,W) fp32): ``upd`` = (coords1 + delta,
    coords1 + delta - coords0) of `core/raft.py:134-135`, written by the flow-head kernel (two
    fewer launches per iteration); None without coords."""
    B, H, W, _ = h.shape
    dev = h.device
    dt = pk.dtype  # operand dtype: bf16, fp16 autocast, or fp32 (split bf16 pair buffers)
    spl = pk.spl
    sh = (B, H, W)
    patch = _bf16(sh + (128,), dev, dt)  # f1_patch writes all 128 channels
    mf = _bf16(sh + (128,), dev, dt)
    ops = _ext.ops()
    ops.f1_patch_(flow, patch, mf, 126)
    c1 = _bf16(sh + (256,), dev, dt)
    cf = _bf16(sh + (256,), dev, dt)
    f1 = _bf16(sh + (128,), dev, dt)

    def conv(name, segs, epi, outs, offs, aux=(), aux_offs=(), split=0, cout=None, bias=None):
        s = SPEC[name]
        cout = cout or s.cout
        w, b = pk.w[name], (pk.b[name] if bias is None else bias)
        if cout != s.cout:  # leading output rows of a fused conv (packed rows are cout-major)
            w, b = w[:C.round_up(cout, 128)], b[:cout]
        k, pad, small = ((1, 1), (0, 0), False) if s.patch else (s.k, s.pad, s.small)
        C.conv_fwd(segs, w, b, k, pad, cout, epi | (C.EPI_SPL if spl else 0), outs, offs, aux,
                   aux_offs, scale=s.scale, split=split, cin_small=2 if small else 0)

    br = _Branch(dev)
    with br:
        conv('f1', [(patch, 0, 128)], C.EPI_RELU_BF16, [f1], [0])
        conv('f2', [(f1, 0, 128)], C.EPI_RELU_BF16, [cf], [192])
    conv('c1', [(corr, 0, CORR_BUF)], C.EPI_RELU_BF16, [c1], [0])
    conv('c2', [(c1, 0, 256)], C.EPI_RELU_BF16, [cf], [0])
    br.join()
    conv('conv', [(cf, 0, 256)], C.EPI_RELU_BF16, [mf], [0])
    gates = {}
    hin = h
    ctx = ctx_maps(pk, inp)
    for tag in ('1', '2'):
        z, rh, r = _bf16(sh + (HD,), dev, dt), _bf16(sh + (HD,), dev, dt), _bf16(sh + (HD,), dev, dt)
        conv('zr' + tag, [(hin, 0, HD), (mf, 0, 128)], C.EPI_GRU_ZR, [z, rh, r],
             [0, 0, 0], aux=[hin], aux_offs=[0], split=HD, bias=ctx['zr' + tag])
        hn, q = _bf16(sh + (HD,), dev, dt), _bf16(sh + (HD,), dev, dt)
        conv('q' + tag, [(rh, 0, HD), (mf, 0, 128)], C.EPI_GRU_Q, [hn, q], [0, 0],
             aux=[hin, z], aux_offs=[0, 0], bias=ctx['q' + tag])
        gates[tag] = (hin, z, rh, r, q)
        hin = hn
    h2 = hin
    delta = torch.empty(B, 2, H, W, device=dev, dtype=torch.float32)
    upd = None

    def fh2(fm):
        nonlocal upd
        if spl:  # split fp32: the MFMA conv kernel (NCHW fp32 epilogue), not the VALU one
            conv('fh2', [(fm, 0, 256)], C.EPI_F32_NCHW, [delta], [0])
            if coords is not None:
                cn = coords + delta
                g0 = getattr(pk, 'grid0', None)
                if g0 is None or g0.shape != cn.shape:
                    g0 = pk.grid0 = coords_grid(B, H, W, device=dev)
                upd = (cn, cn - g0)
        elif coords is not None:
            upd = (torch.empty_like(delta), torch.empty_like(delta))
            ops.fh2_fwd_(fm, pk.fh2_wf, pk.b32, delta, coords.contiguous(), upd[0], upd[1])
        else:
            ops.fh2_fwd_(fm, pk.fh2_wf, pk.b32, delta)

    if need_mask:
        fm = _bf16(sh + (512,), dev, dt)
        conv('head', [(h2, 0, HD)], C.EPI_RELU_BF16, [fm], [0])
        if spl:  # fp32 (B,H,W,576) mask for the upsampling (the fp32 schedule's precision)
            mask = torch.empty(sh + (576,), device=dev, dtype=torch.float32)
        else:
            mask = _bf16(sh + (576,), dev, dt)
        br = _Branch(dev)
        with br:
            conv('m2', [(fm, 256, 256)], C.EPI_F32 if spl else C.EPI_BF16, [mask], [0])
        fh2(fm)
        br.join()
    else:
        fm = _bf16(sh + (256,), dev, dt)
        conv('head', [(h2, 0, HD)], C.EPI_RELU_BF16, [fm], [0], cout=256)
        fh2(fm)
        mask = None
    g1, g2 = gates['1'], gates['2']
    return h2, delta, mask, (corr, patch, c1, cf, f1, mf, inp, *g1, *g2, h2, fm), upd


class _UpdateIter(torch.autograd.Function):
    """One GRU iteration.  Inputs: token, h (B,H,W,128) bf16, inp (B,H,W,128) bf16,
    corr (B,H,W,CORR_BUF) bf16, flow (B,2,H,W) fp32.  Outputs: h', delta (B,2,H,W) fp32,
    mask (B,H,W,576) bf16 (already x0.25); with ``coords`` also coords1 + delta and the new
    flow (see ``_iter_forward``), whose gradients are the delta's."""

    @staticmethod
    def forward(ctx, token, h, inp, corr, flow, state, coords=None):
        h2, delta, mask, saved, upd = _iter_forward(state.packed, h, inp, corr, flow, coords=coords)
        ctx.state = state
        ctx.itr = state.n_iter
        state.n_iter += 1
        ctx.save_for_backward(*saved)
        # an output nobody differentiates arrives as None, not as a zero-filled tensor (the
        # recurrent state's gradient comes through state.dh_carry, see backward)
        ctx.set_materialize_grads(False)
        cnew, fnew = upd if upd is not None else (None, None)
        return h2, delta, mask, cnew, fnew

    @staticmethod
    def backward(ctx, gh, gdelta, gmask, gcoords=None, gflow=None):
        for g in (gcoords, gflow):   # d(coords1 + delta) / d delta = d(flow) / d delta = 1
            if g is not None:
                gdelta = g if gdelta is None else gdelta + g
        st = ctx.state
        # the shared context gradient is accumulated across the iterations' backwards in one
        # buffer (see below), which needs them strictly in reverse order n-1 .. 0
        if st.next_bwd is None:
            # iterations after the last one that received a gradient never run their backward
            st.next_bwd = ctx.itr
        if ctx.itr != st.next_bwd:
            raise RuntimeError('fused update block: iteration %d backward ran out of order '
                               '(expected %d)' % (ctx.itr, st.next_bwd))
        st.next_bwd -= 1
        pk = st.packed
        (corr, patch, c1, cf, f1, mf, inp, h0, z1, rh1, r1, q1, h1, z2, rh2, r2, q2, h2, fm) = \
            ctx.saved_tensors
        B, H, W, _ = h2.shape
        P = B * H * W
        dev = h2.device
        dt = pk.dtype   # bf16 / fp16, or fp32: split bf16 pair buffers
        spl = pk.spl
        sh = (B, H, W)
        ops = _ext.ops()

        def wgrad(name, g, g_off, segs):
            # deferred: summed over all iterations by one launch per conv (_Packed.flush_wgrad)
            pk.defer_wgrad(name, g, g_off, segs)

        def dgrad(name, gsegs, outs, small=False, scale=1.0, gates=None, wpk=None, kcin=None):
            """outs: list of (buffer fp32, offset, slot_cnt, real, acc) or, fusing the backward of a
            ReLU, (buffer bf16, offset, slot_cnt, real, 0, relu_out, relu_out_offset).
            gates: per output, None or (mode, [a0, a1, a2, d_pre, d_pre_z, dh]) -- the ConvGRU
            gate backward fused into that fp32 segment's epilogue (OSeg in launchers.h).
            wpk: packed adjoint weight (default: the layer's); kcin: per output, the input-channel
            prefix it reads (0 = all)."""
            s = SPEC[name]
            ry = [o[5] if len(o) > 5 else o[0] for o in outs]
            # relu offset -1 marks a plain (ungated) bf16 output
            roff = [int(o[6]) if len(o) > 5 else (-1 if o[0].dtype != torch.float32 else 0)
                    for o in outs]
            gmode, gt = [], []
            if gates is not None:
                for gspec in gates:
                    gmode.append(0 if gspec is None else gspec[0])
                    if gspec is not None:
                        gt.extend(gspec[1])
            ops.conv_dgrad_([g[0] for g in gsegs], [g[1] for g in gsegs], [g[2] for g in gsegs],
                            pk.wd[name] if wpk is None else wpk, s.k[0], s.k[1], s.pad[0],
                            s.pad[1], 2 if small else 0,
                            float(scale), [o[0] for o in outs], [o[1] for o in outs],
                            [o[2] for o in outs], [o[3] for o in outs], [o[4] for o in outs],
                            ry, roff, gmode, gt, list(kcin or []), spl)

        # ---- mask head (mask = 0.25 * conv(fm[256:]))
        if gmask is None:
            gmask = _bf16(sh + (576,), dev, dt).zero_()
        elif spl:   # fp32 mask gradient -> split pair operand of the m2 dgrad / wgrad
            gmask = _to_split(gmask.permute(0, 3, 1, 2))
        if gdelta is None:
            gdelta = torch.zeros(B, 2, H, W, device=dev, dtype=torch.float32)
        gmask = gmask.contiguous()
        if gmask.dtype != dt and not spl:
            gmask = gmask.to(dt)
        # the head's ReLU backward is fused into both dgrad epilogues (bf16 pre-activation grads)
        dpre_head = _bf16(sh + (512,), dev, dt)
        gd = gdelta.contiguous().float()
        wgrad('m2', gmask, 0, [(fm, 256, 256)])
        br = _Branch(dev)
        with br:
            dgrad('m2', [(gmask, 0, 576)], [(dpre_head, 256, 256, 256, 0, fm, 256)], scale=0.25)
        if spl:
            # ---- flow head conv2 on the MFMA kernels: the delta gradient as a split operand
            # (2 channels in a 64-wide slot per half)
            gds = _to_split(gd, _bf16(sh + (64,), dev, dt))
            wgrad('fh2', gds, 0, [(fm, 0, 256)])
            dgrad('fh2', [(gds, 0, 64)], [(dpre_head, 0, 256, 256, 0, fm, 0)])
        else:
            # ---- flow head conv2 -> delta (VALU kernels; fp32 output gradient read directly)
            pk.fh2_items.append((gd, fm))
            ops.fh2_dgrad_(gd, pk.fh2_wd, fm, dpre_head)
        br.join()
        # ---- head
        wgrad('head', dpre_head, 0, [(h2, 0, HD)])
        # the recurrent state's gradient: the next iteration's backward hands it over in fp32
        # (state.dh_carry) instead of through autograd, which would round it to h's bf16 dtype
        # and back (two conversion kernels per iteration and a bf16 rounding of dh)
        carry, st.dh_carry = st.dh_carry, None
        if gh is not None and st.zero_h is not None and gh.data_ptr() == st.zero_h.data_ptr():
            gh = None   # the stand-in zero of a carried gradient (below)
        if gh is not None and spl:
            gh = _from_split(gh)   # a split-encoded state gradient from outside the block
        if gh is not None:
            dh = gh.float().contiguous() if carry is None else carry.add_(gh)
        else:
            dh = carry if carry is not None else _f32(sh + (HD,), dev, zero=True)
        halves = (('2', (h1, z2, rh2, r2, q2)), ('1', (h0, z1, rh1, r1, q1)))

        def qgate(half):
            """q / z gate backward of a GRU half-step, fused into the epilogue of the dgrad that
            finalises its output-state gradient: -> (spec, (d pre-q, d pre-z|r, dh of its input));
            the r half of d pre-z|r is written by the q dgrad's epilogue (gate 2)."""
            hin, z, _, _, q = half
            bufs = (_bf16(sh + (HD,), dev, dt), _bf16(sh + (2 * HD,), dev, dt), _f32(sh + (HD,), dev))
            return (1, [z, q, hin, bufs[0], bufs[1], bufs[2]]), bufs

        if _GATES_FUSED:
            gspec, nxt = qgate(halves[0][1])
            dgrad('head', [(dpre_head, 0, 512)], [(dh, 0, HD, HD, 1)], gates=[gspec])
        else:
            dgrad('head', [(dpre_head, 0, 512)], [(dh, 0, HD, HD, 1)])

        # inp is shared by every iteration: the GRU convs' context parts get their input / weight
        # gradients once, from the iterations' summed pre-activation gradients, after the last
        # iteration's backward (11 -> 0, in that order since each needs the next one's dh); the
        # context gradient is handed to autograd by iteration 0
        ctx_g = st.ctx_g
        dmf = _f32(sh + (128,), dev)
        for k, (tag, (hin, z, rh, r, q)) in enumerate(halves):
            if _GATES_FUSED:
                # the q / z gates ran in the epilogue of the previous dgrad (head / z|r+q); the r
                # gate runs in this q dgrad's d(r*h) epilogue, d(r*h) itself is never stored
                dpre_q, dpre_zr, dhp = nxt
                wgrad('q' + tag, dpre_q, 0, [(rh, 0, HD), (mf, 0, 128)])
                dgrad('q' + tag, [(dpre_q, 0, HD)], [(dhp, 0, HD, HD, 0)],
                      gates=[(2, [r, r, hin, dpre_zr, dpre_zr, dhp])],
                      wpk=pk.wd['q' + tag][:HD])
            else:
                dpre_q = _bf16(sh + (HD,), dev, dt)
                dz = _f32(sh + (HD,), dev)
                dhp = _f32(sh + (HD,), dev)
                ops.gru_q_bwd_(dh, z, q, hin, dpre_q, dz, dhp)
                wgrad('q' + tag, dpre_q, 0, [(rh, 0, HD), (mf, 0, 128)])
                drh = _f32(sh + (HD,), dev)
                dgrad('q' + tag, [(dpre_q, 0, HD)], [(drh, 0, HD, HD, 0)],
                      wpk=pk.wd['q' + tag][:HD])
                dpre_zr = _bf16(sh + (2 * HD,), dev, dt)
                ops.gru_zr_bwd_(drh, dz, z, r, hin, dpre_zr, dhp)
            ctx_g.setdefault('q' + tag, []).append(dpre_q)
            ctx_g.setdefault('zr' + tag, []).append(dpre_zr)
            wgrad('zr' + tag, dpre_zr, 0, [(hin, 0, HD), (mf, 0, 128)])
            # one conv for dh (z|r adjoint, K prefix) and d mf (z|r + q adjoints)
            zsegs = [(dpre_zr, 0, 2 * HD), (dpre_q, 0, HD)]
            zw, zk = pk.x['zrq' + tag], [2 * HD, 0]
            zr_outs = [(dhp, 0, HD, HD, 1), (dmf, 0, 128, 128, k)]
            if _GATES_FUSED and k == 0:
                # dhp is now the final gradient of half-step 1's output: its q / z gates here
                gspec, nxt = qgate(halves[1][1])
                dgrad('zr' + tag, zsegs, zr_outs, gates=[gspec, None], wpk=zw, kcin=zk)
            elif _GATES_FUSED:
                # the last accumulation into dmf: the motion-encoder ReLU backward (its forward
                # output is mf) in this epilogue -> bf16 d pre-activation, dmf is never re-read
                dpre_conv = _bf16(sh + (128,), dev, dt)
                dgrad('zr' + tag, zsegs, zr_outs,
                      gates=[None, (3, [mf, mf, mf, dpre_conv, dpre_conv, dmf])], wpk=zw, kcin=zk)
            else:
                dgrad('zr' + tag, zsegs, zr_outs, wpk=zw, kcin=zk)
            dh = dhp
        # ---- motion encoder
        if not _GATES_FUSED:
            dpre_conv = _bf16(sh + (128,), dev, dt)
            ops.relu_bwd_(dmf, 0, mf, 0, dpre_conv, 0, 128, 1.0)
        wgrad('conv', dpre_conv, 0, [(cf, 0, 256)])
        dpre_cf = _bf16(sh + (256,), dev, dt)
        dgrad('conv', [(dpre_conv, 0, 128)], [(dpre_cf, 0, 256, 256, 0, cf, 0)])
        wgrad('c2', dpre_cf, 0, [(c1, 0, 256)])
        wgrad('f2', dpre_cf, 192, [(f1, 0, 128)])
        dpre_c1 = _bf16(sh + (256,), dev, dt)
        dpre_f1 = _bf16(sh + (128,), dev, dt)
        # bf16 (the dtype of the corr input): autograd would otherwise cast an fp32 gradient
        dcorr = _bf16(sh + (CORR_BUF,), dev, dt)
        br = _Branch(dev)
        with br:   # f2's input gradient only feeds f1's (deferred) weight gradient
            dgrad('f2', [(dpre_cf, 192, 64)], [(dpre_f1, 0, 128, 128, 0, f1, 0)])
        dgrad('c2', [(dpre_cf, 0, 192)], [(dpre_c1, 0, 256, 256, 0, c1, 0)])
        dgrad('c1', [(dpre_c1, 0, 256)], [(dcorr, 0, CORR_BUF, 324, 0)])  # slots 324.. unused
        br.join()
        wgrad('f1', dpre_f1, 0, [(patch, 0, 128)])
        wgrad('c1', dpre_c1, 0, [(corr, 0, CORR_BUF)])
        dinp = None
        if ctx.itr == 0:
            # context input / weight gradients of the four GRU convs on the summed gradients
            dinp = _f32(sh + (HD,), dev)
            for j, name in enumerate(GRU_CONVS):
                gsum = _sum_bf16(ctx_g.pop(name), spl)
                cnt = gsum.shape[-1] // 2 if spl else gsum.shape[-1]
                dgrad(name + 'i', [(gsum, 0, cnt)], [(dinp, 0, HD, HD, int(j > 0))])
                wgrad(name + 'i', gsum, 0, [(inp, 0, HD)])
            st.ctx_g = {}
            st.next_bwd = None
        # token: no gradient value (autograd still runs the weight node after every iteration)
        if ctx.itr > 0:
            # h came from iteration itr-1, whose backward runs next (strict order, checked above):
            # autograd gets a broadcast zero of h's shape and dtype (no memory, no kernel) so it
            # still runs that backward, which takes the real fp32 gradient from dh_carry
            st.dh_carry = dh
            if st.zero_h is None:
                st.zero_h = torch.zeros((), device=dev, dtype=h0.dtype)
            if spl and dinp is not None:
                dinp = _to_split(dinp.permute(0, 3, 1, 2))
            return (None, st.zero_h.expand(B, H, W, h0.shape[-1]), dinp, dcorr, None, None, None)
        if spl:
            # split fp32 inputs take split-encoded gradients (same shape and dtype as h / inp)
            dh = _to_split(dh.permute(0, 3, 1, 2))
            if dinp is not None:
                dinp = _to_split(dinp.permute(0, 3, 1, 2))
        return (None, dh, dinp, dcorr, None, None, None)


class HipUpdateBlock:
    """Drives the fused iterations for one forward pass of a BasicUpdateBlock."""

    def __init__(self, update_block, dtype=torch.bfloat16):
        self.state = _State()
        self.state.ub = update_block
        self.state.dtype = dtype
        params = flat_params(update_block)
        self.state.need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        self.state.params = params
        self.state.overlap = _OVERLAP
        self.token = _UpdateWeights.apply(self.state, *params)

    def __call__(self, h, inp, corr, flow, need_mask=True, coords=None):
        """-> (h', delta, mask), or with ``coords`` (the detached coords1) (h', delta, mask,
        coords1 + delta, coords1 + delta - coords0).  Without gradients (inference) the iteration
        runs outside autograd and ``need_mask=False`` skips the mask head (mask is then None)."""
        if not self.state.need_grad and not torch.is_grad_enabled():
            h2, delta, mask, _, upd = _iter_forward(self.state.packed, h, inp, corr, flow,
                                                    need_mask, coords)
            return (h2, delta, mask) + (upd if coords is not None else ())
        out = _UpdateIter.apply(self.token, h, inp, corr, flow, self.state, coords)
        return out if coords is not None else out[:3]


def available(required=False):
    return _ext.gpu_path_enabled(required=required)
