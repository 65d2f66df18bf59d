"""Fused HIP update block of RAFT-small: SmallMotionEncoder + ConvGRU (3x3) + FlowHead.

Reference: `core/update.py:16-31` (ConvGRU), `:62-77` (SmallMotionEncoder), `:99-112`
(SmallUpdateBlock), `core/raft.py:133-139` (upflow8 instead of the convex mask).  One GRU
iteration is ONE autograd node built from the same gfx950 kernels as the full block
(``ops/update_hip.py``): implicit-GEMM bf16 MFMA convs with fused epilogues, hand-written
backward (dgrad on flipped weights, batched weight gradients per step).

Layout: every activation is an NHWC bf16 buffer whose width is a multiple of 64 (the conv's K
step).  The small model's odd widths are carried in padded buffers whose pad channels are exact
zeros, with the padding folded into the packed weights:

* hidden state h: 96 real channels in 128.  convz / convr / convq rows are zero-padded to 128
  (``row_pad``), so the padded gate channels evaluate to z = r = 0.5, q = tanh(0) = 0 and the GRU
  epilogue writes h' = 0 there -- the pads stay zero through every iteration;
* corr: 4 x 49 = 196 taps in 256 (the lookup zero-fills the tail);
* motion features: [cor 96 | flo 32] in one 128-wide buffer (both convs write their slice), then
  [conv 80 | flow 2 | 0 ...] in 128;
* flow_head.conv2 (128 -> 2) runs as a 32-wide-N MFMA conv writing the fp32 NCHW delta.

The backward keeps the accumulating gradients (dh, d inp, d motion) in fp32 and feeds bf16
pre-activation gradients to the dgrad / wgrad kernels, like the full block.

Operand dtype: bf16 (bf16 autocast) or fp16 (fp16 autocast, the reference's --mixed_precision,
`core/raft.py:99`): every 16-bit buffer, packed weight and MFMA of a step is of that type
(``HipSmallUpdateBlock(ub, dtype)``); accumulation and the carried gradients stay fp32.  dtype
fp32 is the fp32 schedule of the full block: every 16-bit buffer is a split-fp32 bf16 [hi | lo]
pair buffer of twice the width, every conv three MFMA products (hi*hi + lo*hi + hi*lo, ~2^-16
relative to fp32), the elementwise backward kernels read and write the pairs.
"""
import torch

from . import _ext
from . import conv as C
from . import update_hip as _UH
from .update_hip import _LayerSpec, Design, _UpdateWeights, _State, _bf16, _f32

HDP = 128        # padded hidden width (96 real)
CORR_BUF_SMALL = 256  # 196 lookup taps zero-padded to a multiple of the K step

_HM_S = [(0, 96), (160, 82)]   # [h | mf] input channels of the small ConvGRU's module weights
_CTX_S = [(96, 64)]            # its context (inp) channels

SMALL_SPECS = [
    _LayerSpec('c1', 96, (1, 1), [196], [CORR_BUF_SMALL], adj_pad=128),
    _LayerSpec('f1', 64, (7, 7), [2], [8], small=True, patch=True),
    _LayerSpec('f2', 32, (3, 3), [64], [64], adj_pad=64, adj_off=32),
    _LayerSpec('conv', 80, (3, 3), [128], [128], adj_pad=128),
    # ConvGRU over [h | inp | mf]: per iteration [h | mf]; the context part (inp, the same in
    # every iteration) runs once per forward / backward as '<name>i' (see ops/update_hip.py)
    _LayerSpec('zr', 256, (3, 3), [96, 82], [HDP, 128], row_pad=HDP, in_sel=_HM_S, no_bias=True),
    _LayerSpec('q', 128, (3, 3), [96, 82], [HDP, 128], row_pad=HDP, in_sel=_HM_S, no_bias=True),
    _LayerSpec('fh1', 128, (3, 3), [96], [HDP]),
    _LayerSpec('fh2', 2, (3, 3), [128], [128], adj_pad=64),
    _LayerSpec('zri', 256, (3, 3), [64], [64], row_pad=HDP, in_sel=_CTX_S),
    _LayerSpec('qi', 128, (3, 3), [64], [64], row_pad=HDP, in_sel=_CTX_S),
]
GRU_S = ('zr', 'q')


def small_module_params(ub):
    e, g, fh = ub.encoder, ub.gru, ub.flow_head
    return {
        'c1': [(e.convc1.weight, e.convc1.bias)],
        'f1': [(e.convf1.weight, e.convf1.bias)],
        'f2': [(e.convf2.weight, e.convf2.bias)],
        'conv': [(e.conv.weight, e.conv.bias)],
        'zr': [(g.convz.weight, g.convz.bias), (g.convr.weight, g.convr.bias)],
        'q': [(g.convq.weight, g.convq.bias)],
        'zri': [(g.convz.weight, g.convz.bias), (g.convr.weight, g.convr.bias)],
        'qi': [(g.convq.weight, g.convq.bias)],
        'fh1': [(fh.conv1.weight, fh.conv1.bias)],
        'fh2': [(fh.conv2.weight, fh.conv2.bias)],
    }


SMALL = Design(SMALL_SPECS, small_module_params)


def _zeros_bf16(shape, dev, dt=torch.bfloat16):
    return _bf16(shape, dev, dt).zero_()   # dt fp32: a zeroed split pair buffer


def _conv(pk, name, segs, epi, outs, offs, aux=(), aux_offs=(), split=0, bias=None):
    s = SMALL.spec[name]
    k, pad, small = ((1, 1), (0, 0), False) if s.patch else (s.k, s.pad, s.small)
    C.conv_fwd(segs, pk.w[name], pk.b[name] if bias is None else bias, k, pad, s.cout,
               epi | (C.EPI_SPL if pk.spl else 0), outs, offs, aux, aux_offs, scale=s.scale,
               split=split, cin_small=2 if small else 0)


def _ctx_maps(pk, inp):
    """conv(inp, W_inp) + bias of the ConvGRU convs, fp32 (B,H,W,cout), once per forward pass."""
    key = (inp.data_ptr(), tuple(inp.shape), inp._version)
    if pk.ctx is not None:
        if key != pk.ctx_key:
            raise RuntimeError('fused update block: every iteration of a forward pass must take '
                               'the same context tensor')
        return pk.ctx
    b, h, w, _ = inp.shape
    pk.ctx = {}
    for name in GRU_S:
        m = torch.empty(b, h, w, SMALL.spec[name + 'i'].cout, device=inp.device, dtype=torch.float32)
        _conv(pk, name + 'i', [(inp, 0, 64)], C.EPI_F32, [m], [0])
        pk.ctx[name] = m
    pk.ctx_key = key
    return pk.ctx


def _iter_forward(pk, h, inp, corr, flow):
    """h (B,H,W,128) bf16 [96 real], inp (B,H,W,64) bf16, corr (B,H,W,256) bf16 [196 real],
    flow (B,2,H,W) fp32 -> (h', delta (B,2,H,W) fp32, saved tensors)."""
    B, H, W, _ = h.shape
    dev = h.device
    sh = (B, H, W)
    dt = pk.dtype   # bf16 / fp16 operand dtype
    ops = _ext.ops()
    patch = _bf16(sh + (128,), dev, dt)
    mf = _zeros_bf16(sh + (128,), dev, dt)    # [conv 80 | flow 2 | zeros]
    ops.f1_patch_(flow, patch, mf, 80)
    cf = _bf16(sh + (128,), dev, dt)          # [cor 96 | flo 32]
    f1 = _bf16(sh + (64,), dev, dt)
    _conv(pk, 'c1', [(corr, 0, CORR_BUF_SMALL)], C.EPI_RELU_BF16, [cf], [0])
    _conv(pk, 'f1', [(patch, 0, 128)], C.EPI_RELU_BF16, [f1], [0])
    _conv(pk, 'f2', [(f1, 0, 64)], C.EPI_RELU_BF16, [cf], [96])
    _conv(pk, 'conv', [(cf, 0, 128)], C.EPI_RELU_BF16, [mf], [0])
    z, rh, r = _bf16(sh + (HDP,), dev, dt), _bf16(sh + (HDP,), dev, dt), _bf16(sh + (HDP,), dev, dt)
    ctx = _ctx_maps(pk, inp)
    _conv(pk, 'zr', [(h, 0, HDP), (mf, 0, 128)], C.EPI_GRU_ZR, [z, rh, r], [0, 0, 0], aux=[h],
          aux_offs=[0], split=HDP, bias=ctx['zr'])
    hn, q = _bf16(sh + (HDP,), dev, dt), _bf16(sh + (HDP,), dev, dt)
    _conv(pk, 'q', [(rh, 0, HDP), (mf, 0, 128)], C.EPI_GRU_Q, [hn, q], [0, 0],
          aux=[h, z], aux_offs=[0, 0], bias=ctx['q'])
    fm = _bf16(sh + (128,), dev, dt)
    _conv(pk, 'fh1', [(hn, 0, HDP)], C.EPI_RELU_BF16, [fm], [0])
    delta = torch.empty(B, 2, H, W, device=dev, dtype=torch.float32)
    _conv(pk, 'fh2', [(fm, 0, 128)], C.EPI_F32_NCHW, [delta], [0])
    return hn, delta, (corr, patch, cf, f1, mf, inp, h, z, rh, r, q, hn, fm)


class _SmallUpdateIter(torch.autograd.Function):
    """One ConvGRU iteration of RAFT-small (inputs as ``_iter_forward``) -> (h', delta)."""

    @staticmethod
    def forward(ctx, token, h, inp, corr, flow, state):
        hn, delta, saved = _iter_forward(state.packed, h, inp, corr, flow)
        ctx.state = state
        ctx.itr = state.n_iter
        state.n_iter += 1
        ctx.save_for_backward(*saved)
        return hn, delta

    @staticmethod
    def backward(ctx, gh, gdelta):
        st = ctx.state
        if st.next_bwd is None:
            st.next_bwd = ctx.itr
        if ctx.itr != st.next_bwd:
            raise RuntimeError('fused update block: iteration %d backward ran out of order '
                               '(expected %d)' % (ctx.itr, st.next_bwd))
        st.next_bwd -= 1
        pk = st.packed
        corr, patch, cf, f1, mf, inp, h, z, rh, r, q, hn, fm = ctx.saved_tensors
        B, H, W, _ = hn.shape
        dev = hn.device
        sh = (B, H, W)
        dt = pk.dtype
        spl = pk.spl   # fp32 schedule: split pair buffers
        ops = _ext.ops()

        def dgrad(name, gsegs, outs, scale=1.0):
            s = SMALL.spec[name]
            ry = [o[5] if len(o) > 5 else o[0] for o in outs]
            roff = [int(o[6]) if len(o) > 5 else (-1 if o[0].dtype != torch.float32 else 0)
                    for o in outs]
            ops.conv_dgrad_([g[0] for g in gsegs], [g[1] for g in gsegs], [g[2] for g in gsegs],
                            pk.wd[name], s.k[0], s.k[1], s.pad[0], s.pad[1], 0, float(scale),
                            [o[0] for o in outs], [o[1] for o in outs], [o[2] for o in outs],
                            [o[3] for o in outs], [o[4] for o in outs], ry, roff, [], [], [], spl)

        # ---- flow head: conv2 (128 -> 2) as an MFMA conv on a 64-wide bf16 gradient
        if spl:   # the fp32 delta gradient as a split operand (2 channels in a 64-wide slot)
            g2 = _UH._to_split(gdelta.float(), _bf16(sh + (64,), dev, dt))
        else:
            g2 = _zeros_bf16(sh + (64,), dev, dt)
            g2[..., :2] = gdelta.permute(0, 2, 3, 1)
        pk.defer_wgrad('fh2', g2, 0, [(fm, 0, 128)])
        dpre_fm = _zeros_bf16(sh + (128,), dev, dt)
        dgrad('fh2', [(g2, 0, 64)], [(dpre_fm, 0, 128, 128, 0, fm, 0)])
        pk.defer_wgrad('fh1', dpre_fm, 0, [(hn, 0, HDP)])
        if gh is not None and spl:
            gh = _UH._from_split(gh)
        dh = gh.float().contiguous() if gh is not None else _f32(sh + (HDP,), dev, zero=True)
        dgrad('fh1', [(dpre_fm, 0, 128)], [(dh, 0, HDP, 96, 1)])
        # ---- ConvGRU (pads: every gradient buffer is zero beyond the 96 real channels); the
        # context part's input / weight gradients come once from the summed gradients (below)
        dmf = _f32(sh + (128,), dev, zero=True)
        dpre_q = _bf16(sh + (HDP,), dev, dt)
        dz = _f32(sh + (HDP,), dev)
        dhp = _f32(sh + (HDP,), dev)
        ops.gru_q_bwd_(dh, z, q, h, dpre_q, dz, dhp)
        pk.defer_wgrad('q', dpre_q, 0, [(rh, 0, HDP), (mf, 0, 128)])
        drh = _f32(sh + (HDP,), dev, zero=True)
        dgrad('q', [(dpre_q, 0, HDP)], [(drh, 0, HDP, 96, 0), (dmf, 0, 128, 82, 1)])
        dpre_zr = _bf16(sh + (2 * HDP,), dev, dt)
        ops.gru_zr_bwd_(drh, dz, z, r, h, dpre_zr, dhp)
        pk.defer_wgrad('zr', dpre_zr, 0, [(h, 0, HDP), (mf, 0, 128)])
        dgrad('zr', [(dpre_zr, 0, 2 * HDP)], [(dhp, 0, HDP, 96, 1), (dmf, 0, 128, 82, 1)])
        st.ctx_g.setdefault('q', []).append(dpre_q)
        st.ctx_g.setdefault('zr', []).append(dpre_zr)
        # ---- motion encoder
        dpre_conv = _zeros_bf16(sh + (128,), dev, dt)
        ops.relu_bwd_(dmf, 0, mf, 0, dpre_conv, 0, 80, 1.0, spl)
        pk.defer_wgrad('conv', dpre_conv, 0, [(cf, 0, 128)])
        dpre_cf = _bf16(sh + (128,), dev, dt)
        dgrad('conv', [(dpre_conv, 0, 128)], [(dpre_cf, 0, 128, 128, 0, cf, 0)])
        pk.defer_wgrad('c1', dpre_cf, 0, [(corr, 0, CORR_BUF_SMALL)])
        pk.defer_wgrad('f2', dpre_cf, 96, [(f1, 0, 64)])
        dpre_f1 = _bf16(sh + (64,), dev, dt)
        # f2's outputs are channels 96..127 of dpre_cf: the adjoint reads [64, 128) with the
        # layer's rows at offset 32 of it (adj_off), c1's rows at [0, 96) of [0, 128)
        dgrad('f2', [(dpre_cf, 64, 64)], [(dpre_f1, 0, 64, 64, 0, f1, 0)])
        pk.defer_wgrad('f1', dpre_f1, 0, [(patch, 0, 128)])
        dcorr = _bf16(sh + (CORR_BUF_SMALL,), dev, dt)
        dgrad('c1', [(dpre_cf, 0, 128)], [(dcorr, 0, CORR_BUF_SMALL, 196, 0)])
        dinp = None
        if ctx.itr == 0:
            dinp = _f32(sh + (64,), dev)
            for j, name in enumerate(GRU_S):
                gsum = _UH._sum_bf16(st.ctx_g.pop(name), spl)
                cnt = gsum.shape[-1] // 2 if spl else gsum.shape[-1]
                dgrad(name + 'i', [(gsum, 0, cnt)], [(dinp, 0, 64, 64, int(j > 0))])
                pk.defer_wgrad(name + 'i', gsum, 0, [(inp, 0, 64)])
            st.ctx_g = {}
            st.next_bwd = None
        if spl:   # split inputs take split-encoded gradients (same shape and dtype as h / inp)
            dhp = _UH._to_split(dhp.permute(0, 3, 1, 2))
            if dinp is not None:
                dinp = _UH._to_split(dinp.permute(0, 3, 1, 2))
        return (None, dhp, dinp, dcorr, None, None)


class HipSmallUpdateBlock:
    """Drives the fused iterations for one forward pass of a SmallUpdateBlock."""

    def __init__(self, update_block, dtype=torch.bfloat16):
        assert dtype in (torch.bfloat16, torch.float16, torch.float32), dtype
        self.state = _State()
        self.state.ub = update_block
        self.state.design = SMALL
        self.state.dtype = dtype
        params = SMALL.flat_params(update_block)
        self.state.need_grad = torch.is_grad_enabled() and any(p.requires_grad for p in params)
        self.state.params = params
        self.state.overlap = _UH._OVERLAP
        self.token = _UpdateWeights.apply(self.state, *params)

    def __call__(self, h, inp, corr, flow):
        """-> (h', delta)"""
        if not self.state.need_grad and not torch.is_grad_enabled():
            hn, delta, _ = _iter_forward(self.state.packed, h, inp, corr, flow)
            return hn, delta
        return _SmallUpdateIter.apply(self.token, h, inp, corr, flow, self.state)
