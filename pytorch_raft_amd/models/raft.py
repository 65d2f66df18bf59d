"""RAFT (Recurrent All-Pairs Field Transforms) -- the one model family of the reference.

API and numerics contract follow `core/raft.py:24-144` (`SURVEY.md` §2.7):

* ``RAFT(args)`` reads ``args.small`` / ``args.mixed_precision`` (+ optional ``dropout``,
  ``alternate_corr``) and WRITES ``args.corr_levels`` / ``args.corr_radius`` (preserved quirk).
* ``forward(image1, image2, iters=12, flow_init=None, upsample=True, test_mode=False)`` takes float
  0..255 (B,3,H,W) images and returns the list of ``iters`` full-resolution flows, or
  ``(flow_low, flow_up)`` in test mode.

MI355X-specific extensions (all optional ``args`` attributes, defaults chosen for gfx950):

* ``corr_impl``   'auto' (HIP kernels on GPU, torch on CPU) | 'hip' | 'torch'
* ``amp_dtype``   autocast dtype for ``mixed_precision`` -- 'bfloat16' (default; MI355X MFMA native)
                  or 'float16' (reference behaviour on CUDA; same fused HIP kernels, fp16 MFMA)
* ``channels_last`` run the encoders in NHWC (MIOpen's NHWC implicit-GEMM solvers)
* ``corr_mode``   'auto' (default) | 'allpairs' | 'onthefly'.  ``alternate_corr=True`` (the
                  reference flag, `core/raft.py:105-108`) always selects the on-the-fly block.
                  'auto' is memory-aware: the all-pairs pyramid (B x (HW/64)^2 x 4/3 elements) is
                  used while it fits in ``RAFT_CORR_BUDGET_GB`` (default: a quarter of the GPU's
                  HBM, 72 GB on MI355X), the O(HW) on-the-fly correlation beyond that.  Both give
                  the same values; all-pairs is the faster of the two at every batch that fits
                  (training, bf16, per-GPU batch 12: on-the-fly runs at 0.91x all-pairs at
                  the chairs shape, profiles/r5/otf_split/, 0.90x at KITTI 288x960),
                  on-the-fly is what makes batch-1024 Sintel inference or 4K frames fit.

In test mode the convex upsampling runs only after the last iteration (the reference computes and
discards it every iteration, `core/raft.py:133-142`); outputs are identical.
"""
import os

import torch
import torch.nn as nn

from .update import BasicUpdateBlock, SmallUpdateBlock
from .extractor import BasicEncoder, SmallEncoder
from .corr import CorrBlock, AlternateCorrBlock
from ..utils.utils import coords_grid, upflow8
from ..ops.upsample import convex_upsample
from ..ops import _ext
from ..ops import conv_fp32

# RAFT_FP32_ENC_MFMA=0: an fp32 model's encoders keep MIOpen fp32 convs (A/B measurements)
_FP32_ENC_MFMA = os.environ.get('RAFT_FP32_ENC_MFMA', '1') != '0'
# RAFT_FP32_FUSED=0: an fp32 model's update block runs eagerly with per-conv split-bf16 convs
_FP32_FUSED = os.environ.get('RAFT_FP32_FUSED', '1') != '0'
# Encoder streams (native path): 1 = one stream; 2 = the context encoder on a side HIP stream
# beside the feature encoder.  Autograd replays every node's backward on its forward's stream, so
# the backwards overlap the same way.  The encoders are independent until the decode; co-running
# fills each other's kernel tails and small launches (round 6 A/B: 484.3 / 488.3 vs 466.1 / 466.8
# pairs/s on one box; the feature encoder's two frames on a third stream as well: 468.6 / 468.0
# vs 476.6 / 480.3 -- profiles/r6/enc_streams/).  Default (unset): 2 under autocast (bf16 and
# fp16), 1 for fp32.  fp16 had kept one stream after an fp16 bench with two streams hit an
# illegal address (profiles/r6/r6i/bench_fp16_2streams.log); with the first call of each input
# signature serial (_ENC_SEEN below) two fp16 runs of 1,500 + 300 and 2,500 + 500 steps ran clean
# at 472.9 / 475.9 pairs/s vs 454.8 on one stream (profiles/r6/stress/).
_ENC_STREAMS = os.environ.get('RAFT_ENC_STREAMS', 'auto')
_SIDE = {}
# Encoder call signatures (input shape, dtypes, grad / train mode, device) already run once: the
# FIRST call of a signature runs both encoders on one stream.  That call (and its backward) is
# where MIOpen searches and compiles its solvers for the strided convs (torch.backends.cudnn.
# benchmark), allocating and freeing its own buffers; two such searches in flight at once on two
# streams through the one MIOpen handle of this thread are the suspected cause of an illegal
# address seen on the first steps of a bench run without a find-db (profiles/r6/stress/
# stress_final_fault.log).  Later calls only replay the found solvers.
_ENC_SEEN = set()


def _enc_side_stream(dev):
    key = dev.index if dev.index is not None else torch.cuda.current_device()
    if key not in _SIDE:
        _SIDE[key] = torch.cuda.Stream(device=dev)
    return _SIDE[key]


def _get(args, name, default):
    return getattr(args, name, default)


def _context_act(cnet, hdim):
    from ..ops import encoder as fast
    return fast.context_act(cnet, hdim)


def _prep_pair(image1, image2, fnet, cnet):
    """``2 * (x / 255) - 1`` of both frames as ONE channels_last (2B,3,H,W) batch in the encoders'
    compute dtype (`core/raft.py:94-95`, `core/extractor.py:176-179`), by the native
    ``image_prep_`` kernel -- when both encoders take the native fast path on it (they would cast
    and lay the frames out exactly so); None otherwise (the eager ops run)."""
    from ..ops import encoder as fast
    if not (image1.is_cuda and image1.dtype == torch.float32 and image2.dtype == torch.float32
            and image1.dim() == 4 and image1.shape[1] == 3 and image1.shape == image2.shape
            and not (image1.requires_grad or image2.requires_grad) and _ext.device_ok(image1)):
        return None
    if not (fast.fast_path_ok(fnet, image1) and fast.fast_path_ok(cnet, image1)):
        return None
    dt = torch.get_autocast_dtype('cuda') if torch.is_autocast_enabled('cuda') else torch.float32
    b, _, h, w = image1.shape
    # image-chunked encoders (huge batches, extractor.py:_chunk_images): the eager preparation
    limit = int(os.environ.get('RAFT_ENC_CHUNK_BYTES', str(2 ** 31 - 1)))
    per_img = fnet.widths[0] * ((h + 1) // 2) * ((w + 1) // 2) * torch.finfo(dt).bits // 8
    if 2 * b > max(1, limit // per_img):
        return None
    out = torch.empty(2 * b, 3, h, w, device=image1.device, dtype=dt,
                      memory_format=torch.channels_last)
    _ext.ops().image_prep_(image1.contiguous(), image2.contiguous(), out)
    return out


_BUDGET = {}


def corr_budget_bytes(device):
    """HBM the all-pairs pyramid may take before 'auto' switches to on-the-fly correlation."""
    env = os.environ.get('RAFT_CORR_BUDGET_GB')
    if env:
        return float(env) * 2 ** 30
    key = (device.type, device.index)
    if key not in _BUDGET:
        _BUDGET[key] = 0.25 * torch.cuda.get_device_properties(device).total_memory
    return _BUDGET[key]


class RAFT(nn.Module):
    def __init__(self, args):
        super().__init__()
        self.args = args
        if args.small:
            self.hidden_dim = hdim = 96
            self.context_dim = cdim = 64
            args.corr_levels = 4
            args.corr_radius = 3
        else:
            self.hidden_dim = hdim = 128
            self.context_dim = cdim = 128
            args.corr_levels = 4
            args.corr_radius = 4
        if not hasattr(self.args, 'dropout'):
            self.args.dropout = 0
        if not hasattr(self.args, 'alternate_corr'):
            self.args.alternate_corr = False

        if args.small:
            self.fnet = SmallEncoder(output_dim=128, norm_fn='instance', dropout=args.dropout)
            self.cnet = SmallEncoder(output_dim=hdim + cdim, norm_fn='none', dropout=args.dropout)
            self.update_block = SmallUpdateBlock(self.args, hidden_dim=hdim)
        else:
            self.fnet = BasicEncoder(output_dim=256, norm_fn='instance', dropout=args.dropout)
            self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn='batch', dropout=args.dropout)
            self.update_block = BasicUpdateBlock(self.args, hidden_dim=hdim)

    # ------------------------------------------------------------------ configuration helpers
    @property
    def corr_impl(self):
        return _get(self.args, 'corr_impl', 'auto')

    @property
    def amp_dtype(self):
        name = _get(self.args, 'amp_dtype', 'bfloat16')
        return {'bfloat16': torch.bfloat16, 'bf16': torch.bfloat16,
                'float16': torch.float16, 'fp16': torch.float16}[name]

    def _autocast(self, device):
        enabled = bool(self.args.mixed_precision) and device.type == 'cuda'
        return torch.autocast(device_type=device.type, dtype=self.amp_dtype, enabled=enabled)

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    def initialize_flow(self, img):
        """flow = coords1 - coords0 on the 1/8 grid."""
        n, _, h, w = img.shape
        coords0 = coords_grid(n, h // 8, w // 8, device=img.device)
        coords1 = coords_grid(n, h // 8, w // 8, device=img.device)
        return coords0, coords1

    def upsample_flow(self, flow, mask):
        """[H/8, W/8, 2] -> [H, W, 2] convex combination (HIP kernel on GPU)."""
        impl = 'torch' if self.corr_impl == 'torch' else 'auto'
        return convex_upsample(flow, mask, impl=impl)

    # ------------------------------------------------------------------ forward
    def forward(self, image1, image2, iters=12, flow_init=None, upsample=True, test_mode=False):
        feats = self.encode(image1, image2)
        return self.decode(*feats, iters=iters, flow_init=flow_init, test_mode=test_mode)

    def encode(self, image1, image2):
        """Feature + context encoders (`core/raft.py:89-114`): -> (fmap1, fmap2, net, inp).

        Split from ``decode`` so the hipGraph training step can replay the launch-bound recurrent
        part while the encoders (a few large MIOpen convolutions) run eagerly."""
        hdim, cdim = self.hidden_dim, self.context_dim
        dev = image1.device
        # corr_impl='torch' = stock reference-semantics ops everywhere (the baseline): no HIP
        # encoder kernels either
        native = self.corr_impl != 'torch'
        self.fnet.allow_native = self.cnet.allow_native = native
        # fp32 model: the encoders' stride-1 convs run as split-bf16 MFMA convs (one scope per
        # encoder call, so each conv's deferred weight gradient covers exactly that call)
        fp32_mfma = native and self._use_fp32_mfma(image1) and _FP32_ENC_MFMA
        with self._autocast(dev), conv_fp32.enabled(fp32_mfma):
            # both encoders on the native fast path: normalisation, batch cat, cast and
            # channels_last layout of the frames in one kernel; the context encoder reads frame1's
            # half of that batch in place
            pair = _prep_pair(image1, image2, self.fnet, self.cnet) if native else None
        if pair is None:
            image1 = (2 * (image1 / 255.0) - 1.0).contiguous()
            image2 = (2 * (image2 / 255.0) - 1.0).contiguous()
            if bool(_get(self.args, 'channels_last', False)):
                image1 = image1.contiguous(memory_format=torch.channels_last)
                image2 = image2.contiguous(memory_format=torch.channels_last)
        side = None
        sig = (tuple(image1.shape), image1.dtype, self.amp_dtype, bool(self.args.mixed_precision),
               torch.is_grad_enabled(), self.training, str(dev))
        first_call = sig not in _ENC_SEEN
        _ENC_SEEN.add(sig)
        if (not first_call and self._enc_streams() >= 2 and pair is not None and dev.type == 'cuda'
                and not torch.cuda.is_current_stream_capturing()):
            main = torch.cuda.current_stream(dev)
            side = _enc_side_stream(dev)
            side.wait_stream(main)
            pair.record_stream(side)

        def context():
            with self._autocast(dev), conv_fp32.enabled(fp32_mfma):
                cnet = self.cnet(image1 if pair is None else pair[:image1.shape[0]])
                # native: both activations in one pass, as the fused block's NHWC operands
                act = _context_act(cnet, hdim) if native else None
                if act is not None:
                    return act
                net, inp = torch.split(cnet, [hdim, cdim], dim=1)
                return torch.tanh(net), torch.relu(inp)

        self.last_enc_streams = 2 if side is not None else 1
        if side is not None:
            with torch.cuda.stream(side):
                net, inp = context()
        with self._autocast(dev), conv_fp32.enabled(fp32_mfma):
            if pair is None:
                fmap1, fmap2 = self.fnet([image1, image2])
            else:
                fmap1, fmap2 = torch.split(self.fnet(pair), [image1.shape[0]] * 2, dim=0)
        if side is None:
            net, inp = context()
        else:
            main.wait_stream(side)
            net.record_stream(main)
            inp.record_stream(main)
        return fmap1, fmap2, net, inp

    def _enc_streams(self):
        if _ENC_STREAMS != 'auto':
            return int(_ENC_STREAMS)
        return 2 if self.args.mixed_precision else 1

    def decode(self, fmap1, fmap2, net, inp, iters=12, flow_init=None, test_mode=False):
        """Correlation volume + GRU iterations + upsampling (`core/raft.py:102-144`)."""
        otf = self._use_onthefly(fmap1)
        self.last_corr = 'on-the-fly' if otf else 'all-pairs'
        if not (self._bf16_corr_ok(fmap1) and not otf):
            # the reference runs the correlation in fp32 (`core/raft.py:102-103`); the bf16 HIP
            # build takes the bf16 encoder outputs as they are (same products, fp32 accumulation)
            fmap1 = fmap1.float().contiguous()
            fmap2 = fmap2.float().contiguous()
        # bf16 mixed precision: bf16 MFMA correlation; fp32 model and fp16 autocast: the
        # reference's fp32 correlation (`core/raft.py:102-107`, outside autocast)
        corr_prec = 'bf16' if (self.args.mixed_precision and self.amp_dtype == torch.bfloat16) \
            else 'fp32'
        if otf:
            # bf16: bf16 MFMA operands; fp32: split-bf16 (fp32-accurate) forward and backward
            corr_fn = AlternateCorrBlock(fmap1, fmap2, radius=self.args.corr_radius,
                                         impl=self.corr_impl, precision=corr_prec)
        else:
            corr_fn = CorrBlock(fmap1, fmap2, radius=self.args.corr_radius, impl=self.corr_impl,
                                precision=corr_prec, nhwc_lookup=self._use_fused_update(fmap1))
        dev = fmap1.device
        b, _, h8, w8 = fmap1.shape
        coords0 = coords_grid(b, h8, w8, device=dev)
        # the same grid: coords1 is only ever rebound (coords1 + delta), never written in place
        coords1 = coords0 if flow_init is None else coords0 + flow_init

        if self._use_fused_update(fmap1):
            return self._iterate_fused(net, inp, corr_fn, coords0, coords1, iters, test_mode)

        # fp32 model: split-bf16 MFMA update-block convs for this decode (the iterations share the
        # packed split weights)
        with conv_fp32.enabled(self._use_fp32_mfma(fmap1)):
            return self._iterate_eager(net, inp, corr_fn, coords0, coords1, iters, test_mode)

    def _iterate_eager(self, net, inp, corr_fn, coords0, coords1, iters, test_mode):
        dev = coords0.device
        flow_predictions = []
        flow_up = None
        for itr in range(iters):
            coords1 = coords1.detach()
            corr = corr_fn(coords1)
            flow = coords1 - coords0
            with self._autocast(dev):
                net, up_mask, delta_flow = self.update_block(net, inp, corr, flow)
            coords1 = coords1 + delta_flow
            if test_mode and itr < iters - 1:
                continue
            if up_mask is None:
                flow_up = upflow8(coords1 - coords0)
            else:
                flow_up = self.upsample_flow(coords1 - coords0, up_mask)
            flow_predictions.append(flow_up)

        if test_mode:
            return coords1 - coords0, flow_up
        return flow_predictions

    def _use_onthefly(self, fmap):
        """Correlation block choice (see ``corr_mode`` in the module docstring)."""
        mode = _get(self.args, 'corr_mode', 'auto')
        if self.args.alternate_corr or mode == 'onthefly':
            return True
        if mode == 'allpairs' or fmap.device.type != 'cuda':
            return False
        b, _, h, w = fmap.shape
        n = h * w
        esz = 2 if self._bf16_corr_ok(fmap) else 4
        pyramid = b * n * n * esz * (1 + 1 / 4 + 1 / 16 + 1 / 64)
        return pyramid > corr_budget_bytes(fmap.device)

    def _bf16_corr_ok(self, fmap):
        return (fmap.dtype == torch.bfloat16 and self.corr_impl != 'torch' and
                bool(self.args.mixed_precision) and _ext.device_ok(fmap))

    # ------------------------------------------------------------------ fused HIP update path
    def _use_fp32_mfma(self, img):
        """fp32 model on a GPU: the update-block convs run as split-bf16 MFMA convs
        (ops/conv_fp32.py, ~2^-16 relative to fp32) instead of MIOpen fp32 convs."""
        impl = _get(self.args, 'update_impl', 'auto')
        return (impl != 'torch' and self.corr_impl != 'torch' and not self.args.mixed_precision
                and _ext.device_ok(img) and _ext.gpu_path_enabled())

    def _use_fused_update(self, img):
        """Fused MFMA update block: GPU and mixed precision -- bf16 or fp16 autocast (full and
        small model; the operand dtype of the conv kernels' MFMAs) -- or the fp32 schedule (full and
        small model; split-fp32 operands: bf16 [hi | lo] pairs, three products per conv;
        RAFT_FP32_FUSED=0 keeps the per-conv split path of ops/conv_fp32.py)."""
        impl = _get(self.args, 'update_impl', 'auto')
        if impl == 'torch' or self.corr_impl == 'torch' or not _ext.device_ok(img):
            return False
        ok = self.args.mixed_precision and self.amp_dtype in (torch.bfloat16, torch.float16)
        ok = ok or (not self.args.mixed_precision and _FP32_FUSED)
        if not ok:
            if impl == 'hip':
                raise ValueError("update_impl='hip' needs mixed precision (bf16 / fp16), or the "
                                 "full model in fp32")
            return False
        from ..ops import update_hip
        return update_hip.available(required=(impl == 'hip'))

    def _iterate_fused_small(self, net, inp, corr_fn, coords0, coords1, iters, test_mode):
        """RAFT-small: fused ConvGRU iterations (ops/update_hip_small.py), upflow8 output."""
        from ..ops.update_hip_small import HipSmallUpdateBlock, CORR_BUF_SMALL, HDP
        from ..ops.update_hip import split_nhwc
        # bf16 / fp16 operands, or fp32 (split bf16 pairs)
        adt = self.amp_dtype if self.args.mixed_precision else torch.float32
        hub = HipSmallUpdateBlock(self.update_block, dtype=adt)
        if adt == torch.float32:
            h, x = split_nhwc(net.float(), HDP), split_nhwc(inp.float())
        else:
            h = torch.nn.functional.pad(net.to(adt).permute(0, 2, 3, 1),
                                        (0, HDP - net.shape[1])).contiguous()
            x = inp.to(adt).permute(0, 2, 3, 1).contiguous()
        flow_predictions = []
        flow_up = None
        flow = coords1 - coords0
        for itr in range(iters):
            coords1 = coords1.detach()
            corr = corr_fn.lookup_nhwc(coords1, CORR_BUF_SMALL, adt)
            flow = flow.detach()   # = coords1 - coords0 (see _iterate_fused)
            h, delta_flow = hub(h, x, corr, flow)
            coords1 = coords1 + delta_flow
            flow = coords1 - coords0
            if test_mode and itr < iters - 1:
                continue
            flow_up = upflow8(flow)
            flow_predictions.append(flow_up)
        if test_mode:
            return flow, flow_up
        return flow_predictions

    def _iterate_fused(self, net, inp, corr_fn, coords0, coords1, iters, test_mode):
        if self.args.small:
            return self._iterate_fused_small(net, inp, corr_fn, coords0, coords1, iters, test_mode)
        from ..ops.update_hip import HipUpdateBlock, CORR_BUF, split_nhwc
        # operand dtype of the fused block: bf16, fp16 autocast, or fp32 (split bf16 pairs)
        adt = self.amp_dtype if self.args.mixed_precision else torch.float32
        hub = HipUpdateBlock(self.update_block, dtype=adt)
        if adt == torch.float32:
            h, x = split_nhwc(net.float()), split_nhwc(inp.float())
        else:
            h = net.to(adt).permute(0, 2, 3, 1).contiguous()
            x = inp.to(adt).permute(0, 2, 3, 1).contiguous()
        flow_predictions = []
        flow_up = None
        flow = coords1 - coords0
        for itr in range(iters):
            coords1 = coords1.detach()
            corr = corr_fn.lookup_nhwc(coords1, CORR_BUF, adt)
            # flow = coords1 - coords0 of the detached coords: the previous iteration's upsampling
            # input, detached (same values; one subtraction kernel per iteration instead of two)
            flow = flow.detach()
            last = itr == iters - 1
            # coords1 + delta and the new flow come out of the flow-head kernel (no add kernels)
            h, _, up_mask, coords1, flow = hub(h, x, corr, flow, need_mask=last or not test_mode,
                                               coords=coords1)
            if test_mode and itr < iters - 1:
                continue
            flow_up = convex_upsample(flow, up_mask, nhwc=True)
            flow_predictions.append(flow_up)
        if test_mode:
            return flow, flow_up
        return flow_predictions
