"""One RAFT training step, shared by ``train.py`` and ``bench.py``.

Reference hot loop (`train.py:161-181`): zero_grad -> H2D copy -> optional noise (CPU randn + H2D)
-> DataParallel forward -> sequence_loss (4 host syncs) -> scaled backward (reduce to GPU0) ->
unscale / clip / step / schedule / scaler update.

Here the step is host-sync free: noise comes from the device RNG, the loss and its metrics are one
fused HIP reduction kept on the device, clipping uses the foreach global norm and AdamW is the fused
multi-tensor kernel.  Two execution modes:

* eager (``TrainState.step``): gradients are all-reduced over RCCL in buckets overlapped with
  backward on a side HIP stream (``parallel.dist.GradSync``);
* HIP-graph (``GraphedTrainStep``): RAFT issues thousands of small kernels per step (12 GRU
  iterations forward + backward), so on MI355X the eager step is launch-bound.  The recurrent
  part -- correlation, the GRU iterations forward AND backward, upsampling and the loss -- is
  captured once into a hipGraph (torch.cuda.CUDAGraph == hipGraph on ROCm) and replayed; the
  encoders (large MIOpen convolutions) and the clip + fused-AdamW update run eagerly around it.
  With several ranks the update-block gradients (final after the replay) go out as ONE flat RCCL
  all-reduce that overlaps the eager encoder backward, and the encoder gradients are bucketed
  (``GradSync``: post-accumulate-grad hooks launch each bucket on a side stream while the rest of
  the encoder backward runs).  The learning rate lives in a device tensor so the OneCycle
  schedule keeps working under replay.

A device-side non-finite flag is accumulated for failure detection and checked at logging cadence.
"""
import os

import torch
import torch.distributed as dist

from ..ops.loss import sequence_loss
from ..parallel import dist as pdist
from .optim import fetch_optimizer, clip_grad_norm_, clip_and_step, FusedAdamW


# RAFT_PHASE_MARKS=1: an empty marker kernel before and after each decode replay, so a kernel
# trace splits into encoder forward / decode (update block, correlation, loss) / encoder backward +
# update (scripts/prof_diff.py --phases, scripts/categorize.py)
_PHASE_MARKS = os.environ.get('RAFT_PHASE_MARKS', '0') == '1'
# RAFT_HOST_TIMING=1: host wall time of each part of a graphed step (encode issue, replay call,
# encoder-backward issue, update issue), averaged and printed to stderr at exit -- shows where the
# host waits on the device
_HOST_TIMING = os.environ.get('RAFT_HOST_TIMING', '0') == '1'
_HT = {}


def _ht(key, t0):
    import time
    t = time.perf_counter()
    _HT.setdefault(key, []).append(t - t0)
    return t


if _HOST_TIMING:
    import atexit
    import sys as _sys

    def _ht_report():
        for k, v in _HT.items():
            v = sorted(v)
            print('host %-16s median %8.3f ms  p90 %8.3f ms  over %d steps'
                  % (k, 1e3 * v[len(v) // 2], 1e3 * v[int(len(v) * 0.9)], len(v)), file=_sys.stderr)
    atexit.register(_ht_report)


def _phase_mark():
    from ..ops import _ext
    _ext.ops().phase_mark()


class TrainState:
    def __init__(self, model, args, device, sync=True, graph_ready=False):
        self.model = model
        self.args = args
        self.device = device
        amp_fp16 = bool(getattr(args, 'mixed_precision', False)) and \
            getattr(args, 'amp_dtype', 'bfloat16') in ('float16', 'fp16')
        self.optimizer, self.scheduler = fetch_optimizer(args, model, capturable=graph_ready,
                                                         amp_fp16=amp_fp16)
        self.scaler = torch.amp.GradScaler('cuda', enabled=amp_fp16 and device.type == 'cuda')
        self.sync = None
        if sync and pdist.world_size() > 1 and not graph_ready:
            self.sync = pdist.GradSync(model, bucket_mb=getattr(args, 'bucket_mb', 8.0),
                                       order=pdist.raft_grad_order)
        self.has_buffers = any(True for _ in model.buffers())
        if device.type == 'cuda':
            # optional: batched update-block weight gradients on a side stream, overlapped with
            # the encoder backward (gradients land in .grad at the end of backward).  Measured
            # neutral on MI355X at the chairs shape (the wgrad grids already fill every CU), so
            # off unless args.wgrad_overlap is set.
            from ..ops import update_hip
            update_hip.set_wgrad_overlap(getattr(args, 'wgrad_overlap', False))
        self.nonfinite = torch.zeros((), device=device)
        self.total_steps = 0

    def add_noise(self, image1, image2):
        # stdv ~ U(0, 5) per step, as `train.py:168-170`, drawn on the device
        stdv = torch.empty((), device=image1.device).uniform_(0.0, 5.0)
        image1 = (image1 + stdv * torch.randn_like(image1)).clamp(0.0, 255.0)
        image2 = (image2 + stdv * torch.randn_like(image2)).clamp(0.0, 255.0)
        return image1, image2

    def forward_backward(self, image1, image2, flow, valid):
        args = self.args
        if getattr(args, 'add_noise', False):
            image1, image2 = self.add_noise(image1, image2)
        preds = self.model(image1, image2, iters=args.iters)
        loss, metrics = sequence_loss(preds, flow, valid, args.gamma)
        self.scaler.scale(loss).backward()
        return loss, metrics

    def apply_update(self, loss):
        clip_and_step(self.optimizer, self.model.parameters(), self.args.clip, self.scaler)
        self.nonfinite += (~torch.isfinite(loss.detach())).float()
        _count_skipped(self.optimizer, self.scaler, self.nonfinite)

    def step(self, image1, image2, flow, valid):
        self.optimizer.zero_grad(set_to_none=True)
        if self.has_buffers and pdist.world_size() > 1:
            pdist.broadcast_buffers(self.model)  # DataParallel semantics: replica 0's BN stats
        if self.sync is not None:
            self.sync.prepare()
        loss, metrics = self.forward_backward(image1, image2, flow, valid)
        if self.sync is not None:
            self.sync.finish()
        self.apply_update(loss)
        self.scheduler.step()
        self.total_steps += 1
        metrics = dict(metrics)
        metrics['loss'] = loss.detach()
        return loss, metrics

    def check_finite(self):
        """Host-side check of the accumulated non-finite flag (call at logging cadence)."""
        bad = float(self.nonfinite.item())
        if pdist.is_dist():
            t = torch.tensor([bad], device=self.device)
            torch.distributed.all_reduce(t)
            bad = float(t.item())
        return bad == 0.0


def _count_skipped(optimizer, scaler, counter):
    """A finite loss with a non-finite gradient norm makes the native AdamW skip the step on the
    device.  Without an enabled GradScaler (bf16 / fp32 training) that is a failure, not an
    overflow back-off: add it to the device non-finite counter so ``check_finite`` reports it."""
    skipped = getattr(optimizer, 'last_skipped', None)
    if skipped is not None and not (scaler is not None and scaler.is_enabled()):
        counter += skipped.reshape(())


class GraphedTrainStep:
    """hipGraph-replayed training step around a ``TrainState`` built with ``graph_ready=True``.

    What is captured: the launch-bound recurrent part -- correlation volume, the 12 GRU
    iterations forward AND backward (the fused update block's ~900 kernels), convex upsampling and
    the sequence loss (``RAFT.decode`` + ``sequence_loss`` + backward to the encoder outputs).
    What runs eagerly: the two encoders, forward and backward (``RAFT.encode``, ~100 large MIOpen
    convolutions + fused norm nodes), and the parameter update (a few multi-tensor kernels).
    MIOpen's strided-convolution backward solvers are not replay-safe (replay 0 matches eager
    bit for bit, later replays read stale workspace / output state: profiles/r2/graph_cmp_*.log),
    and the encoders are not launch-bound anyway, so keeping them out of the graph costs nothing.

    Per step: eager encode -> copy the four encoder outputs into the graph's static leaves ->
    replay g_dec (fills the update-block .grad and the leaves' .grad) -> (ranks > 1: ONE flat
    RCCL all-reduce of the update-block gradients starts) -> eager encoder backward from the
    leaves' gradients, whose post-accumulate-grad hooks launch the encoder gradient buckets
    (``GradSync``, side stream) as each bucket's last gradient lands -> wait for all of them ->
    clip + fused AdamW (multi-tensor kernels, eager).

    The warm-up steps needed before capture (MIOpen solver search, allocator, lazy optimizer
    state) are real training steps; their effect on the weights, BN statistics, optimizer moments
    and LR schedule is rolled back after capture, so the first replayed step is step 0 of the run
    and a graphed run follows the eager trajectory (``tests/test_graph_gpu.py``).
    """

    def __init__(self, st, example, warmup=2):
        assert st.device.type == 'cuda', 'graph capture needs a GPU'
        # fp16 autocast: the GradScaler's loss scale is a device tensor the captured backward
        # multiplies by, and the unscale / overflow skip / scale update run on the device inside
        # FusedAdamW's step (no host sync), so fp16 steps replay like bf16 ones
        assert not st.scaler.is_enabled() or isinstance(st.optimizer, FusedAdamW), \
            'graph capture with a GradScaler needs the device-side FusedAdamW step'
        self.st = st
        self.world = pdist.world_size()
        model = st.model
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.dec_params = [p for n, p in named if n.startswith('update_block')]
        self.enc_params = [p for n, p in named if not n.startswith('update_block')]
        # ranks > 1: the update-block gradients are final after the decode replay and go out as
        # one flat all-reduce while the eager encoder backward runs; the encoder gradients are
        # all-reduced in buckets launched by post-accumulate-grad hooks during that backward
        self.params = self.dec_params + self.enc_params
        self.n_dec = sum(p.numel() for p in self.dec_params)
        self.flat = (torch.zeros(self.n_dec, device=st.device, dtype=torch.float32)
                     if self.world > 1 else None)
        self.enc_sync = None
        if self.world > 1:
            self.enc_sync = pdist.GradSync(model, bucket_mb=getattr(st.args, 'enc_bucket_mb', 2.0),
                                           order=pdist.raft_grad_order, params=self.enc_params)
        for p in self.params:
            p.grad = None
        # learning rate as a device tensor (fused AdamW reads it in-graph)
        self.lr = []
        for g in st.optimizer.param_groups:
            t = torch.tensor(float(g['lr']), device=st.device, dtype=torch.float32)
            g['lr'] = t
            self.lr.append(t)

        stream = torch.cuda.Stream(device=st.device)
        self.stream = stream
        snap = self._snapshot()
        stream.wait_stream(torch.cuda.current_stream(st.device))
        with torch.cuda.stream(stream):
            if self.world > 1:
                # before any other launch: every kernel choice is made on rank 0
                self._tune_on_rank0(example)
            # static leaves of the decode graph, shaped / strided like the encoder outputs
            with torch.no_grad():
                feats = model.encode(example[0], example[1])
            self.sfeat = [f.detach().clone().requires_grad_(True) for f in feats]
            self.sflow = example[2].detach().clone()
            self.svalid = example[3].detach().clone()
            del feats
            for _ in range(warmup):  # MIOpen find / autotune / allocator warm-up: real steps
                self._step_body(*example, graphs=False)
        torch.cuda.current_stream(st.device).wait_stream(stream)
        torch.cuda.synchronize(st.device)

        self.g_dec = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_dec, stream=stream):
            self.loss, self.metrics = self._decode()
        for p in self.dec_params:
            if p.grad is None:  # no gradient this step (fixed tensors for the replays)
                p.grad = torch.zeros_like(p)
        self.dec_grads = [p.grad for p in self.dec_params]
        self.warmup_steps = warmup
        self._restore(snap)

    def _tune_on_rank0(self, example):
        """Kernel choices are made ONCE, on rank 0, and every rank runs them: rank 0 runs a
        forward + backward alone (no collectives) while the others wait -- it autotunes the
        conv tiles and MIOpen's find writes its choices to the shared user find-db -- then the
        tuned tile table is broadcast and imported, and the other ranks pre-warm with autotune
        off (their MIOpen finds hit rank 0's db records).  Identical kernels mean identical
        reduction orders on every rank, and the tuning cost is paid once per node.  Effects on
        the weights / BN statistics are rolled back with the warm-up steps."""
        from ..ops import _ext
        ops = _ext.ops()   # loads the native library (nothing ran yet)
        me = pdist.rank()
        if me != 0:
            ops.conv_set_autotune(0)
        if me == 0:
            self._prewarm(example)
        pdist.barrier(self.st.device)
        pdist.share_conv_tuning(self.st.device)
        if me != 0:
            try:
                self._prewarm(example)
            finally:
                # back to the environment's default: a geometry first seen later (another
                # resolution, an eval pass) is tuned, as on rank 0
                ops.conv_set_autotune(-1)
        self.autotune_runs = int(ops.conv_autotune_runs())
        pdist.barrier(self.st.device)

    def _prewarm(self, example):
        # a purely local pass: the encoder buckets' all-reduce hooks must not fire (the other
        # ranks are not in a collective)
        if self.enc_sync is not None:
            self.enc_sync.paused = True
        try:
            feats = self.st.model.encode(example[0], example[1])
            preds = self.st.model.decode(*feats, iters=self.st.args.iters)
            loss, _ = sequence_loss(preds, example[2], example[3], self.st.args.gamma)
            loss.backward()
            del feats, preds, loss
        finally:
            if self.enc_sync is not None:
                self.enc_sync.paused = False
        for p in self.params:
            p.grad = None

    # ---------------------------------------------------------------- pieces of one step
    def _decode(self):
        """The captured part: decode + loss + backward to the static leaves / update block."""
        st = self.st
        for p in self.dec_params:
            p.grad = None
        for s in self.sfeat:
            s.grad = None
        preds = st.model.decode(*self.sfeat, iters=st.args.iters)
        loss, metrics = sequence_loss(preds, self.sflow, self.svalid, st.args.gamma)
        st.scaler.scale(loss).backward()   # fp16: times the device loss scale; else the loss
        return loss, metrics

    def _encode_and_stage(self, image1, image2, flow, valid):
        st = self.st
        if getattr(st.args, 'add_noise', False):
            image1, image2 = st.add_noise(image1, image2)
        feats = st.model.encode(image1, image2)
        with torch.no_grad():
            for s, f in zip(self.sfeat, feats):
                s.copy_(f)
            if self.sflow.data_ptr() != flow.data_ptr():
                self.sflow.copy_(flow, non_blocking=True)
            if self.svalid.data_ptr() != valid.data_ptr():
                self.svalid.copy_(valid, non_blocking=True)
        return feats

    def _encoder_backward(self, feats):
        torch.autograd.backward(list(feats), [s.grad for s in self.sfeat])

    def _forward_backward_sync(self, image1, image2, flow, valid, graphs=True):
        """Forward + backward of one step; on return every gradient is the all-rank mean."""
        st = self.st
        # encoder gradients are handed over by AccumulateGrad each step (no zero fill, no add
        # kernel per parameter); the update-block gradients live in the decode graph's pool
        if _HOST_TIMING:
            import time
            t0 = time.perf_counter()
        for p in (self.enc_params if graphs else self.params):
            p.grad = None
        if st.has_buffers and self.world > 1:
            pdist.broadcast_buffers(st.model)  # DataParallel semantics: replica 0's BN stats
        feats = self._encode_and_stage(image1, image2, flow, valid)
        if _HOST_TIMING:
            t0 = _ht('encode', t0)
        if graphs:
            if _PHASE_MARKS:
                _phase_mark()
            self.g_dec.replay()
            if _PHASE_MARKS:
                _phase_mark()
            if _HOST_TIMING:
                t0 = _ht('replay', t0)
            loss = self.loss
        else:
            loss, _ = self._decode()
            for p in self.dec_params:
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
        work = self._allreduce_dec()                 # overlaps the encoder backward
        if self.enc_sync is not None:
            self.enc_sync.prepare()
        self._encoder_backward(feats)
        del feats
        if _HOST_TIMING:
            t0 = _ht('enc_backward', t0)
        if self.enc_sync is not None:
            self.enc_sync.finish()                   # buckets with no gradient go out as zeros
        for p in self.enc_params:
            if p.grad is None:
                p.grad = torch.zeros_like(p)
        if work is not None:
            work.wait()
            self._unpack()
        self.grads = [p.grad for p in self.params]
        return loss

    def _step_body(self, image1, image2, flow, valid, graphs=True):
        loss = self._forward_backward_sync(image1, image2, flow, valid, graphs)
        if _HOST_TIMING:
            import time
            t0 = time.perf_counter()
        # clip + fused AdamW: a handful of multi-tensor launches, issued eagerly (the encoder
        # gradients are fresh tensors every step)
        self._update_graphable(loss)
        self._sched()
        if _HOST_TIMING:
            _ht('update', t0)
        return loss

    def _allreduce_dec(self):
        """Pack the update-block gradients into ``flat`` and start its (sum) all-reduce."""
        if self.world <= 1:
            return None
        torch.cat([p.grad.reshape(-1) for p in self.dec_params], out=self.flat)
        return dist.all_reduce(self.flat, async_op=True)

    def _unpack(self):
        grads = [p.grad for p in self.dec_params]
        views, off = [], 0
        for g in grads:
            n = g.numel()
            views.append(self.flat[off:off + n].view_as(g))
            off += n
        torch._foreach_copy_(grads, views)
        torch._foreach_mul_(grads, 1.0 / self.world)

    def _update_graphable(self, loss):
        st = self.st
        clip_and_step(st.optimizer, self.params, st.args.clip, st.scaler)
        st.nonfinite += (~torch.isfinite(loss.detach())).float()
        _count_skipped(st.optimizer, st.scaler, st.nonfinite)

    def _sched(self):
        st = self.st
        st.scheduler.step()
        for g, t in zip(st.optimizer.param_groups, self.lr):
            v = g['lr']
            if not torch.is_tensor(v):
                t.fill_(float(v))
                g['lr'] = t

    # ---------------------------------------------------------------- warm-up roll-back
    @torch.no_grad()
    def _snapshot(self):
        st = self.st
        opt_state = {}
        for p in self.params:
            stt = st.optimizer.state.get(p)
            if stt:
                opt_state[p] = {k: v.clone() if torch.is_tensor(v) else v for k, v in stt.items()}
        scaler = None
        if st.scaler.is_enabled() and st.scaler._scale is not None:
            scaler = (st.scaler._scale.clone(), st.scaler._growth_tracker.clone())
        return dict(model={k: v.clone() for k, v in st.model.state_dict().items()},
                    opt=opt_state, sched=st.scheduler.state_dict(), nonfinite=st.nonfinite.clone(),
                    scaler=scaler)

    @torch.no_grad()
    def _restore(self, snap):
        """In-place roll-back (the graphs hold these storages) of the warm-up steps."""
        st = self.st
        for k, v in st.model.state_dict().items():
            v.copy_(snap['model'][k])
        for p in self.params:
            stt = st.optimizer.state.get(p)
            if not stt:
                continue
            old = snap['opt'].get(p)
            for k, v in stt.items():
                if not torch.is_tensor(v):
                    if old is not None:
                        stt[k] = old[k]
                    continue
                if old is None:
                    v.zero_()  # fresh AdamW state: step 0, zero moments
                else:
                    v.copy_(old[k])
        st.scheduler.load_state_dict(snap['sched'])
        for g, t, v in zip(st.optimizer.param_groups, self.lr, st.scheduler.get_last_lr()):
            t.fill_(float(v))
            g['lr'] = t
        st.nonfinite.copy_(snap['nonfinite'])
        if st.scaler.is_enabled() and st.scaler._scale is not None:
            if snap['scaler'] is not None:
                st.scaler._scale.copy_(snap['scaler'][0])
                st.scaler._growth_tracker.copy_(snap['scaler'][1])
            else:   # created by the warm-up steps: back to the initial scale
                st.scaler._scale.fill_(st.scaler._init_scale)
                st.scaler._growth_tracker.zero_()
        torch.cuda.synchronize(st.device)

    # ---------------------------------------------------------------- public
    def step(self, image1, image2, flow, valid):
        st = self.st
        self._step_body(image1, image2, flow, valid, graphs=True)
        st.total_steps += 1
        metrics = dict(self.metrics)
        metrics['loss'] = self.loss.detach()
        return self.loss, metrics

    def check_finite(self):
        return self.st.check_finite()
