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
  iterations forward + backward), so on MI355X the eager step is launch-bound.  The whole
  forward + loss + backward is captured once into a hipGraph (torch.cuda.CUDAGraph == hipGraph on
  ROCm) and replayed; with several ranks the graph packs the gradients into ONE flat buffer,
  which is all-reduced with a single RCCL call between the replays, and the unpack + clip +
  fused-AdamW update is a second graph.  The learning rate lives in a device tensor so the
  OneCycle schedule keeps working
  under replay.

A device-side non-finite flag is accumulated for failure detection and checked at logging cadence.
"""
import torch
import torch.distributed as dist

from ..ops.loss import sequence_loss
from ..parallel import dist as pdist
from .optim import fetch_optimizer, clip_grad_norm_


class TrainState:
    def __init__(self, model, args, device, sync=True, graph_ready=False):
        self.model = model
        self.args = args
        self.device = device
        self.optimizer, self.scheduler = fetch_optimizer(args, model, capturable=graph_ready)
        amp_fp16 = bool(getattr(args, 'mixed_precision', False)) and \
            getattr(args, 'amp_dtype', 'bfloat16') in ('float16', 'fp16')
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
        self.scaler.unscale_(self.optimizer)
        clip_grad_norm_(self.model.parameters(), self.args.clip)
        self.scaler.step(self.optimizer)
        self.scaler.update()
        self.nonfinite += (~torch.isfinite(loss.detach())).float()

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


class GraphedTrainStep:
    """hipGraph-captured training step around a ``TrainState`` built with ``graph_ready=True``.

    The warm-up steps needed before capture (MIOpen solver search, allocator, lazy optimizer
    state) are real training steps; their effect on the weights, BN statistics, optimizer moments
    and LR schedule is rolled back after capture, so the first replay is step 0 of the run and a
    graphed run follows the same trajectory as an eager one (``tests/test_graph_gpu.py``).
    Host cost per step is one replay of each graph (~0.4 ms) instead of ~1000 kernel launches
    through Python and autograd (~16-20 ms of host time per step on MI355X).
    """

    def __init__(self, st, example, warmup=3):
        assert st.device.type == 'cuda', 'graph capture needs a GPU'
        assert not st.scaler.is_enabled(), 'use bf16 autocast (no GradScaler) with graph capture'
        self.st = st
        self.world = pdist.world_size()
        model = st.model
        self.params = [p for p in model.parameters() if p.requires_grad]
        numel = sum(p.numel() for p in self.params)
        # Gradients: .grad is None when backward starts, so every AccumulateGrad hands its
        # incoming gradient over (no zero fill, no add kernel per parameter -- 143 of them when
        # .grad were views of one persistent buffer).  Captured, those tensors live in the graph
        # pool at fixed addresses.  With world > 1 the graph ends by packing them into ``flat``
        # (one cat), which is all-reduced between the two replays and unpacked by the update graph.
        self.flat = torch.zeros(numel, device=st.device, dtype=torch.float32) if self.world > 1 else None
        self.grads = None
        for p in self.params:
            p.grad = None
        # learning rate as a device tensor (fused AdamW reads it in-graph)
        self.lr = []
        for g in st.optimizer.param_groups:
            t = torch.tensor(float(g['lr']), device=st.device, dtype=torch.float32)
            g['lr'] = t
            self.lr.append(t)
        self.static = [t.clone() for t in example]

        # warm-up AND capture on ONE side stream: autograd runs each parameter's AccumulateGrad
        # on the stream its node was first used on, so a warm-up on another stream would leave
        # the gradient accumulation outside the captured stream (the grads of a replay are then
        # never written into ``flat``)
        stream = torch.cuda.Stream(device=st.device)
        self.stream = stream
        snap = self._snapshot()
        stream.wait_stream(torch.cuda.current_stream(st.device))
        with torch.cuda.stream(stream):
            for _ in range(warmup):  # MIOpen find / allocator warm-up; these are real steps
                loss, _ = self._fwd_bwd()
                self._post()
                self._update_graphable(loss)
                self._sched()
                del loss
        torch.cuda.current_stream(st.device).wait_stream(stream)
        torch.cuda.synchronize(st.device)

        self.g_fb = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_fb, stream=stream):
            self.loss, self.metrics = self._fwd_bwd()
        self.g_up = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_up, pool=self.g_fb.pool(), stream=stream):
            self._update_graphable(self.loss)
        self.warmup_steps = warmup
        self._restore(snap)

    @torch.no_grad()
    def _snapshot(self):
        st = self.st
        opt_state = {}
        for p in self.params:
            stt = st.optimizer.state.get(p)
            if stt:
                opt_state[p] = {k: v.clone() if torch.is_tensor(v) else v for k, v in stt.items()}
        return dict(model={k: v.clone() for k, v in st.model.state_dict().items()},
                    opt=opt_state, sched=st.scheduler.state_dict(), nonfinite=st.nonfinite.clone())

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
        torch.cuda.synchronize(st.device)

    def _fwd_bwd(self):
        for p in self.params:
            p.grad = None
        out = self.st.forward_backward(*self.static)
        for p in self.params:
            if p.grad is None:  # no gradient this step (keeps the optimizer's tensor list fixed)
                p.grad = torch.zeros_like(p)
        self.grads = [p.grad for p in self.params]
        if self.flat is not None:
            torch.cat([g.reshape(-1) for g in self.grads], out=self.flat)
        return out

    def _post(self):
        if self.world > 1:
            dist.all_reduce(self.flat)

    def _unpack(self):
        if self.flat is None:
            return
        views, off = [], 0
        for g in self.grads:
            n = g.numel()
            views.append(self.flat[off:off + n].view_as(g))
            off += n
        torch._foreach_copy_(self.grads, views)
        torch._foreach_mul_(self.grads, 1.0 / self.world)

    def _update_graphable(self, loss):
        st = self.st
        self._unpack()
        clip_grad_norm_(self.params, st.args.clip)
        st.optimizer.step()
        st.nonfinite += (~torch.isfinite(loss.detach())).float()

    def _sched(self):
        st = self.st
        st.scheduler.step()
        for g, t in zip(st.optimizer.param_groups, self.lr):
            v = g['lr']
            if not torch.is_tensor(v):
                t.fill_(float(v))
                g['lr'] = t

    def step(self, image1, image2, flow, valid):
        st = self.st
        for s, x in zip(self.static, (image1, image2, flow, valid)):
            if s.data_ptr() != x.data_ptr():
                s.copy_(x, non_blocking=True)
        if st.has_buffers and self.world > 1:
            pdist.broadcast_buffers(st.model)
        self.g_fb.replay()
        self._post()
        self.g_up.replay()
        self._sched()
        st.total_steps += 1
        metrics = dict(self.metrics)
        metrics['loss'] = self.loss.detach()
        return self.loss, metrics

    def check_finite(self):
        return self.st.check_finite()
