"""One RAFT training step, shared by ``train.py`` and ``bench.py``.

Reference hot loop (`train.py:161-181`): zero_grad -> H2D copy -> optional noise (CPU randn + H2D)
-> DataParallel forward -> sequence_loss (4 host syncs) -> scaled backward (reduce to GPU0) ->
unscale / clip / step / schedule / scaler update.

Here the step is host-sync free: noise comes from the device RNG, the loss and its metrics are one
fused HIP reduction kept on the device, gradients are all-reduced over RCCL in buckets overlapped
with backward (``parallel.dist.GradSync``), clipping uses the foreach global norm and AdamW is the
fused multi-tensor kernel.  A device-side non-finite flag is accumulated for failure detection and
checked by the caller at its logging cadence.
"""
import torch

from ..ops.loss import sequence_loss
from ..parallel import dist as pdist
from .optim import fetch_optimizer, clip_grad_norm_


class TrainState:
    def __init__(self, model, args, device, sync=True):
        self.model = model
        self.args = args
        self.device = device
        self.optimizer, self.scheduler = fetch_optimizer(args, model)
        amp_fp16 = bool(getattr(args, 'mixed_precision', False)) and \
            getattr(args, 'amp_dtype', 'bfloat16') in ('float16', 'fp16')
        self.scaler = torch.amp.GradScaler('cuda', enabled=amp_fp16 and device.type == 'cuda')
        self.sync = None
        if sync and pdist.world_size() > 1:
            self.sync = pdist.GradSync(model, bucket_mb=getattr(args, 'bucket_mb', 8.0),
                                       order=pdist.raft_grad_order)
        self.has_buffers = any(True for _ in model.buffers())
        self.nonfinite = torch.zeros((), device=device)
        self.total_steps = 0

    def add_noise(self, image1, image2):
        # stdv ~ U(0, 5) per step, as `train.py:168-170`, drawn on the device
        stdv = torch.empty((), device=image1.device).uniform_(0.0, 5.0)
        image1 = (image1 + stdv * torch.randn_like(image1)).clamp(0.0, 255.0)
        image2 = (image2 + stdv * torch.randn_like(image2)).clamp(0.0, 255.0)
        return image1, image2

    def step(self, image1, image2, flow, valid):
        args = self.args
        model = self.model
        self.optimizer.zero_grad(set_to_none=True)
        if getattr(args, 'add_noise', False):
            image1, image2 = self.add_noise(image1, image2)
        if self.has_buffers and pdist.world_size() > 1:
            pdist.broadcast_buffers(model)  # DataParallel semantics: replica 0's BN stats
        preds = model(image1, image2, iters=args.iters)
        loss, metrics = sequence_loss(preds, flow, valid, args.gamma)
        if self.sync is not None:
            self.sync.prepare()
        self.scaler.scale(loss).backward()
        if self.sync is not None:
            self.sync.finish()
        self.scaler.unscale_(self.optimizer)
        clip_grad_norm_(model.parameters(), args.clip)
        self.scaler.step(self.optimizer)
        self.scheduler.step()
        self.scaler.update()
        self.nonfinite += (~torch.isfinite(loss.detach())).float()
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
