"""Optimizer + LR schedule (reference `fetch_optimizer`, `train.py:79-86`).

AdamW(lr, weight_decay, eps) and OneCycleLR(max_lr=lr, total_steps=num_steps+100, pct_start=0.05,
cycle_momentum=False, anneal_strategy='linear').  On GPU (no GradScaler) the update is
:class:`FusedAdamW`: the global-norm gradient clip and AdamW over all ~150 parameter tensors in
three launches of the native multi-tensor kernel (``csrc/kernels/adamw.hip``: one workgroup per
4096-element chunk of any tensor).  torch's fused AdamW took 4 launches x ~72 us plus the foreach
clip on RAFT's 5.3 M parameters.  With a GradScaler (fp16) or on the CPU it is torch's AdamW.
"""
import os

import torch
import torch.optim as optim


class FusedAdamW(optim.Optimizer):
    """torch.optim.AdamW semantics (non-amsgrad, decoupled weight decay) on the native multi-tensor
    kernel; ``step(max_norm=c)`` first clips the gradients' global 2-norm to ``c`` exactly as
    ``torch.nn.utils.clip_grad_norm_`` does (coefficient min(1, c / (norm + 1e-6))), on the device,
    without writing the clipped gradients back.  ``lr`` may be a float or a one-element device
    tensor (the graph-ready step keeps it on the device; the LR scheduler fills it)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.last_norm = None

    @torch.no_grad()
    def step(self, closure=None, max_norm=None):
        assert closure is None, 'FusedAdamW takes no closure'
        from ..ops import _ext
        ops = _ext.ops()
        for group in self.param_groups:
            ps, gs, ms, vs = [], [], [], []
            for p in group['params']:
                if p.grad is None:
                    continue
                st = self.state[p]
                if not st:
                    # a CPU tensor like torch's step counter: snapshots / roll-backs that treat
                    # every tensor entry alike (GraphedTrainStep._restore) reset it too
                    st['step'] = torch.zeros((), dtype=torch.float32)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.contiguous_format)
                st['step'] += 1
                ps.append(p)
                gs.append(p.grad.contiguous())
                ms.append(st['exp_avg'])
                vs.append(st['exp_avg_sq'])
            if not ps:
                continue
            b1, b2 = group['betas']
            t = int(self.state[ps[0]]['step'].item())   # CPU tensor: no device sync
            lr = group['lr']
            lr_t = lr if isinstance(lr, torch.Tensor) else None
            self.last_norm = ops.adamw_step_(
                ps, gs, ms, vs, lr_t, 0.0 if lr_t is not None else float(lr), b1, b2,
                group['eps'], group['weight_decay'], 1.0 - b1 ** t, 1.0 - b2 ** t,
                float(max_norm) if max_norm else 0.0)
        return None


def _use_fused_adamw(params, amp_fp16):
    # RAFT_FUSED_ADAMW=0: torch's fused AdamW + foreach clip (A/B)
    if os.environ.get('RAFT_FUSED_ADAMW', '1') == '0':
        return False
    if amp_fp16 or not params or not params[0].is_cuda:
        return False
    try:
        from ..ops import _ext
        return _ext.gpu_path_enabled(required=False)
    except Exception:  # noqa: BLE001 - no native library: torch's AdamW
        return False


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def fetch_optimizer(args, model, fused=None, capturable=False, amp_fp16=False):
    params = [p for p in model.parameters() if p.requires_grad]
    if fused is None:
        fused = bool(params) and params[0].is_cuda
    kw = dict(lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon)
    if fused and _use_fused_adamw(params, amp_fp16):
        optimizer = FusedAdamW(params, **kw)
    else:
        if capturable:
            kw['capturable'] = True
        try:
            optimizer = optim.AdamW(params, fused=fused, **kw)
        except (RuntimeError, TypeError):
            optimizer = optim.AdamW(params, **kw)
    scheduler = optim.lr_scheduler.OneCycleLR(optimizer, args.lr, args.num_steps + 100,
                                              pct_start=0.05, cycle_momentum=False,
                                              anneal_strategy='linear')
    return optimizer, scheduler


def clip_and_step(optimizer, parameters, max_norm, scaler=None):
    """Global-norm clip + optimizer step: folded into one native pass for FusedAdamW, otherwise
    torch's foreach clip (after the scaler's unscale) and the (scaler's) step."""
    if isinstance(optimizer, FusedAdamW) and (scaler is None or not scaler.is_enabled()):
        optimizer.step(max_norm=max_norm)
        return
    if scaler is not None:
        scaler.unscale_(optimizer)
    clip_grad_norm_(parameters, max_norm)
    if scaler is not None:
        scaler.step(optimizer)
        scaler.update()
    else:
        optimizer.step()


def clip_grad_norm_(parameters, max_norm):
    """Global-norm clip with no host sync (torch's foreach implementation)."""
    params = [p for p in parameters if p.grad is not None]
    return torch.nn.utils.clip_grad_norm_(params, max_norm, foreach=True)
