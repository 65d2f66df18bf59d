"""Optimizer + LR schedule (reference `fetch_optimizer`, `train.py:79-86`).

AdamW(lr, weight_decay, eps) and OneCycleLR(max_lr=lr, total_steps=num_steps+100, pct_start=0.05,
cycle_momentum=False, anneal_strategy='linear').  On GPU the AdamW update runs as torch's fused
multi-tensor kernel (``fused=True``): one launch for all 5.3 M parameters instead of a per-tensor loop.
"""
import torch
import torch.optim as optim


def count_parameters(model):
    return sum(p.numel() for p in model.parameters() if p.requires_grad)


def fetch_optimizer(args, model, fused=None, capturable=False):
    params = [p for p in model.parameters() if p.requires_grad]
    if fused is None:
        fused = bool(params) and params[0].is_cuda
    kw = dict(lr=args.lr, weight_decay=args.wdecay, eps=args.epsilon)
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


def clip_grad_norm_(parameters, max_norm):
    """Global-norm clip with no host sync (torch's foreach implementation)."""
    params = [p for p in parameters if p.grad is not None]
    return torch.nn.utils.clip_grad_norm_(params, max_norm, foreach=True)
