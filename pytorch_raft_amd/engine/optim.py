"""Optimizer + LR schedule (reference `fetch_optimizer`, `train.py:79-86`).

AdamW(lr, weight_decay, eps) and OneCycleLR(max_lr=lr, total_steps=num_steps+100, pct_start=0.05,
cycle_momentum=False, anneal_strategy='linear').  On GPU the update is :class:`FusedAdamW`: the
global-norm gradient clip, the fp16 GradScaler's unscale / overflow skip and AdamW over all ~150
parameter tensors in three launches of the native multi-tensor kernel (``csrc/kernels/adamw.hip``:
one workgroup per 4096-element chunk of any tensor).  torch's fused AdamW took 4 launches x ~72 us
plus the foreach clip on RAFT's 5.3 M parameters.  On the CPU it is torch's AdamW.
"""
import os

import torch
import torch.optim as optim


def _same_walk(x, y):
    """True when the flat walks of two dense tensors of one shape visit the same elements in the
    same order: equal strides over every dim of size > 1 (a size-1 dim's stride is irrelevant --
    a channels_last 1x1 conv weight and its contiguous gradient agree)."""
    if x.shape != y.shape:
        return False
    return all(n <= 1 or a == b for n, a, b in zip(x.shape, x.stride(), y.stride()))


class FusedAdamW(optim.Optimizer):
    """torch.optim.AdamW semantics (non-amsgrad, decoupled weight decay) on the native multi-tensor
    kernel.  ``step(max_norm=c, scaler=s)`` is, in one pass over the gradients of EVERY group,
    ``s.unscale_(opt); clip_grad_norm_(all params, c); s.step(opt); s.update()``:

    * the clip coefficient min(1, c / (norm + 1e-6)) comes from the global 2-norm over all groups
      (as ``torch.nn.utils.clip_grad_norm_`` over all parameters), and the clipped (unscaled)
      gradients are written back to ``.grad`` (``write_grad=False`` skips that store);
    * with an enabled GradScaler the gradients are unscaled by 1/S inside the kernels, a
      non-finite norm skips the whole step on the device (parameters, moments and step counts
      untouched) and the scale is updated on the device (``torch._amp_update_scale_``): no host
      sync, so the step can run inside a replayed training step;
    * every tensor keeps its own device step counter (advanced only on finite steps), so tensors
      that missed gradients on earlier steps get their own bias corrections, as in torch.

    ``lr`` may be a float or a one-element device tensor (the graph-ready step keeps it on the
    device; the LR scheduler fills it)."""

    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=1e-2):
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay))
        self.last_norm = None

    @torch.no_grad()
    def step(self, closure=None, max_norm=None, scaler=None, write_grad=True):
        assert closure is None, 'FusedAdamW takes no closure'
        from ..ops import _ext
        ops = _ext.ops()
        ps, gs, ms, vs, steps, gof, copy_back = [], [], [], [], [], [], []
        lr_t, lrs, b1s, b2s, epss, wds = [], [], [], [], [], []
        for gi, group in enumerate(self.param_groups):
            for p in group['params']:
                if p.grad is None:
                    continue
                st = self.state[p]
                # the native kernels walk parameter, gradient and moments as flat arrays: all
                # four in the parameter's dense layout (contiguous, or a channels_last model's)
                if not st:
                    st['step'] = torch.zeros((), dtype=torch.float32, device=p.device)
                    st['exp_avg'] = torch.zeros_like(p)
                    st['exp_avg_sq'] = torch.zeros_like(p)
                elif st['step'].device != p.device or st['step'].dtype != torch.float32:
                    st['step'] = st['step'].to(p.device, torch.float32)  # a loaded CPU counter
                for k in ('exp_avg', 'exp_avg_sq'):
                    if not _same_walk(st[k], p):  # loaded state / model re-laid out since
                        st[k] = torch.empty_like(p).copy_(st[k])
                g = p.grad
                if not _same_walk(g, p):
                    # never rebind p.grad: a replayed graph keeps writing the tensor it captured.
                    # The kernel gets a re-laid-out copy; the clipped gradient is copied back.
                    tmp = torch.empty_like(p).copy_(g)
                    copy_back.append((g, tmp))
                    g = tmp
                ps.append(p)
                gs.append(g)
                ms.append(st['exp_avg'])
                vs.append(st['exp_avg_sq'])
                steps.append(st['step'])
                gof.append(gi)
            lr = group['lr']
            is_t = isinstance(lr, torch.Tensor)
            lr_t.append(lr if is_t else torch.empty(0))
            lrs.append(0.0 if is_t else float(lr))
            b1, b2 = group['betas']
            b1s.append(float(b1))
            b2s.append(float(b2))
            epss.append(float(group['eps']))
            wds.append(float(group['weight_decay']))
        if not ps:
            return None
        inv = found = None
        use_scaler = scaler is not None and scaler.is_enabled()
        if use_scaler:
            assert scaler._scale is not None, 'GradScaler.scale() must run before the step'
            inv = scaler._scale.double().reciprocal().float()
            found = torch.zeros(1, device=ps[0].device)
        res = ops.adamw_step_(ps, gs, ms, vs, steps, gof, lr_t, lrs, b1s, b2s, epss, wds,
                              float(max_norm) if max_norm else 0.0, inv, found, bool(write_grad))
        self.last_norm = res[:2]
        self.last_skipped = res[2:3]  # 1.0 when a non-finite gradient norm skipped the step
        if write_grad:
            for g, tmp in copy_back:
                g.copy_(tmp)
        if use_scaler:
            torch._amp_update_scale_(scaler._scale, scaler._growth_tracker, found,
                                     scaler._growth_factor, scaler._backoff_factor,
                                     scaler._growth_interval)
        return None


def _use_fused_adamw(params, amp_fp16):
    # RAFT_FUSED_ADAMW=0: torch's fused AdamW + foreach clip (A/B)
    if os.environ.get('RAFT_FUSED_ADAMW', '1') == '0':
        return False
    if not params or not params[0].is_cuda:
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
    if isinstance(optimizer, FusedAdamW):
        optimizer.step(max_norm=max_norm, scaler=scaler)
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
