"""RAFT sequence loss (reference `train.py:47-72`) with device-side metrics.

``sequence_loss(preds, gt, valid, gamma, max_flow)`` returns ``(loss, metrics)`` where ``metrics`` is a
dict of 0-d device tensors (epe, 1px, 3px, 5px): the caller decides when to synchronise (the trainer
does it once per logging window) instead of the reference's four ``.item()`` syncs per step.
``metrics_to_host`` converts to plain floats.
"""
import torch

from . import _ext

MAX_FLOW = 400


def torch_sequence_loss(flow_preds, flow_gt, valid, gamma=0.8, max_flow=MAX_FLOW):
    n = len(flow_preds)
    mag = torch.sum(flow_gt ** 2, dim=1).sqrt()
    v = (valid >= 0.5) & (mag < max_flow)
    loss = 0.0
    for i, pred in enumerate(flow_preds):
        w = gamma ** (n - i - 1)
        loss = loss + w * (v[:, None] * (pred - flow_gt).abs()).mean()
    epe = torch.sum((flow_preds[-1] - flow_gt) ** 2, dim=1).sqrt()
    vf = v.float()
    cnt = vf.sum()
    metrics = {
        'epe': (epe * vf).sum() / cnt,
        '1px': ((epe < 1).float() * vf).sum() / cnt,
        '3px': ((epe < 3).float() * vf).sum() / cnt,
        '5px': ((epe < 5).float() * vf).sum() / cnt,
    }
    return loss, metrics


class _SeqLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flow_gt, valid, gamma, max_flow, *preds):
        stats = _ext.ops().seq_loss_fwd(list(preds), flow_gt, valid, gamma, max_flow)
        ctx.save_for_backward(flow_gt, valid, *preds)
        ctx.gamma, ctx.max_flow = gamma, max_flow
        ctx.mark_non_differentiable(stats)
        return stats[0].clone(), stats

    @staticmethod
    def backward(ctx, dloss, _dstats):
        flow_gt, valid, *preds = ctx.saved_tensors
        grads = _ext.ops().seq_loss_bwd(list(preds), flow_gt, valid, dloss.reshape(1).float().contiguous(),
                                        ctx.gamma, ctx.max_flow)
        return (None, None, None, None, *grads)


def sequence_loss(flow_preds, flow_gt, valid, gamma=0.8, max_flow=MAX_FLOW, impl='auto'):
    use_hip = (impl != 'torch' and _ext.device_ok(flow_gt) and len(flow_preds) <= 32
               and _ext.gpu_path_enabled(required=(impl == 'hip')))
    if not use_hip:
        return torch_sequence_loss(flow_preds, flow_gt, valid, gamma, max_flow)
    preds = [p.float().contiguous() for p in flow_preds]
    loss, stats = _SeqLoss.apply(flow_gt.float().contiguous(), valid.float().contiguous(),
                                 float(gamma), float(max_flow), *preds)
    metrics = {'epe': stats[1], '1px': stats[2], '3px': stats[3], '5px': stats[4]}
    return loss, metrics


def metrics_to_host(metrics):
    keys = list(metrics.keys())
    vals = torch.stack([metrics[k].detach().float().reshape(()) for k in keys]).cpu().tolist()
    return dict(zip(keys, vals))
