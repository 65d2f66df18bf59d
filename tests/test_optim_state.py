"""FusedAdamW bookkeeping on the CPU: state_dict round trip (checkpoint / resume), the OneCycle
schedule driving its param groups, and the CPU fallback of ``fetch_optimizer``."""
import argparse

import torch

from pytorch_raft_amd.engine.optim import FusedAdamW, fetch_optimizer


def test_fused_adamw_state_dict_round_trip():
    ps = [torch.nn.Parameter(torch.randn(3, 4)), torch.nn.Parameter(torch.randn(5))]
    o = FusedAdamW(ps, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    for p in ps:
        o.state[p]['step'] = torch.tensor(3.0)
        o.state[p]['exp_avg'] = torch.randn_like(p)
        o.state[p]['exp_avg_sq'] = torch.rand_like(p)
    sd = o.state_dict()
    q = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    o2 = FusedAdamW(q, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    o2.load_state_dict(sd)
    for p, pq in zip(ps, q):
        for k in ('step', 'exp_avg', 'exp_avg_sq'):
            assert torch.equal(o2.state[pq][k], o.state[p][k]), k
    sched = torch.optim.lr_scheduler.OneCycleLR(o2, 1e-3, 1000, pct_start=0.05,
                                                cycle_momentum=False, anneal_strategy='linear')
    lr0 = o2.param_groups[0]['lr']
    o2.step = lambda *a, **k: None   # no native library needed for the schedule
    sched.step()
    assert o2.param_groups[0]['lr'] != lr0


def test_fetch_optimizer_cpu_is_torch_adamw():
    m = torch.nn.Linear(4, 3)
    args = argparse.Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100)
    opt, _ = fetch_optimizer(args, m)
    assert isinstance(opt, torch.optim.AdamW)
