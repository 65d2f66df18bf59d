"""Uninitialised-memory probe: fill the caching allocator's free memory with 0xFF bytes (NaN in
bf16 and fp32) before each eager training step; a kernel that reads memory it never wrote then
produces NaN.  Also runs the graphed step under a few MIOpen settings.  usage: diag_poison.py <mode>"""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pytorch_raft_amd.models.raft import RAFT
from pytorch_raft_amd.engine.trainer import TrainState, GraphedTrainStep
from pytorch_raft_amd.data.synthetic import device_batches

mode = sys.argv[1]
dev = torch.device('cuda', 0)
torch.cuda.set_device(dev)
torch.backends.cudnn.benchmark = mode != 'graph_nobench'
alt = 'alt' in mode
a = argparse.Namespace(small=False, mixed_precision=True, amp_dtype='bfloat16', alternate_corr=alt,
                       dropout=0.0, corr_impl='auto', lr=4e-4, wdecay=1e-4, epsilon=1e-8,
                       num_steps=100000, iters=12, gamma=0.8, clip=1.0, add_noise=False)
torch.manual_seed(1234)
m = RAFT(a).to(dev).train()
bs = device_batches(12, 368, 496, dev, count=2, seed=0)


def poison(gb=12):
    x = torch.empty(int(gb * 2 ** 30), dtype=torch.uint8, device=dev)
    x.fill_(0xFF)
    del x


if mode.startswith('poison'):
    st = TrainState(m, a, dev)
    for k in range(4):
        poison()
        st.optimizer.zero_grad(set_to_none=True)
        loss, _ = st.forward_backward(*bs[k % 2])
        bad = [n for n, p in m.named_parameters() if p.grad is not None and not torch.isfinite(p.grad).all()]
        print(mode, 'step', k, 'loss', float(loss.detach()), 'nonfinite grads', len(bad), bad[:6], flush=True)
        st.apply_update(loss)
elif mode == 'graph_cmp':
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    st = TrainState(m, a, dev, graph_ready=True)
    g = GraphedTrainStep(st, bs[0], warmup=2)
    gr = []
    for k in range(2):
        for s_, x in zip(g.static, bs[k % 2]):
            s_.copy_(x)
        g.g_fb.replay()
        torch.cuda.synchronize()
        gr.append({n: p.grad.detach().float().clone() for n, p in m.named_parameters()})
        g.g_up.replay()
        g._sched()
        torch.cuda.synchronize()
    # eager reference from the same initial state
    m2 = RAFT(a).to(dev).train()
    m2.load_state_dict(sd)
    st2 = TrainState(m2, a, dev)
    er = []
    for k in range(2):
        st2.optimizer.zero_grad(set_to_none=True)
        loss, _ = st2.forward_backward(*bs[k % 2])
        er.append({n: p.grad.detach().float().clone() for n, p in m2.named_parameters()})
        st2.apply_update(loss)
        st2.scheduler.step()
    for k in range(2):
        rows = []
        for n in er[k]:
            e, q = er[k][n], gr[k][n]
            rows.append((float((q - e).norm() / (e.norm() + 1e-20)), n))
        rows.sort(reverse=True)
        print('replay', k, 'worst', [(round(r, 4), n) for r, n in rows[:12]], flush=True)
        print('replay', k, 'median rel', sorted(r for r, _ in rows)[len(rows) // 2], flush=True)
elif mode == 'graph_which':
    st = TrainState(m, a, dev, graph_ready=True)
    g = GraphedTrainStep(st, bs[0], warmup=2)
    for k in range(3):
        for s_, x in zip(g.static, bs[k % 2]):
            s_.copy_(x)
        g.g_fb.replay()
        torch.cuda.synchronize()
        bad = [n for n, p in m.named_parameters() if not torch.isfinite(p.grad).all()]
        good = [n for n, p in m.named_parameters() if torch.isfinite(p.grad).all()]
        print('replay', k, 'loss', float(g.loss), 'nonfinite', len(bad), bad, flush=True)
        print('replay', k, 'finite', good[:200], flush=True)
        g.g_up.replay()
        g._sched()
        torch.cuda.synchronize()
else:
    st = TrainState(m, a, dev, graph_ready=True)
    g = GraphedTrainStep(st, bs[0], warmup=2)
    out = []
    for k in range(12):
        loss, _ = g.step(*bs[k % 2])
        torch.cuda.synchronize()
        gn = float(torch.cat([p.grad.reshape(-1) for p in g.params]).norm())
        out.append((round(float(loss.detach()), 2), gn == gn))
    print(mode, out, flush=True)
    bad = [n for n, p in m.named_parameters() if not torch.isfinite(p.grad).all()]
    print(mode, 'nonfinite grads at end', len(bad), bad[:8], flush=True)
