"""Diagnose (1) host vs GPU bound eager step, (2) hipGraph training step correctness/timing."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pytorch_raft_amd.models.raft import RAFT
from pytorch_raft_amd.engine.trainer import TrainState, GraphedTrainStep
from pytorch_raft_amd.data.synthetic import device_batches

dev = torch.device('cuda', 0)
torch.backends.cudnn.benchmark = True


def margs():
    return argparse.Namespace(small=False, mixed_precision=True, amp_dtype='bfloat16',
                              alternate_corr=False, dropout=0.0, corr_impl='auto',
                              lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000, iters=12,
                              gamma=0.8, clip=1.0, add_noise=False)


def timed(stepper, batches, n):
    torch.cuda.synchronize()
    host = 0.0
    t0 = time.perf_counter()
    for k in range(n):
        b = batches[k % len(batches)]
        t = time.perf_counter()
        stepper.step(*b)
        host += time.perf_counter() - t
    torch.cuda.synchronize()
    return 1000 * (time.perf_counter() - t0) / n, 1000 * host / n


mode = sys.argv[1] if len(sys.argv) > 1 else 'all'
if mode in ('all', 'host'):
    for B in (1, 4, 12):
        torch.manual_seed(1234)
        a = margs()
        m = RAFT(a).to(dev).train()
        st = TrainState(m, a, dev)
        bs = device_batches(B, 368, 496, dev, count=2)
        timed(st, bs, 4)
        ms, host = timed(st, bs, 10)
        print('eager B=%d: %.2f ms/step, host issue %.2f ms/step' % (B, ms, host), flush=True)

if mode in ('all', 'graph'):
    B = 12
    torch.manual_seed(1234)
    a = margs()
    m = RAFT(a).to(dev).train()
    sd = {k: v.clone() for k, v in m.state_dict().items()}
    bs = device_batches(B, 368, 496, dev, count=2)
    st = TrainState(m, a, dev)
    st.optimizer.zero_grad(set_to_none=True)
    le, _ = st.forward_backward(*bs[0])
    ge = {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}
    print('eager loss', float(le.detach()), flush=True)
    eager = []
    for k in range(3):
        loss, _ = st.step(*bs[k % 2])
        eager.append(float(loss.detach()))
    print('eager losses', eager, flush=True)
    torch.manual_seed(1234)
    m2 = RAFT(a).to(dev).train()
    m2.load_state_dict(sd)
    st2 = TrainState(m2, a, dev, graph_ready=True)
    g = GraphedTrainStep(st2, bs[0], warmup=1)
    print('after capture: nonfinite flag', float(st2.nonfinite), flush=True)
    with torch.no_grad():
        m2.load_state_dict(sd)
    g.static[0].copy_(bs[0][0]); g.static[1].copy_(bs[0][1]); g.static[2].copy_(bs[0][2]); g.static[3].copy_(bs[0][3])
    g.g_fb.replay()
    torch.cuda.synchronize()
    print('graph loss (same weights, batch 0)', float(g.loss), flush=True)
    worst = []
    for n, p in m2.named_parameters():
        if n in ge:
            d = float((p.grad - ge[n]).norm() / (ge[n].norm() + 1e-12))
            fin = bool(torch.isfinite(p.grad).all())
            worst.append((d, n, fin))
    worst.sort(reverse=True)
    print('grad rel diff worst 8:', worst[:8], flush=True)
    print('grad rel diff best 3:', worst[-3:], flush=True)
    gl = []
    for k in range(4):
        loss, _ = g.step(*bs[k % 2])
        gl.append(float(loss))
    print('graph losses', gl, 'nonfinite', float(st2.nonfinite), flush=True)
    ms, host = timed(g, bs, 10)
    print('graph B=12: %.2f ms/step, host issue %.2f ms/step' % (ms, host), flush=True)
    torch.cuda.synchronize()
    t = time.perf_counter(); g.g_fb.replay(); th = time.perf_counter() - t
    torch.cuda.synchronize(); tt = time.perf_counter() - t
    print('g_fb.replay host %.2f ms, to completion %.2f ms' % (1000 * th, 1000 * tt), flush=True)
