"""20-step loss trajectories: eager vs graphed step (same init, same batches)."""
import argparse, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pytorch_raft_amd.models.raft import RAFT
from pytorch_raft_amd.engine.trainer import TrainState, GraphedTrainStep
from pytorch_raft_amd.data.synthetic import device_batches

dev = torch.device('cuda', 0)
torch.backends.cudnn.benchmark = True
B = int(sys.argv[1]) if len(sys.argv) > 1 else 12
N = 20


def margs():
    return argparse.Namespace(small=False, mixed_precision=True, amp_dtype='bfloat16',
                              alternate_corr=False, dropout=0.0, corr_impl='auto',
                              lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000, iters=12,
                              gamma=0.8, clip=1.0, add_noise=False)


torch.manual_seed(1234)
m = RAFT(margs()).to(dev).train()
sd = {k: v.clone() for k, v in m.state_dict().items()}
bs = device_batches(B, 368, 496, dev, count=2)
st = TrainState(m, margs(), dev)
el = []
for k in range(N):
    loss, _ = st.step(*bs[k % 2])
    el.append(round(float(loss.detach()), 3))
print('eager', el, flush=True)
m2 = RAFT(margs()).to(dev).train()
m2.load_state_dict(sd)
st2 = TrainState(m2, margs(), dev, graph_ready=True)
g = GraphedTrainStep(st2, bs[0], warmup=2)
gl, gn = [], []
for k in range(N):
    loss, _ = g.step(*bs[k % 2])
    gl.append(round(float(loss.detach()), 3))
    gn.append(round(float(torch.cat([p.grad.reshape(-1) for p in m2.parameters()]).norm()), 3))
print('graph', gl, flush=True)
print('graph grad norms', gn, flush=True)
bad = [n for n, p in m2.named_parameters() if not torch.isfinite(p).all()]
print('non-finite params', bad[:10], flush=True)
