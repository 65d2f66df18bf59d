"""Pipelined (no per-step sync) graphed steps, exactly like bench.py: per-step loss / grad-norm
snapshots cloned on device, read after the loop."""
import argparse, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
from pytorch_raft_amd.models.raft import RAFT
from pytorch_raft_amd.engine.trainer import TrainState, GraphedTrainStep
from pytorch_raft_amd.data.synthetic import device_batches
from pytorch_raft_amd.parallel import dist as pdist

dev = pdist.init_distributed()
torch.backends.cudnn.benchmark = True
a = argparse.Namespace(small=False, mixed_precision=True, amp_dtype='bfloat16', alternate_corr=False,
                       dropout=0.0, corr_impl='auto', channels_last=False, lr=4e-4, wdecay=1e-4,
                       epsilon=1e-8, num_steps=100000, iters=12, gamma=0.8, clip=1.0, add_noise=False)
torch.manual_seed(1234)
m = RAFT(a).to(dev).train()
st = TrainState(m, a, dev, graph_ready=True)
bs = device_batches(12, 368, 496, dev, count=2, seed=0)
g = GraphedTrainStep(st, bs[0], warmup=2)
mode = sys.argv[1] if len(sys.argv) > 1 else 'pipelined'
snaps = []
host = []
for k in range(25):
    t = time.perf_counter()
    loss, _ = g.step(*bs[k % 2])
    host.append(time.perf_counter() - t)
    snaps.append((loss.detach().clone(), st.nonfinite.clone(),
                  torch.cat([p.grad.reshape(-1) for p in g.params]).norm()))
    if mode == 'sync':
        torch.cuda.synchronize()
torch.cuda.synchronize()
print(mode, 'losses', [round(float(s[0]), 3) for s in snaps], flush=True)
print(mode, 'nonfinite', [float(s[1]) for s in snaps], flush=True)
print(mode, 'gnorm', [round(float(s[2]), 3) for s in snaps], flush=True)
print(mode, 'host ms', [round(1000 * h, 2) for h in host], flush=True)
