"""Multi-process data parallelism on CPU (gloo) -- the fake cluster for the RCCL path."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp
import torch.nn as nn


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


class Toy(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Conv2d(3, 8, 3, padding=1)
        self.bn = nn.BatchNorm2d(8)
        self.b = nn.Conv2d(8, 2, 3, padding=1)

    def forward(self, x):
        h = torch.relu(self.bn(self.a(x)))
        for _ in range(3):  # weight reuse, like the GRU iterations
            h = h + torch.tanh(self.a(x)) * 0.1
        return self.b(h)


def _data():
    g = torch.Generator().manual_seed(0)
    return torch.randn(8, 3, 10, 12, generator=g), torch.randn(8, 2, 10, 12, generator=g)


def _worker(rank, world, port, outdir, bucket_mb):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from pytorch_raft_amd.parallel import dist as pdist
    pdist.init_distributed(device=torch.device('cpu'))
    torch.manual_seed(rank)  # different init on purpose: broadcast must fix it
    m = Toy()
    pdist.broadcast_module(m)
    sync = pdist.GradSync(m, bucket_mb=bucket_mb)
    x, y = _data()
    per = x.shape[0] // world
    xs, ys = x[rank * per:(rank + 1) * per], y[rank * per:(rank + 1) * per]
    sync.prepare()
    loss = (m(xs) - ys).square().mean()
    loss.backward()
    sync.finish()
    grads = [p.grad.clone() for p in m.parameters()]
    torch.save({'grads': grads, 'params': [p.detach().clone() for p in m.parameters()]},
               os.path.join(outdir, 'r%d.pt' % rank))
    pdist.destroy()


@pytest.mark.parametrize('bucket_mb', [0.0001, 8.0])
def test_gradsync_equals_full_batch(tmp_path, bucket_mb):
    world = 2
    mp.spawn(_worker, args=(world, _port(), str(tmp_path), bucket_mb), nprocs=world, join=True)
    r0 = torch.load(str(tmp_path / 'r0.pt'), weights_only=True)
    r1 = torch.load(str(tmp_path / 'r1.pt'), weights_only=True)
    # the broadcast made parameters identical
    for a, b in zip(r0['params'], r1['params']):
        assert torch.equal(a, b)
    # single-process gradient over the full batch with rank 0's weights
    m = Toy()
    with torch.no_grad():
        for p, v in zip(m.parameters(), r0['params']):
            p.copy_(v)
    x, y = _data()
    # BN statistics are per replica (DataParallel semantics): emulate with two half batches
    loss = 0.5 * ((m(x[:4]) - y[:4]).square().mean() + (m(x[4:]) - y[4:]).square().mean())
    loss.backward()
    for p, g0, g1 in zip(m.parameters(), r0['grads'], r1['grads']):
        torch.testing.assert_close(g0, g1)
        torch.testing.assert_close(g0, p.grad, atol=1e-6, rtol=1e-5)


def _train_worker(rank, world, port, outdir):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(2)
    import argparse
    from pytorch_raft_amd.parallel import dist as pdist
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.engine.trainer import TrainState
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    dev = pdist.init_distributed(device=torch.device('cpu'))
    args = argparse.Namespace(small=True, mixed_precision=False, lr=1e-4, wdecay=1e-4, epsilon=1e-8,
                              num_steps=10, iters=2, gamma=0.8, clip=1.0, add_noise=False)
    torch.manual_seed(0)
    m = RAFT(args)
    pdist.broadcast_module(m)
    st = TrainState(m, args, dev)
    i1, i2, f, v = make_pair_batch(1, 128, 128, seed=rank)
    for _ in range(2):
        st.step(i1, i2, f, v)
    assert st.check_finite()
    torch.save([p.detach().clone() for p in m.parameters()], os.path.join(outdir, 't%d.pt' % rank))
    pdist.destroy()


def test_raft_small_dp_training_stays_in_sync(tmp_path):
    world = 2
    mp.spawn(_train_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    a = torch.load(str(tmp_path / 't0.pt'), weights_only=True)
    b = torch.load(str(tmp_path / 't1.pt'), weights_only=True)
    for x, y in zip(a, b):
        assert torch.equal(x, y)
