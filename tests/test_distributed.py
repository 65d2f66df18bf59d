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


def _subset_worker(rank, world, port, outdir):
    """GradSync over a parameter subset (the graphed step's encoder buckets): only those
    gradients are averaged, the others keep this rank's local value."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(1)
    from pytorch_raft_amd.parallel import dist as pdist
    pdist.init_distributed(device=torch.device('cpu'))
    torch.manual_seed(0)
    m = Toy()
    sub = list(m.a.parameters()) + list(m.bn.parameters())
    sync = pdist.GradSync(m, bucket_mb=0.00002, params=sub)
    assert {id(p) for p in sync.bucket_of} == {id(p) for p in sub} and len(sync.buckets) > 1
    x, y = _data()
    per = x.shape[0] // world
    sync.prepare()
    loss = (m(x[rank * per:(rank + 1) * per]) - y[rank * per:(rank + 1) * per]).square().mean()
    loss.backward()
    sync.finish()
    torch.save({'sub': [p.grad.clone() for p in sub], 'b': [p.grad.clone() for p in m.b.parameters()],
                'log': sync.launch_log, 'n': len(sub)}, os.path.join(outdir, 's%d.pt' % rank))
    pdist.destroy()


def test_gradsync_parameter_subset(tmp_path):
    world = 2
    mp.spawn(_subset_worker, args=(world, _port(), str(tmp_path)), nprocs=world, join=True)
    r0 = torch.load(str(tmp_path / 's0.pt'), weights_only=True)
    r1 = torch.load(str(tmp_path / 's1.pt'), weights_only=True)
    for a, b in zip(r0['sub'], r1['sub']):
        assert torch.equal(a, b)            # averaged over the ranks
    assert any(not torch.equal(a, b) for a, b in zip(r0['b'], r1['b']))  # left local
    # buckets went out from the hooks while the backward still had subset gradients pending
    assert r0['log'][0][1] < r0['n']


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


def _full_worker(rank, world, port, outdir, frozen):
    """Full RAFT (BatchNorm cnet) through the real TrainState / GradSync eager path."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank),
                      MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    torch.set_num_threads(2)
    import argparse
    from pytorch_raft_amd.parallel import dist as pdist
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.engine.trainer import TrainState
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    dev = pdist.init_distributed(device=torch.device('cpu'))
    args = argparse.Namespace(small=False, mixed_precision=False, lr=1e-4, wdecay=1e-4,
                              epsilon=1e-8, num_steps=10, iters=2, gamma=0.8, clip=1e9,
                              add_noise=False, bucket_mb=1.0)
    torch.manual_seed(rank)           # different init on purpose: the broadcast must fix it
    m = RAFT(args).train()
    if frozen:
        m.freeze_bn()
    pdist.broadcast_module(m)
    st = TrainState(m, args, dev)
    assert st.sync is not None and len(st.sync.buckets) > 1
    i1, i2, f, v = make_pair_batch(2 * world, 128, 128, seed=11)
    sl = slice(2 * rank, 2 * rank + 2)
    w0 = [p.detach().clone() for p in m.parameters()]
    bufs0 = [b.detach().clone() for b in m.buffers()]
    st.optimizer.zero_grad(set_to_none=True)
    st.sync.prepare()
    st.forward_backward(i1[sl], i2[sl], f[sl], v[sl])
    st.sync.finish()
    out = dict(grads=[p.grad.detach().clone() for p in m.parameters()], w0=w0, bufs0=bufs0,
               log=list(st.sync.launch_log), hooks=st.sync.hooks_fired,
               bucket_params=[[n for n, q in m.named_parameters() if any(q is x for x in b.params)]
                              for b in st.sync.buckets])
    # BatchNorm buffers: DataParallel keeps replica 0's statistics -> broadcast from rank 0
    pdist.broadcast_buffers(m)
    out['bufs1'] = [b.detach().clone() for b in m.buffers()]
    torch.save(out, os.path.join(outdir, 'f%d.pt' % rank))
    pdist.destroy()


@pytest.mark.parametrize('frozen', [True, False])
def test_full_raft_dp_gradsync_overlap_and_bn_semantics(tmp_path, frozen):
    """Full RAFT, 2 gloo ranks, the real TrainState + GradSync path:
    * buckets follow raft_grad_order and the update-block bucket is all-reduced DURING backward
      (launched before the encoders' gradients are final);
    * with frozen BN (every stage after chairs) the averaged DP gradient equals the single-process
      gradient of the global batch;
    * BN running statistics end identical on every rank (rank 0's, DataParallel semantics)."""
    import argparse
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.engine.trainer import TrainState
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    world = 2
    mp.spawn(_full_worker, args=(world, _port(), str(tmp_path), frozen), nprocs=world, join=True)
    r = [torch.load(str(tmp_path / ('f%d.pt' % k)), weights_only=False) for k in range(world)]
    # bucket order + overlap: the first bucket holds update-block parameters only and launched
    # while encoder gradients were still pending
    assert all(n.startswith('update_block') for n in r[0]['bucket_params'][0])
    first_bucket, fired = r[0]['log'][0]
    assert first_bucket == 0 and fired < r[0]['hooks'], r[0]['log']
    enc_total = sum(len(b) for b in r[0]['bucket_params'][1:])
    assert r[0]['hooks'] - fired >= enc_total // 2
    for a, b in zip(r[0]['grads'], r[1]['grads']):
        assert torch.equal(a, b)
    for a, b in zip(r[0]['bufs1'], r[1]['bufs1']):
        assert torch.equal(a, b)
    if frozen:
        args = argparse.Namespace(small=False, mixed_precision=False, lr=1e-4, wdecay=1e-4,
                                  epsilon=1e-8, num_steps=10, iters=2, gamma=0.8, clip=1e9,
                                  add_noise=False)
        m = RAFT(args).train()
        m.freeze_bn()
        with torch.no_grad():
            for p, w in zip(m.parameters(), r[0]['w0']):
                p.copy_(w)
            for b, v in zip(m.buffers(), r[0]['bufs0']):
                b.copy_(v)
        st = TrainState(m, args, torch.device('cpu'), sync=False)
        i1, i2, f, v = make_pair_batch(2 * world, 128, 128, seed=11)
        st.forward_backward(i1, i2, f, v)
        num = sum(float((p.grad - g).norm() ** 2) for p, g in zip(m.parameters(), r[0]['grads']))
        den = sum(float(p.grad.norm() ** 2) for p in m.parameters())
        assert (num / den) ** 0.5 < 1e-4, (num / den) ** 0.5


def test_bench_cli_two_ranks_cpu(tmp_path):
    """bench.py itself under torch.distributed.run with 2 gloo ranks on the CPU: the JSON line is
    printed once (rank 0), aggregates over ranks and names the data-parallel degree."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', OMP_NUM_THREADS='2')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()),
           os.path.join(root, 'bench.py'), '--gpus', '2', '--steps', '1', '--warmup', '1',
           '--small', '--size', '128', '128', '--iters', '2', '--batch', '1']
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout
    res = json.loads(lines[0])
    assert res['n_gpus'] == 2 and res['config']['parallelism'] == 'dp2'
    assert res['config']['global_batch'] == 2 and res['loss_finite']
