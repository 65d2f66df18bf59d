"""Data-parallel rehearsal on the GPU: 2 ranks on ONE MI355X (gloo moves the CUDA tensors through
the host -- RCCL refuses two ranks per device).  Both training paths are covered: the eager step
(bucketed all-reduce from post-accumulate-grad hooks on a side stream) and the hipGraph step
(flat all-reduce between the two replays).  The averaged DP gradient must equal the single-process
full-batch gradient, and the graphed ranks must hold identical weights after two steps."""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    # a free port below the kernel's ephemeral range (32768+): a port handed out by bind(0) is an
    # ephemeral one that an outgoing connection on the shared box can take before the launcher
    # binds it (EADDRINUSE)
    import random
    for _ in range(64):
        p = random.randrange(20000, 32000)
        s = socket.socket()
        try:
            s.bind(('127.0.0.1', p))
            return p
        except OSError:
            continue
        finally:
            s.close()
    raise RuntimeError('no free port in 20000-32000')


def _run(mode, precision, backend):
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    if precision == 'fp32':
        # immediate-mode MIOpen solvers: no per-shape fp32 benchmark search (minutes on a fresh
        # box, and several batch shapes run here); the check compares gradients, not speed
        env.setdefault('MIOPEN_FIND_MODE', 'FAST')
    if backend == 'gloo':
        env['RAFT_DIST_BACKEND'] = 'gloo'
    else:
        env.pop('RAFT_DIST_BACKEND', None)
    for attempt in range(3):
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node',
               '2', '--master-addr', '127.0.0.1', '--master-port', str(_port()),
               os.path.join(ROOT, 'scripts', 'dp_rehearsal.py')] + \
            (['--graph'] if mode == 'graph' else []) + (['--fp32'] if precision == 'fp32' else [])
        r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=170)
        # the rendezvous store failing to bind its port ends the launcher before any rank starts
        # (nothing has touched the GPU): only that case takes another port
        if r.returncode == 0 or 'EADDRINUSE' not in r.stdout + r.stderr:
            return r
    return r


@pytest.mark.parametrize('precision', ['bf16', 'fp32'])
@pytest.mark.parametrize('mode', ['eager', 'graph'])
def test_dp_rehearsal(ext_ops, mode, precision):
    """fp32 pins the all-reduce math (DP gradient == mean of the ranks' same-shape single-process
    gradients to 1e-5, full-batch gradient to 1e-3); the graphed mode also checks that rank 0's
    kernel choices are the ones every rank runs."""
    r = _run(mode, precision, 'gloo')
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'dp rehearsal' in out, out[-2000:]
    print([l for l in out.splitlines() if 'dp rehearsal' in l][0])


@pytest.mark.parametrize('precision', ['bf16', 'fp32'])
def test_dp_rccl_two_gpus(ext_ops, precision):
    """The same graphed DP step over RCCL, one GPU per rank: needs >= 2 visible GPUs (the driver's
    multi-GPU node; skipped on a one-GPU box)."""
    import torch
    if torch.cuda.device_count() < 2:
        pytest.skip('needs 2 GPUs for an RCCL rehearsal')
    r = _run('graph', precision, 'nccl')
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    line = [l for l in out.splitlines() if 'dp rehearsal' in l][0]
    assert 'backend=nccl' in line and 'ranks_identical=True' in line, line
    print(line)
