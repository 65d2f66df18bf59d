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
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('mode', ['eager', 'graph'])
def test_dp_rehearsal(ext_ops, mode):
    env = dict(os.environ, RAFT_DIST_BACKEND='gloo', MASTER_ADDR='127.0.0.1')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', '2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()),
           os.path.join(ROOT, 'scripts', 'dp_rehearsal.py')] + (['--graph'] if mode == 'graph' else [])
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=160)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert 'dp rehearsal' in out, out[-2000:]
    print([l for l in out.splitlines() if 'dp rehearsal' in l][0])
