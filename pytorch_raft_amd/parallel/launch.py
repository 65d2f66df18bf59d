"""Process launcher: ``--gpus 0 1 ...`` semantics of the reference's train.py (`train.py:138,229`)
mapped onto one process per GPU.

If the current process already runs under torchrun (``WORLD_SIZE`` in the environment) the function
is simply called.  Otherwise, for more than one GPU, ``len(gpus)`` worker processes are spawned with
torchrun-style environment variables (rendezvous on 127.0.0.1) and worker ``r`` drives ``gpus[r]``.
"""
import os
import socket

import torch.multiprocessing as mp


def _free_port():
    s = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(local_rank, fn, gpus, port, args):
    os.environ['RANK'] = str(local_rank)
    os.environ['LOCAL_RANK'] = str(local_rank)
    os.environ['WORLD_SIZE'] = str(len(gpus))
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    os.environ['RAFT_AMD_DEVICE'] = str(gpus[local_rank]) if gpus[local_rank] is not None else ''
    fn(args)


def launch(fn, args, gpus):
    """Run ``fn(args)`` once per GPU in ``gpus`` (list of device indices or None for CPU ranks)."""
    if 'WORLD_SIZE' in os.environ or len(gpus) <= 1:
        if len(gpus) == 1 and 'WORLD_SIZE' not in os.environ and gpus[0] is not None:
            os.environ['RAFT_AMD_DEVICE'] = str(gpus[0])
        return fn(args)
    port = _free_port()
    mp.spawn(_worker, args=(fn, list(gpus), port, args), nprocs=len(gpus), join=True)
