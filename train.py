#!/usr/bin/env python
"""RAFT training CLI -- flag-compatible with the reference `train.py:217-247`.

    python train.py --name raft-chairs --stage chairs --validation chairs --gpus 0 1 \
        --num_steps 100000 --batch_size 10 --lr 0.0004 --image_size 368 496 --wdecay 0.0001

Differences (additive only):
* ``--gpus`` spawns one process per listed GPU (RCCL data parallel) instead of nn.DataParallel;
  ``--batch_size`` stays the GLOBAL batch.  Under torchrun the environment decides.
* ``--mixed_precision`` autocasts to bf16 by default on MI355X (``--amp_dtype float16`` for fp16 +
  GradScaler like the reference).
* new: ``--alternate_corr`` (differentiable on-the-fly correlation), ``--corr_impl``,
  ``--synthetic`` (no dataset needed), ``--resume`` (optimizer/scheduler/step sidecar),
  ``--val_freq``, ``--sum_freq``, ``--num_workers``, ``--channels_last``, ``--profile``,
  ``--checkpoint_dir``, ``--hipgraph`` (graph-replayed training step).
"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_raft_amd.models.raft import RAFT  # noqa: E402
from pytorch_raft_amd.parallel import dist as pdist  # noqa: E402
from pytorch_raft_amd.parallel.launch import launch  # noqa: E402
from pytorch_raft_amd.engine.trainer import TrainState  # noqa: E402
from pytorch_raft_amd.engine.logger import Logger  # noqa: E402
from pytorch_raft_amd.engine.optim import count_parameters  # noqa: E402
from pytorch_raft_amd.engine import checkpoint as ckpt  # noqa: E402
from pytorch_raft_amd.engine import evaluate  # noqa: E402

MAX_FLOW = 400
SUM_FREQ = 100
VAL_FREQ = 5000


def build_parser():
    p = argparse.ArgumentParser()
    p.add_argument('--name', default='raft', help='name your experiment')
    p.add_argument('--stage', help='determines which dataset to use for training')
    p.add_argument('--restore_ckpt', help='restore checkpoint')
    p.add_argument('--small', action='store_true', help='use small model')
    p.add_argument('--validation', type=str, nargs='+')
    p.add_argument('--lr', type=float, default=0.00002)
    p.add_argument('--num_steps', type=int, default=100000)
    p.add_argument('--batch_size', type=int, default=6)
    p.add_argument('--image_size', type=int, nargs='+', default=[384, 512])
    p.add_argument('--gpus', type=int, nargs='+', default=[0, 1])
    p.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    p.add_argument('--iters', type=int, default=12)
    p.add_argument('--wdecay', type=float, default=.00005)
    p.add_argument('--epsilon', type=float, default=1e-8)
    p.add_argument('--clip', type=float, default=1.0)
    p.add_argument('--dropout', type=float, default=0.0)
    p.add_argument('--gamma', type=float, default=0.8, help='exponential weighting')
    p.add_argument('--add_noise', action='store_true')
    # additive MI355X-native options
    p.add_argument('--alternate_corr', action='store_true', help='on-the-fly correlation (O(HW) memory)')
    p.add_argument('--corr_impl', default='auto', choices=['auto', 'hip', 'torch'])
    p.add_argument('--amp_dtype', default='bfloat16', choices=['bfloat16', 'float16'])
    p.add_argument('--channels_last', action='store_true')
    p.add_argument('--synthetic', action='store_true', help='train on synthetic pairs (no dataset)')
    p.add_argument('--resume', action='store_true', help='resume optimizer/scheduler/step from sidecar')
    p.add_argument('--val_freq', type=int, default=VAL_FREQ)
    p.add_argument('--sum_freq', type=int, default=SUM_FREQ)
    p.add_argument('--num_workers', type=int, default=4)
    p.add_argument('--checkpoint_dir', default='checkpoints')
    p.add_argument('--logdir', default=None)
    p.add_argument('--bucket_mb', type=float, default=8.0)
    p.add_argument('--seed', type=int, default=1234)
    p.add_argument('--profile', type=str, default=None, help='write a torch.profiler trace here')
    p.add_argument('--cpu', action='store_true', help='force CPU (gloo) training')
    p.add_argument('--hipgraph', dest='hipgraph', action='store_true', default=True,
                   help='(default on a GPU) replay the recurrent part of each step -- correlation, '
                        'GRU iterations fwd+bwd, upsampling, loss -- as one hipGraph; encoders and '
                        'the update run eagerly around it (fixed crop; bf16 or fp32)')
    p.add_argument('--eager', '--no_hipgraph', dest='hipgraph', action='store_false',
                   help='issue every kernel of the step eagerly')
    p.add_argument('--enc_bucket_mb', type=float, default=2.0,
                   help='graphed step, ranks > 1: encoder gradient bucket size (MB)')
    return p


def _synthetic_loader(args, rank, world):
    from pytorch_raft_amd.data.synthetic import SyntheticPairs
    ds = SyntheticPairs(size=tuple(args.image_size), length=max(64, args.batch_size * 8), seed=rank)
    from pytorch_raft_amd.data.datasets import per_rank_batch
    per_rank = per_rank_batch(args.batch_size, world, rank)
    return torch.utils.data.DataLoader(ds, batch_size=per_rank, shuffle=True, drop_last=True,
                                       num_workers=0)


def worker(args):
    dev_env = os.environ.get('RAFT_AMD_DEVICE', '')
    device = None
    if args.cpu or not torch.cuda.is_available():
        device = torch.device('cpu')
    elif dev_env:
        device = torch.device('cuda', int(dev_env))
    device = pdist.init_distributed(device=device)
    rank, world = pdist.rank(), pdist.world_size()
    if device.type == 'cuda':
        # fixed crop size: let MIOpen time its encoder conv solvers once and keep the fastest
        torch.backends.cudnn.benchmark = True
    torch.manual_seed(args.seed)  # identical init on every rank (weights are also broadcast)
    np.random.seed(args.seed)

    model = RAFT(args)
    if rank == 0:
        print('Parameter Count: %d' % count_parameters(model))
    if args.restore_ckpt is not None:
        ckpt.load_weights(model, args.restore_ckpt, strict=False)
    model.to(device)
    if args.channels_last:
        model = model.to(memory_format=torch.channels_last)
    model.train()
    if args.stage != 'chairs':
        model.freeze_bn()
    pdist.broadcast_module(model)
    # after the weights are in sync, every rank draws its own device-side noise / dropout stream
    # (one DataParallel process would draw different numbers for each replica's slice)
    torch.manual_seed(args.seed + rank)
    np.random.seed(args.seed + rank)

    if args.synthetic or args.stage is None:
        loader = _synthetic_loader(args, rank, world)
    else:
        from pytorch_raft_amd.data.datasets import fetch_dataloader
        loader = fetch_dataloader(args, rank=rank, world=world, num_workers=args.num_workers)

    # fp16 autocast needs the GradScaler's host-side inf checks: that step runs eagerly
    use_graph = (args.hipgraph and device.type == 'cuda' and
                 not (args.mixed_precision and args.amp_dtype == 'float16'))
    st = TrainState(model, args, device, graph_ready=use_graph)
    stepper = st  # replaced by the graphed step at the first batch (capture needs its shapes)
    total_steps = 0
    if args.resume and args.restore_ckpt is not None:
        s = ckpt.load_training_state(args.restore_ckpt, st.optimizer, st.scheduler, st.scaler)
        if s is not None:
            total_steps = int(s['step'])
    per_rank = max(1, args.batch_size // world)  # per_rank_batch() already warned on rank 0
    logger = Logger(model, st.scheduler, logdir=args.logdir or os.path.join('runs', args.name),
                    sum_freq=args.sum_freq, enabled=(rank == 0), pairs_per_step=per_rank * world)
    logger.total_steps = total_steps
    os.makedirs(args.checkpoint_dir, exist_ok=True)

    prof = None
    if args.profile and rank == 0:
        from torch.profiler import profile, ProfilerActivity, schedule
        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA],
                       schedule=schedule(wait=2, warmup=2, active=5, repeat=1),
                       on_trace_ready=torch.profiler.tensorboard_trace_handler(args.profile))
        prof.__enter__()

    should_keep_training = True
    epoch = 0
    t_start = time.time()
    while should_keep_training:
        if hasattr(loader, 'sampler') and hasattr(loader.sampler, 'set_epoch'):
            loader.sampler.set_epoch(epoch)
        for data_blob in loader:
            image1, image2, flow, valid = [x.to(device, non_blocking=True) for x in data_blob]
            if use_graph and stepper is st:
                from pytorch_raft_amd.engine.trainer import GraphedTrainStep
                stepper = GraphedTrainStep(st, (image1, image2, flow, valid), warmup=2)
            loss, metrics = stepper.step(image1, image2, flow, valid)
            logger.push({k: v for k, v in metrics.items() if k != 'loss'})
            if prof is not None:
                prof.step()

            if total_steps % args.sum_freq == args.sum_freq - 1:
                if not st.check_finite():
                    raise FloatingPointError('non-finite loss detected at step %d' % (total_steps + 1))

            if total_steps % args.val_freq == args.val_freq - 1:
                if rank == 0:
                    path = os.path.join(args.checkpoint_dir, '%d_%s.pth' % (total_steps + 1, args.name))
                    ckpt.save_weights(model, path)
                    ckpt.save_training_state(path, st.optimizer, st.scheduler, total_steps + 1, st.scaler)
                    results = {}
                    for val_dataset in (args.validation or []):
                        results.update(evaluate.VALIDATORS[val_dataset](model))
                    logger.write_dict(results)
                pdist.barrier(device)
                model.train()
                if args.stage != 'chairs':
                    model.freeze_bn()

            total_steps += 1
            if total_steps > args.num_steps:
                should_keep_training = False
                break
        epoch += 1

    if prof is not None:
        prof.__exit__(None, None, None)
    logger.close()
    path = os.path.join(args.checkpoint_dir, '%s.pth' % args.name)
    if rank == 0:
        ckpt.save_weights(model, path)
        ckpt.save_training_state(path, st.optimizer, st.scheduler, total_steps, st.scaler)
        print('done: %d steps in %.1fs -> %s' % (total_steps, time.time() - t_start, path))
    pdist.barrier(device)
    pdist.destroy()
    return path


def train(args):
    gpus = args.gpus
    if args.cpu or not torch.cuda.is_available():
        gpus = [None] * max(1, len(gpus) if 'WORLD_SIZE' not in os.environ else 1)
        if len(gpus) > 1:
            args.cpu = True
    else:
        n = torch.cuda.device_count()
        gpus = [g for g in gpus if g < n] or [0]
    return launch(worker, args, gpus)


if __name__ == '__main__':
    args = build_parser().parse_args()
    torch.manual_seed(args.seed)
    np.random.seed(args.seed)
    if not os.path.isdir(args.checkpoint_dir):
        os.makedirs(args.checkpoint_dir, exist_ok=True)
    train(args)
