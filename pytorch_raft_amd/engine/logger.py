"""Training logger (reference `Logger`, `train.py:89-133`).

Same console format -- ``[{step:6d}, {lr:10.7f}] m1, m2, ...`` with metric names sorted -- and the same
cadence (printed when ``total_steps % SUM_FREQ == SUM_FREQ - 1``).  Differences, all MI355X-driven:

* metrics are pushed as device tensors and summed on the device; the host syncs once per window,
  after ONE all-reduce that averages the window's sums over the data-parallel ranks (the
  reference's DataParallel loss/metrics are computed on the gathered global batch);
* TensorBoard is used if importable, otherwise scalars go to ``runs/<name>/scalars.jsonl``;
* throughput (image pairs / s) is reported alongside the loss metrics.
"""
import json
import os
import time

import torch

SUM_FREQ = 100


class _JsonlWriter:
    def __init__(self, logdir):
        os.makedirs(logdir, exist_ok=True)
        self.f = open(os.path.join(logdir, 'scalars.jsonl'), 'a')

    def add_scalar(self, key, value, step):
        self.f.write(json.dumps({'key': key, 'value': float(value), 'step': int(step),
                                 'time': time.time()}) + '\n')
        self.f.flush()

    def close(self):
        self.f.close()


def make_writer(logdir):
    try:
        from torch.utils.tensorboard import SummaryWriter  # noqa: F401
        return SummaryWriter(logdir)
    except Exception:
        return _JsonlWriter(logdir)


class Logger:
    def __init__(self, model, scheduler, logdir='runs', sum_freq=SUM_FREQ, enabled=True,
                 pairs_per_step=None):
        self.model = model
        self.scheduler = scheduler
        self.total_steps = 0
        self.running = {}
        self.writer = None
        self.logdir = logdir
        self.sum_freq = sum_freq
        self.enabled = enabled
        self.pairs_per_step = pairs_per_step
        self._t0 = time.time()
        self._steps_in_window = 0
        self.history = []

    def _flush(self):
        keys = sorted(self.running.keys())
        vals = torch.stack([self.running[k].detach().float().reshape(()) for k in keys])
        # every rank pushes its own shard's metrics: average them over ranks (SURVEY §2.4 "metrics
        # all-reduced on device every SUM_FREQ steps") -- one small collective per window, and
        # every rank calls _flush at the same step, so the collective is matched
        world = 1
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            world = torch.distributed.get_world_size()
            if world > 1:
                torch.distributed.all_reduce(vals)
        vals = (vals / world).cpu().tolist()
        means = [v / self.sum_freq for v in vals]
        lr = float(self.scheduler.get_last_lr()[0]) if self.scheduler is not None else 0.0
        line = '[{:6d}, {:10.7f}] '.format(self.total_steps + 1, lr)
        line += ('{:10.4f}, ' * len(means)).format(*means)
        dt = time.time() - self._t0
        if self.pairs_per_step and dt > 0:
            line += ' {:.1f} pairs/s'.format(self.pairs_per_step * self._steps_in_window / dt)
        self.history.append(dict(zip(keys, means), step=self.total_steps + 1))
        if self.enabled:
            print(line, flush=True)
            if self.writer is None:
                self.writer = make_writer(self.logdir)
            for k, v in zip(keys, means):
                self.writer.add_scalar(k, v, self.total_steps)
        self._t0 = time.time()
        self._steps_in_window = 0

    def push(self, metrics):
        self.total_steps += 1
        self._steps_in_window += 1
        for k, v in metrics.items():
            v = v if torch.is_tensor(v) else torch.tensor(float(v))
            v = v.detach().float()
            if k in self.running:
                self.running[k] = self.running[k] + v
            else:
                self.running[k] = v.clone()
        if self.total_steps % self.sum_freq == self.sum_freq - 1:
            self._flush()
            self.running = {}

    def write_dict(self, results):
        if not self.enabled:
            return
        if self.writer is None:
            self.writer = make_writer(self.logdir)
        for k, v in results.items():
            self.writer.add_scalar(k, v, self.total_steps)

    def close(self):
        if self.writer is not None:
            self.writer.close()
