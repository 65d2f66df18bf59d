"""One-process-per-GPU data parallelism over RCCL (torch.distributed backend 'nccl' on ROCm).

Replaces the reference's single-process ``nn.DataParallel`` (`train.py:138`, call sites C1-C6 in
`SURVEY.md` §2.4: per-forward parameter broadcast, scatter/gather through GPU0, a non-overlapped
``nccl.reduce`` of gradients to GPU0 and a GPU0-only optimizer step).

Here:
* parameters are broadcast ONCE at start-up; every rank runs the full optimizer step on identical
  all-reduced gradients, so nothing is re-broadcast per step;
* gradients are all-reduced in flat buckets (``GradSync``) launched from post-accumulate-grad hooks
  on a side HIP stream while the rest of backward runs.  Bucket order follows the order in which
  RAFT's gradients become final: the update block (shared across all GRU iterations, final after
  the iteration-0 backward) first, then the encoders from the last layer to the first;
* BatchNorm running statistics follow DataParallel semantics (replica 0's are authoritative):
  ``broadcast_buffers`` copies rank 0's buffers to all ranks, one coalesced broadcast;
* xGMI on MI355X is point-to-point (7 links per GPU), so a handful of multi-MB buckets keeps every
  RCCL ring channel busy; RAFT's 21 MB of fp32 gradients need ~0.1-0.3 ms per step.

CPU tests run the same code with the 'gloo' backend.
"""
import datetime
import os

import torch
import torch.distributed as dist


def env_world():
    return int(os.environ.get('WORLD_SIZE', '1'))


def env_rank():
    return int(os.environ.get('RANK', '0'))


def env_local_rank():
    return int(os.environ.get('LOCAL_RANK', os.environ.get('RANK', '0')))


def is_dist():
    return dist.is_available() and dist.is_initialized()


def rank():
    return dist.get_rank() if is_dist() else 0


def world_size():
    return dist.get_world_size() if is_dist() else 1


def is_main():
    return rank() == 0


def init_distributed(backend=None, device=None, timeout_s=1800):
    """Initialise the default process group from torchrun-style env vars (no-op for world 1).

    Returns the torch.device this rank should use.
    """
    ws = env_world()
    if device is None:
        if torch.cuda.is_available():
            device = torch.device('cuda', env_local_rank() % max(torch.cuda.device_count(), 1))
        else:
            device = torch.device('cpu')
    if device.type == 'cuda':
        torch.cuda.set_device(device)
    if ws > 1 and not is_dist():
        if backend is None:
            # RAFT_DIST_BACKEND=gloo: rehearse the multi-rank GPU path with several ranks on ONE
            # GPU (RCCL refuses two ranks per device); gloo reduces CUDA tensors via the host
            backend = os.environ.get('RAFT_DIST_BACKEND') or \
                ('nccl' if device.type == 'cuda' else 'gloo')
        os.environ.setdefault('MASTER_ADDR', '127.0.0.1')
        os.environ.setdefault('MASTER_PORT', '29511')
        kw = dict(backend=backend, timeout=datetime.timedelta(seconds=timeout_s))
        if backend == 'nccl':
            kw['device_id'] = device
        dist.init_process_group(**kw)
    return device


def barrier(device=None):
    if is_dist():
        if device is not None and device.type == 'cuda' and dist.get_backend() == 'nccl':
            dist.barrier(device_ids=[device.index])
        else:
            dist.barrier()


def destroy():
    if is_dist():
        dist.destroy_process_group()


@torch.no_grad()
def broadcast_module(module, src=0):
    """Broadcast all parameters and buffers from ``src`` (coalesced into one flat buffer per dtype)."""
    if not is_dist():
        return
    tensors = [p.data for p in module.parameters()] + [b for b in module.buffers()]
    _broadcast_coalesced(tensors, src)


@torch.no_grad()
def broadcast_buffers(module, src=0):
    if not is_dist():
        return
    bufs = [b for b in module.buffers()]
    if bufs:
        _broadcast_coalesced(bufs, src)


def _broadcast_coalesced(tensors, src):
    by_dtype = {}
    for t in tensors:
        by_dtype.setdefault((t.dtype, t.device), []).append(t)
    for (_, _), ts in by_dtype.items():
        flat = torch.cat([t.reshape(-1) for t in ts])
        dist.broadcast(flat, src)
        off = 0
        for t in ts:
            n = t.numel()
            t.copy_(flat[off:off + n].view_as(t))
            off += n


def conv_tuning_table():
    """This process's autotuned conv configs: (n, 13) int64 rows (key, config, tile); empty
    without the native library."""
    try:
        from ..ops import _ext
        rows = _ext.ops().conv_tune_table()
    except (AttributeError, RuntimeError, ImportError, OSError):
        return torch.zeros(0, 13, dtype=torch.int64)
    return torch.tensor(rows, dtype=torch.int64).view(-1, 13)


def share_conv_tuning(device, src=0):
    """Rank ``src``'s autotuned conv configs -> every rank (broadcast, then imported into the
    native tile cache), so all ranks launch identical kernels with identical reduction orders.
    Returns the number of rows imported on this rank (0 on ``src``)."""
    if not is_dist():
        return 0
    dev = device if dist.get_backend() == 'nccl' else torch.device('cpu')
    table = conv_tuning_table() if rank() == src else torch.zeros(0, 13, dtype=torch.int64)
    n = torch.tensor([table.shape[0]], dtype=torch.int64, device=dev)
    dist.broadcast(n, src)
    buf = table.to(dev) if rank() == src else torch.zeros(int(n.item()), 13, dtype=torch.int64,
                                                          device=dev)
    if int(n.item()) > 0:
        dist.broadcast(buf, src)
    if rank() == src or int(n.item()) == 0:
        return 0
    from ..ops import _ext
    return int(_ext.ops().conv_tune_import(buf.cpu().reshape(-1).tolist()))


@torch.no_grad()
def all_reduce_mean(t):
    if is_dist():
        dist.all_reduce(t)
        t.div_(world_size())
    return t


class _Bucket:
    __slots__ = ('params', 'numel', 'pending', 'flat', 'work', 'event', 'launched', 'streams')

    def __init__(self, params):
        self.params = params
        self.numel = sum(p.numel() for p in params)
        self.pending = len(params)
        self.flat = None
        self.work = None
        self.event = None
        self.launched = False
        self.streams = set()   # streams the bucket's gradients were accumulated on (this step)


class GradSync:
    """Bucketed, backward-overlapped gradient all-reduce (mean) for a replicated module.

    Usage per step::

        sync.prepare()           # before backward
        loss.backward()          # hooks launch bucket all-reduces as buckets complete
        sync.finish()            # waits, writes averaged grads back (any unfinished bucket too)
    """

    def __init__(self, module, bucket_mb=8.0, comm_dtype=None, order=None, params=None):
        """``params``: sync only these parameters of ``module`` (default: all that require grad);
        ``order(module, params)`` returns them in the order their gradients become final."""
        self.world = world_size()
        self.comm_dtype = comm_dtype
        if params is None:
            params = [p for p in module.parameters() if p.requires_grad]
        else:
            params = [p for p in params if p.requires_grad]
        if order is not None:
            params = order(module, params)
        else:
            params = list(reversed(params))  # last-defined layers finish backward first
        cap = int(bucket_mb * 1024 * 1024)
        self.buckets = []
        cur, cur_bytes = [], 0
        for p in params:
            cur.append(p)
            cur_bytes += p.numel() * p.element_size()
            if cur_bytes >= cap:
                self.buckets.append(_Bucket(cur))
                cur, cur_bytes = [], 0
        if cur:
            self.buckets.append(_Bucket(cur))
        self.bucket_of = {}
        for b in self.buckets:
            for p in b.params:
                self.bucket_of[p] = b
        self.stream = None
        self.enabled = self.world > 1
        self.paused = False
        self.hooks = []
        # overlap evidence: (bucket index, gradients finalised so far) at each bucket launch
        self.hooks_fired = 0
        self.launch_log = []
        if self.enabled:
            for p in params:
                self.hooks.append(p.register_post_accumulate_grad_hook(self._hook))

    def _comm_stream(self, device):
        if device.type != 'cuda':
            return None
        if self.stream is None:
            self.stream = torch.cuda.Stream(device=device)
        return self.stream

    def prepare(self):
        self.hooks_fired = 0
        self.launch_log = []
        for b in self.buckets:
            b.pending = len(b.params)
            b.work = None
            b.launched = False
            b.streams = set()

    @torch.no_grad()
    def _launch(self, b):
        b.launched = True
        ref = b.params[0]
        dev = ref.device
        dtype = self.comm_dtype or ref.dtype
        s = self._comm_stream(dev)
        if s is not None:
            # every stream a gradient of the bucket was accumulated on (the encoders run on
            # several streams, and autograd replays each backward node on its forward's stream)
            s.wait_stream(torch.cuda.current_stream(dev))
            for st in b.streams:
                s.wait_stream(st)
            ctx = torch.cuda.stream(s)
        else:
            ctx = _nullctx()
        with ctx:
            if b.flat is None or b.flat.dtype != dtype or b.flat.device != dev:
                b.flat = torch.empty(b.numel, dtype=dtype, device=dev)
            # parameters without a gradient this step contribute zeros: fill their slice of the
            # flat buffer directly on the comm stream (no main-stream temporaries for it to race)
            off = 0
            for p in b.params:
                n = p.numel()
                dst = b.flat[off:off + n]
                if p.grad is None:
                    dst.zero_()
                else:
                    dst.copy_(p.grad.reshape(-1))
                off += n
            b.flat.div_(self.world)
            b.work = dist.all_reduce(b.flat, async_op=True)

    def _hook(self, p):
        if self.paused:  # a local pass with no collective partner (rank-0 kernel tuning)
            return
        self.hooks_fired += 1
        b = self.bucket_of[p]
        if p.is_cuda:
            b.streams.add(torch.cuda.current_stream(p.device))
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self.launch_log.append((self.buckets.index(b), self.hooks_fired))
            self._launch(b)

    @torch.no_grad()
    def finish(self):
        if not self.enabled:
            return
        for b in self.buckets:
            if not b.launched:  # params that got no grad this step
                self._launch(b)
        dev = self.buckets[0].params[0].device
        s = self._comm_stream(dev)
        for b in self.buckets:
            b.work.wait()
        if s is not None:
            torch.cuda.current_stream(dev).wait_stream(s)
        for b in self.buckets:
            off = 0
            for p in b.params:
                n = p.numel()
                src = b.flat[off:off + n].view_as(p)
                if p.grad is None:
                    p.grad = src.to(p.dtype).clone()
                else:
                    p.grad.copy_(src)
                off += n

    def remove(self):
        for h in self.hooks:
            h.remove()
        self.hooks = []


class _nullctx:
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def raft_grad_order(module, params):
    """Bucket order for RAFT: update block first (final after iteration 0), then cnet / fnet
    from their last layer to their first (the order their backward reaches them)."""
    named = dict((id(p), n) for n, p in module.named_parameters())

    def key(p):
        n = named.get(id(p), '')
        n = n[len('module.'):] if n.startswith('module.') else n
        if n.startswith('update_block'):
            group = 0
        elif n.startswith('cnet'):
            group = 1
        else:
            group = 2
        return group

    order_index = {id(p): i for i, p in enumerate(params)}
    return sorted(params, key=lambda p: (key(p), -order_index[id(p)]))
