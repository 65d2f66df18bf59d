#!/usr/bin/env python
"""Headline benchmark: RAFT training throughput (image pairs / s, whole node).

Config (BASELINE.json): RAFT full, FlyingChairs-shape 368x496 synthetic pairs, iters=12, per-GPU
batch 12, bf16 autocast, random-init weights, full training step (forward + sequence loss +
backward + RCCL gradient all-reduce + grad-clip + fused AdamW + OneCycle).  Weak scaling: per-GPU
work is fixed, ``value`` is the aggregate over all ranks.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--impl hip|torch] [--alternate_corr]

N>1 is launched by the driver via ``python -m torch.distributed.run --nproc-per-node N ... bench.py
--gpus N``; this script reads RANK / LOCAL_RANK / WORLD_SIZE from the environment.
``--impl torch`` runs the stock reference-semantics ops (MIOpen convs, grid_sample CorrBlock,
unfold upsampling, eager loss): that is the baseline the HIP path is compared with.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

METRIC = ('training image-pairs/sec (whole node), RAFT FlyingChairs 368x496 iters=12, '
          'at 1/2/4/8 MI355X')
# stock PyTorch-ROCm execution of the reference semantics on one MI355X (batch 12,
# 368x496, iters 12, 10 warm-up / 50 timed steps), per compute dtype -- scaled ideally to N GPUs
# for vs_baseline.  A run is compared only with the stock run of ITS dtype at the headline
# config (per-GPU batch 12); any other config reports vs_baseline = null.
STOCK_PAIRS_PER_GPU = {'bf16': 102.705, 'fp32': 66.85}
HEADLINE_BATCH = 12


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch', type=int, default=12, help='per-GPU batch')
    ap.add_argument('--size', type=int, nargs=2, default=[368, 496])
    ap.add_argument('--iters', type=int, default=12)
    ap.add_argument('--impl', choices=['hip', 'torch'], default='hip')
    ap.add_argument('--precision', choices=['bf16', 'fp16', 'fp32'], default='bf16')
    ap.add_argument('--alternate_corr', action='store_true')
    ap.add_argument('--corr_mode', choices=['auto', 'allpairs', 'onthefly'], default='auto',
                    help="auto: all-pairs while the pyramid fits RAFT_CORR_BUDGET_GB, else on-the-fly")
    ap.add_argument('--max_flow', type=float, default=20.0,
                    help='synthetic ground-truth flow magnitude (px)')
    ap.add_argument('--channels_last', action='store_true')
    ap.add_argument('--small', action='store_true')
    ap.add_argument('--freeze_bn', action='store_true',
                    help='frozen context-encoder batch norm (train.py stages after chairs)')
    ap.add_argument('--hipgraph', action='store_true', default=True,
                    help='(default) replay forward+backward and the update as two hipGraphs: the '
                         'host cost of a step drops from ~1000 Python/autograd launches to 2 replays')
    ap.add_argument('--eager', '--no_hipgraph', dest='hipgraph', action='store_false',
                    help='issue every kernel eagerly (RCCL buckets overlapped with backward)')
    ap.add_argument('--profile', type=str, default=None, help='torch.profiler trace dir')
    ap.add_argument('--profile_stack', action='store_true',
                    help='with --profile: record Python stacks and write stacks.txt (ops grouped by '
                         'the source lines that issued them; use with --eager to see the decode)')
    ap.add_argument('--json_out', type=str, default=None)
    ap.add_argument('--dump_tune', type=str, default=None,
                    help='rank 0 writes the conv tile table it ran with (persisted picks + fresh '
                         'autotune picks) to this path (see pytorch_raft_amd/tune_db/)')
    ap.add_argument('--probe_steps', type=int, default=3,
                    help='steps issued on an idle queue after the timed region (host-issue probe; '
                         'more of them = a synchronized-step stress run)')
    ap.add_argument('--trace_markers', action='store_true',
                    help='launch a marker spin kernel right before and after the timed steps')
    ap.add_argument('--roctx_region', action='store_true',
                    help='bracket the timed steps with roctxProfilerResume/Pause '
                         '(use with rocprofv3 --selected-regions)')
    return ap.parse_args(argv)


def _roctx():
    import ctypes
    for name in ('librocprofiler-sdk-roctx.so.1', '/opt/rocm/lib/librocprofiler-sdk-roctx.so'):
        try:
            lib = ctypes.CDLL(name)
            lib.roctxProfilerResume.argtypes = [ctypes.c_uint64]
            lib.roctxProfilerPause.argtypes = [ctypes.c_uint64]
            return lib
        except OSError:
            continue
    return None


def _heartbeat(period=30.0):
    """stderr liveness line every ``period`` s (MIOpen's first-call solver search for the stock /
    fp32 paths can run for minutes without output); stdout stays the single JSON line."""
    import threading

    t0 = time.perf_counter()

    def beat():
        while True:
            time.sleep(period)
            print('bench: alive %.0f s' % (time.perf_counter() - t0), file=sys.stderr, flush=True)

    threading.Thread(target=beat, daemon=True).start()
    # RAFT_STACK_DUMP=<s>: every <s> seconds also print every thread's Python stack (where a
    # slow first step spends its time, without a debugger)
    dump = float(os.environ.get('RAFT_STACK_DUMP', '0') or 0)
    if dump > 0:
        import faulthandler
        faulthandler.dump_traceback_later(dump, repeat=True, file=sys.stderr)


def main(argv=None):
    a = parse(argv)
    if int(os.environ.get('RANK', '0')) == 0:
        _heartbeat()
    import torch
    from pytorch_raft_amd.parallel import dist as pdist
    from pytorch_raft_amd.models.raft import RAFT
    from pytorch_raft_amd.engine.trainer import TrainState
    from pytorch_raft_amd.data.synthetic import device_batches

    if int(os.environ.get('WORLD_SIZE', '1')) != a.gpus and a.gpus > 1 and 'WORLD_SIZE' not in os.environ:
        # convenience: self-launch when run directly with --gpus N
        import subprocess
        import socket
        with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:  # a free rendezvous port
            s.bind(('127.0.0.1', 0))
            port = s.getsockname()[1]
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1',
               '--nproc-per-node', str(a.gpus), '--master-addr', '127.0.0.1',
               '--master-port', str(port), os.path.abspath(__file__)] + (argv or sys.argv[1:])
        sys.exit(subprocess.call(cmd))

    device = pdist.init_distributed()
    world = pdist.world_size()
    rank = pdist.rank()
    torch.manual_seed(1234 + rank)
    torch.backends.cudnn.benchmark = True

    margs = argparse.Namespace(
        small=a.small, mixed_precision=a.precision != 'fp32',
        amp_dtype='float16' if a.precision == 'fp16' else 'bfloat16',
        alternate_corr=a.alternate_corr, dropout=0.0, corr_mode=a.corr_mode,
        corr_impl='torch' if a.impl == 'torch' else 'auto',
        channels_last=a.channels_last,
        lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000, iters=a.iters, gamma=0.8,
        clip=1.0, add_noise=False)
    torch.manual_seed(1234)  # identical init on every rank (also broadcast below)
    model = RAFT(margs).to(device)
    if a.channels_last:
        model = model.to(memory_format=torch.channels_last)
    model.train()
    if a.freeze_bn:
        model.freeze_bn()
    pdist.broadcast_module(model)
    if a.impl == 'torch':
        import pytorch_raft_amd.ops.loss as L
        _orig = L.sequence_loss

        def _torch_loss(*x, **k):
            k['impl'] = 'torch'
            return _orig(*x, **k)
        import pytorch_raft_amd.engine.trainer as T
        T.sequence_loss = _torch_loss
    # the graphed step replays the decode (bf16 / fp16: fused update block, fp16 with the
    # device-side GradScaler inside the fused AdamW step; fp32: split-bf16 MFMA convs, no MIOpen
    # call)
    use_graph = device.type == 'cuda' and a.hipgraph and a.impl == 'hip'

    st = TrainState(model, margs, device, graph_ready=use_graph)

    h, w = a.size
    batches = device_batches(a.batch, h, w, device, count=2, seed=17 * rank, max_flow=a.max_flow)

    if use_graph:
        from pytorch_raft_amd.engine.trainer import GraphedTrainStep
        # capture runs 2 eager warm-up steps (rolled back afterwards), then records the graphs;
        # the a.warmup untimed steps below are graph replays
        stepper = GraphedTrainStep(st, batches[0], warmup=2)
    else:
        stepper = st

    host_issue = []

    last_note = [time.perf_counter()]

    def run(n):
        for k in range(n):
            i1, i2, fl, va = batches[k % len(batches)]
            t_issue = time.perf_counter()
            stepper.step(i1, i2, fl, va)
            host_issue.append(time.perf_counter() - t_issue)
            if rank == 0 and time.perf_counter() - last_note[0] > 20.0:
                # liveness for long (fp32 / stock) runs; stdout stays the single JSON line
                print('bench: step %d/%d issued' % (k + 1, n), file=sys.stderr, flush=True)
                last_note[0] = time.perf_counter()

    run(a.warmup)
    if device.type == 'cuda':
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats()
    pdist.barrier(device)
    prof = None
    if a.profile and rank == 0:
        from torch.profiler import profile, ProfilerActivity
        prof = profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=False,
                       with_stack=a.profile_stack)
        prof.__enter__()
    roctx = _roctx() if a.roctx_region else None
    if roctx is not None:
        roctx.roctxProfilerResume(0)
    if a.trace_markers and device.type == 'cuda':
        # a tiny spin kernel on each side of the timed steps: scripts/prof_diff.py --markers
        # aggregates exactly the kernels between them in a plain --kernel-trace
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(a.steps)
    if device.type == 'cuda':
        torch.cuda.synchronize()
    pdist.barrier(device)
    elapsed = time.perf_counter() - t0
    if a.trace_markers and device.type == 'cuda':
        torch.cuda._sleep(1000)
        torch.cuda.synchronize()
    if roctx is not None:
        roctx.roctxProfilerPause(0)
    if prof is not None:
        prof.__exit__(None, None, None)
        os.makedirs(a.profile, exist_ok=True)
        with open(os.path.join(a.profile, 'ops.txt'), 'w') as f:
            f.write(prof.key_averages().table(sort_by='self_cuda_time_total', row_limit=80))
            f.write('\n\n')
            f.write(prof.key_averages().table(sort_by='cuda_time_total', row_limit=60))
        if a.profile_stack:
            with open(os.path.join(a.profile, 'stacks.txt'), 'w') as f:
                f.write(prof.key_averages(group_by_stack_n=7).table(
                    sort_by='self_cuda_time_total', row_limit=400, max_name_column_width=60))
    # host cost of issuing one step on an idle queue (outside the timed region): in the timed
    # loop the host runs ahead until the HIP queue is full, so per-step issue time there is
    # back-pressure, not host work
    probe = []
    for k in range(max(1, a.probe_steps)):
        if device.type == 'cuda':
            torch.cuda.synchronize()
        i1, i2, fl, va = batches[k % len(batches)]
        t_issue = time.perf_counter()
        stepper.step(i1, i2, fl, va)
        probe.append(time.perf_counter() - t_issue)
    if device.type == 'cuda':
        torch.cuda.synchronize()
    if a.dump_tune and rank == 0 and device.type == 'cuda':
        from pytorch_raft_amd.ops import _ext
        n = _ext.dump_conv_tune_db(a.dump_tune)
        print('bench: %d conv tile picks -> %s' % (n, a.dump_tune), file=sys.stderr, flush=True)
    t = torch.tensor([elapsed], device=device, dtype=torch.float64)
    if pdist.is_dist():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(t.item())
    peak = torch.cuda.max_memory_allocated(device) / 2 ** 30 if device.type == 'cuda' else 0.0
    # a hipGraph replay allocates nothing (its private pool was sized at capture): the reserved
    # peak is the footprint that includes the graphed decode's buffers
    reserved = torch.cuda.max_memory_reserved(device) / 2 ** 30 if device.type == 'cuda' else 0.0
    nonfinite_steps = float(st.nonfinite.item())
    ok = st.check_finite()
    pairs = a.batch * world * a.steps
    value = pairs / elapsed
    metric = METRIC
    if (h, w) != (368, 496) or a.iters != 12 or a.small:
        metric = 'training image-pairs/sec (whole node), RAFT%s %dx%d iters=%d, at %d MI355X' % (
            '-small' if a.small else '', h, w, a.iters, world)
    extra = []
    if a.precision != 'bf16':
        extra.append(a.precision)
    if a.batch != HEADLINE_BATCH:
        extra.append('per-GPU batch %d' % a.batch)
    if extra:
        metric += ' [%s]' % ', '.join(extra)
    base = STOCK_PAIRS_PER_GPU.get(a.precision)
    headline = ((h, w) == (368, 496) and a.iters == 12 and not a.small and not a.freeze_bn
                and a.batch == HEADLINE_BATCH and base is not None)
    res = {
        'metric': metric,
        'value': round(value, 3),
        'unit': 'image-pairs/s',
        'n_gpus': world,
        'steps': a.steps,
        'warmup': a.warmup,
        'ms_per_step': round(1000.0 * elapsed / a.steps, 3),
        'higher_is_better': True,
        'scaling': 'weak',
        'vs_baseline': round(value / (base * world), 3) if headline else None,
        'dtype': a.precision,
        'data': 'synthetic (random smooth texture pairs, %dx%d, generated on device; random-init weights)' % (h, w),
        'config': {
            'model': 'RAFT-small' if a.small else 'RAFT (full, 5.26M params)',
            'global_batch': a.batch * world,
            'per_gpu_batch': a.batch,
            'seq_len': None,
            'image_size': [h, w],
            'iters': a.iters,
            'parallelism': 'dp%d' % world,
            'impl': a.impl,
            'corr': getattr(model, 'last_corr', None), 'corr_mode': a.corr_mode,
            'hipgraph': use_graph,
            'freeze_bn': a.freeze_bn,
        },
        'peak_hbm_gib_rank0': round(peak, 2),
        'peak_reserved_gib_rank0': round(reserved, 2),
        'loss_finite': ok,
        'nonfinite_steps': nonfinite_steps,
        # host time to issue one step on an idle queue (3 extra untimed steps); vs ms_per_step
        # it says how far the step is from being host-bound
        'host_issue_ms': round(1000.0 * sum(probe) / len(probe), 3),
        # issue time inside the timed loop (includes waiting on a full HIP queue)
        'host_issue_pipelined_ms': round(1000.0 * sum(host_issue[-a.steps:]) / max(1, a.steps), 3),
    }
    if rank == 0:
        line = json.dumps(res)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, 'w') as f:
                f.write(line + '\n')
    pdist.destroy()


if __name__ == '__main__':
    main()
