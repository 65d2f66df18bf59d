#!/usr/bin/env python
"""Inference benchmark (BASELINE.json config 5): RAFT full, Sintel-shape 436x1024 pairs (padded to
440x1024 as `evaluate.py:95-127` does), iters=32, test mode, large batch, hipGraph-captured.

    python bench_infer.py [--batch B] [--steps K] [--warmup W] [--iters 32] [--size 436 1024]
                          [--graph] [--alternate_corr] [--impl hip|torch] [--precision bf16|fp32]

Prints ONE JSON line: image pairs/s on one GPU (each step = one batched ``model(..., test_mode=True)``
call including padding / unpadding), with HIP-synchronised wall time around K steps.
``--impl torch`` is the stock reference-semantics path (MIOpen convs, grid_sample lookups, eager
GRU, per-iteration convex upsample disabled as in our test mode) for comparison.
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=16)
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--iters', type=int, default=32)
    ap.add_argument('--size', type=int, nargs=2, default=[436, 1024])
    ap.add_argument('--graph', action='store_true', help='capture the forward as one hipGraph')
    ap.add_argument('--alternate_corr', action='store_true')
    ap.add_argument('--corr_mode', choices=['auto', 'allpairs', 'onthefly'], default='auto',
                    help="auto: all-pairs while the pyramid fits RAFT_CORR_BUDGET_GB, else on-the-fly")
    ap.add_argument('--impl', choices=['hip', 'torch'], default='hip')
    ap.add_argument('--precision', choices=['bf16', 'fp32'], default='bf16')
    ap.add_argument('--small', action='store_true')
    ap.add_argument('--flow_init_px', type=float, default=0.0,
                    help='warm-start flow magnitude (px at 1/8 res x 8): large lookup coordinates')
    ap.add_argument('--discontinuous', action='store_true',
                    help='flow_init piecewise constant on 4x4-cell blocks (motion boundaries)')
    a = ap.parse_args(argv)

    import torch
    from pytorch_raft_amd.models.raft import RAFT
    from pytorch_raft_amd.engine.inference import FlowInference

    dev = torch.device('cuda', 0) if torch.cuda.is_available() else torch.device('cpu')
    margs = argparse.Namespace(small=a.small, mixed_precision=a.precision == 'bf16',
                               amp_dtype='bfloat16', alternate_corr=a.alternate_corr, dropout=0.0,
                               corr_mode=a.corr_mode,
                               corr_impl='torch' if a.impl == 'torch' else 'auto')
    torch.manual_seed(1234)
    model = RAFT(margs).to(dev).eval()
    runner = FlowInference(model, iters=a.iters, pad_mode='sintel',
                           graph=a.graph and dev.type == 'cuda' and a.impl == 'hip')
    h, w = a.size
    g = torch.Generator(device=dev).manual_seed(7)
    i1 = torch.rand(a.batch, 3, h, w, device=dev, generator=g) * 255
    i2 = torch.roll(i1, shifts=(3, -5), dims=(2, 3)).contiguous()

    finit = None
    if a.flow_init_px > 0:
        ph, pw = (h + 7) // 8, (w + 7) // 8
        if a.discontinuous:
            lo = torch.rand(a.batch, 2, (ph + 3) // 4, (pw + 3) // 4, device=dev, generator=g)
            finit = torch.nn.functional.interpolate(lo, scale_factor=4, mode='nearest')[..., :ph, :pw]
        else:
            lo = torch.rand(a.batch, 2, max(ph // 8, 2), max(pw // 8, 2), device=dev, generator=g)
            finit = torch.nn.functional.interpolate(lo, size=(ph, pw), mode='bilinear',
                                                    align_corners=False)
        # flow at 1/8 resolution is in 1/8-res pixels: +-P full-res px = +-P/8 cells
        finit = ((finit * 2 - 1) * (a.flow_init_px / 8.0)).contiguous()

    for _ in range(a.warmup):
        out = runner(i1, i2, finit)
    if dev.type == 'cuda':
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        out = runner(i1, i2, finit)
    if dev.type == 'cuda':
        torch.cuda.synchronize()
    el = time.perf_counter() - t0
    flow_low, flow_up = out
    finite = bool(torch.isfinite(flow_up).all().item())
    # allocator peak over warm-up + timed steps (a graph replay allocates nothing: its pool was
    # sized during capture, which max_memory_reserved covers) and the device's own used bytes
    peak = torch.cuda.max_memory_allocated(dev) / 2 ** 30 if dev.type == 'cuda' else 0.0
    reserved = torch.cuda.max_memory_reserved(dev) / 2 ** 30 if dev.type == 'cuda' else 0.0
    if dev.type == 'cuda':
        free, total = torch.cuda.mem_get_info(dev)
        used = (total - free) / 2 ** 30
    else:
        used, total = 0.0, 0
    res = {
        'metric': 'inference image-pairs/sec (1 GPU), RAFT Sintel %dx%d iters=%d test_mode' % (h, w, a.iters),
        'value': round(a.batch * a.steps / el, 3),
        'unit': 'image-pairs/s',
        'n_gpus': 1,
        'steps': a.steps,
        'warmup': a.warmup,
        'ms_per_step': round(1000.0 * el / a.steps, 3),
        'ms_per_pair': round(1000.0 * el / (a.steps * a.batch), 3),
        'higher_is_better': True,
        'dtype': a.precision,
        'data': 'synthetic (uniform noise pairs, random-init weights)',
        'config': {'model': 'RAFT-small' if a.small else 'RAFT (full)', 'batch': a.batch,
                   'image_size': [h, w], 'padded': [(h + 7) // 8 * 8, (w + 7) // 8 * 8],
                   'iters': a.iters, 'impl': a.impl, 'hipgraph': runner.graph,
                   'corr': getattr(model, 'last_corr', None), 'corr_mode': a.corr_mode,
                   'flow_init_px': a.flow_init_px, 'discontinuous': a.discontinuous},
        'out_shape': list(flow_up.shape),
        'peak_hbm_gib': round(peak, 2),
        'peak_reserved_gib': round(reserved, 2),
        'device_used_gib': round(used, 2),
        'device_total_gib': round(total / 2 ** 30, 1),
        'finite': finite,
    }
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
