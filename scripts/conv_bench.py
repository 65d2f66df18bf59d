"""Per-geometry timing of the update block's implicit-GEMM convs (one GRU iteration: batch 12,
46x62 at 1/8 resolution), forward (bf16 out) and the adjoint input-gradient conv (fp32 out).
usage: conv_bench.py [names] [reps]"""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv as C  # noqa: E402

GEOS = [  # name, cout, k, cin segs
    ('c1', 256, (1, 1), [384]),
    ('c2', 192, (3, 3), [256]),
    ('f2', 64, (3, 3), [128]),
    ('conv', 126, (3, 3), [256]),
    ('zr1', 256, (1, 5), [128, 128]),   # [h | mf]: the context part is hoisted (update_hip.py)
    ('q1', 128, (1, 5), [128, 128]),
    ('zr2', 256, (5, 1), [128, 128]),
    ('q2', 128, (5, 1), [128, 128]),
    ('head', 512, (3, 3), [128]),
    ('m2', 576, (1, 1), [256]),
]


def timeit(fn, reps):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    only = sys.argv[1].split(',') if len(sys.argv) > 1 and sys.argv[1] != 'all' else None
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device('cuda')
    B, H, W = int(__import__('os').environ.get('CB_BATCH', '12')), 46, 62
    P = B * H * W
    torch.manual_seed(0)
    tot = [0.0, 0.0]
    for name, cout, k, segs in GEOS:
        if only and name not in only:
            continue
        pad = (k[0] // 2, k[1] // 2)
        cin = sum(segs)
        bufs = [torch.randn(B, H, W, c, device=dev).to(torch.bfloat16) for c in segs]
        w = torch.randn(cout, cin, *k, device=dev) * 0.05
        bias = torch.zeros(cout, device=dev)
        wpk = C.pack_weight(w, segs, segs)
        out = torch.empty(B, H, W, C.round_up(cout, 64), device=dev, dtype=torch.bfloat16)
        in_segs = [(b, 0, c) for b, c in zip(bufs, segs)]
        fwd = lambda: C.conv_fwd(in_segs, wpk, bias, k, pad, cout, C.EPI_BF16, [out], [0])  # noqa
        tf = timeit(fwd, reps)
        # adjoint: input = forward output gradient (cout padded to 64), output = fp32 dx
        cpad = C.round_up(cout, 64)
        g = torch.randn(B, H, W, cpad, device=dev).to(torch.bfloat16)
        wd = C.pack_weight_dgrad(w, [cout], [cpad])
        dx = torch.empty(B, H, W, cin, device=dev)
        zb = torch.zeros(cin, device=dev)
        bwd = lambda: C.conv_fwd([(g, 0, cpad)], wd, zb, k, pad, cin, C.EPI_F32, [dx], [0])  # noqa
        tb = timeit(bwd, reps)
        ff = 2.0 * P * cout * cin * k[0] * k[1]
        print(f'{name:5s} {str(k):7s} cin {cin:4d} cout {cout:4d}: fwd {tf:7.1f} us '
              f'({ff / tf / 1e6:6.1f} TF/s)  dgrad {tb:7.1f} us ({ff / tb / 1e6:6.1f} TF/s)',
              flush=True)
        tot[0] += tf
        tot[1] += tb
    print(f'total fwd {tot[0]:.1f} us  dgrad {tot[1]:.1f} us (x12 iterations: '
          f'{12 * tot[0] / 1e3:.2f} / {12 * tot[1] / 1e3:.2f} ms)')


if __name__ == '__main__':
    main()
