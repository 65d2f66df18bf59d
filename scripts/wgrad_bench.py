"""Per-geometry timing of the update block's weight-gradient launches (12 GRU iterations, batch 12,
46x62 at 1/8 resolution): tap-fused kernel vs the packed-K tile kernel, plus their agreement."""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv as C  # noqa: E402

GEOS = [  # name, cout, k, segs
    ('c1', 256, (1, 1), [384]),
    ('c2', 192, (3, 3), [256]),
    ('f1', 128, (1, 1), [128]),
    ('f2', 64, (3, 3), [128]),
    ('conv', 126, (3, 3), [256]),
    ('zr1', 256, (1, 5), [128, 128, 128]),
    ('q1', 128, (1, 5), [128, 128, 128]),
    ('zr2', 256, (5, 1), [128, 128, 128]),
    ('q2', 128, (5, 1), [128, 128, 128]),
    ('head', 512, (3, 3), [128]),
    ('m2', 576, (1, 1), [256]),
]


def main():
    dev = torch.device('cuda')
    B, H, W, n = 12, 46, 62, 12
    torch.manual_seed(0)
    tot = {'taps': 0.0, 'tile': 0.0}
    only = sys.argv[1].split(',') if len(sys.argv) > 1 else None
    impls = sys.argv[2].split(',') if len(sys.argv) > 2 else ['taps', 'tile']
    for name, cout, k, segs in GEOS:
        if only and name not in only:
            continue
        pad = (k[0] // 2, k[1] // 2)
        items = []
        for _ in range(n):
            g = (torch.randn(B, H, W, C.round_up(cout, 8), device=dev) * 0.1).to(torch.bfloat16)
            bufs = [torch.randn(B, H, W, c, device=dev).to(torch.bfloat16) for c in segs]
            items.append((g, bufs))
        kpad = k[0] * k[1] * sum(segs)
        res = {}
        for impl in impls:
            dw = torch.zeros(cout, kpad, device=dev)
            db = torch.zeros(cout, device=dev)

            def run():
                if impl == 'taps':
                    C.conv_wgrad_taps(items, 0, [0] * len(segs), segs, k, pad, cout, dw, db)
                else:
                    C._WG_IMPL_SAVE = C._WG_IMPL
                    C._WG_IMPL = 'tile'
                    C.conv_wgrad_multi(items, 0, [0] * len(segs), segs, k, pad, cout, dw, db)
                    C._WG_IMPL = C._WG_IMPL_SAVE
            run()
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 10
            e0.record()
            for _ in range(reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            us = e0.elapsed_time(e1) * 1e3 / reps
            dw.zero_()
            db.zero_()
            run()
            res[impl] = (us, dw.clone(), db.clone())
            tot[impl] += us
        flops = 2.0 * cout * kpad * B * H * W * n
        line = f'{name:5s} cout {cout:4d} k {k} cin {sum(segs):4d}:'
        for impl in impls:
            line += f' {impl} {res[impl][0]:8.1f} us ({flops / res[impl][0] / 1e6:7.1f} TF/s)'
        if len(impls) == 2:
            d = (res['taps'][1] - res['tile'][1]).abs().max() / res['tile'][1].abs().max()
            line += f'  rel diff {d.item():.2e}'
        print(line, flush=True)
    print('total ' + '  '.join(f'{i} {tot[i]:.1f} us' for i in impls))


if __name__ == '__main__':
    main()
