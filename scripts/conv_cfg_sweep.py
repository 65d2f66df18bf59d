"""Forward / dgrad time of every conv config (forced) per update-block layer at batch 12, 46x62.
usage: conv_cfg_sweep.py [names] [cfgs]"""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv as C  # noqa: E402
from scripts.conv_bench import GEOS, timeit  # noqa: E402


def main():
    only = sys.argv[1].split(',') if len(sys.argv) > 1 and sys.argv[1] != 'all' else None
    cfgs = [int(c) for c in sys.argv[2].split(',')] if len(sys.argv) > 2 else list(range(34))
    dev = torch.device('cuda')
    B, H, W = 12, 46, 62
    from pytorch_raft_amd.ops import _ext
    ops = _ext.ops()
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
        res = []
        for cfg in cfgs:
            ops.conv_set_forced_cfg(cfg)
            try:
                t = timeit(lambda: C.conv_fwd(in_segs, wpk, bias, k, pad, cout, C.EPI_RELU_BF16,
                                              [out], [0]), 20)
                res.append((t, cfg))
            except RuntimeError:
                pass
            finally:
                ops.conv_set_forced_cfg(-1)
        res.sort()
        print(f'{name:5s} ' + '  '.join(f'{c}:{t:.1f}' for t, c in res[:12]), flush=True)


if __name__ == '__main__':
    main()
