"""Window geometry the on-the-fly backward sees in the bench step.

Records the lookup coordinates of one training forward (bench config, on-the-fly correlation)
and reports, per pyramid level, the 8x8-tile bounding boxes (per iteration and the union over
the step's iterations) and how many tiles have every pixel's windows inside a 15x15 grid.
    python scripts/otf_geometry.py [--batch 12] [--iters 12]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_raft_amd.models.raft import RAFT  # noqa: E402
from pytorch_raft_amd.ops import corr as corr_ops  # noqa: E402


def tile_stats(cs, h, w, levels, r=4, tp=8, ug=15):
    E = 2 * r + 2
    out = []
    for l in range(levels):
        hl, wl = h >> l, w >> l
        x0 = torch.stack([torch.floor(c[:, 0] / 2 ** l).long() - r for c in cs])  # (N,B,H,W)
        y0 = torch.stack([torch.floor(c[:, 1] / 2 ** l).long() - r for c in cs])
        hit = (x0 <= wl - 1) & (x0 + E - 1 >= 0) & (y0 <= hl - 1) & (y0 + E - 1 >= 0)
        big = 1 << 20
        n, b = x0.shape[:2]
        ph, pw = (-h) % tp, (-w) % tp

        def tiles(t, fill):
            t = torch.nn.functional.pad(t.float(), (0, pw, 0, ph), value=fill)
            return t.reshape(n, b, (h + ph) // tp, tp, (w + pw) // tp, tp)

        mnx = tiles(torch.where(hit, x0, big), big).amin(dim=(3, 5))
        mxx = tiles(torch.where(hit, x0 + E - 1, -big), -big).amax(dim=(3, 5))
        mny = tiles(torch.where(hit, y0, big), big).amin(dim=(3, 5))
        mxy = tiles(torch.where(hit, y0 + E - 1, -big), -big).amax(dim=(3, 5))

        def area(a, b_, c, d):
            bw = (torch.clamp(b_, max=wl - 1) - torch.clamp(a, min=0) + 1).clamp(min=0)
            bh = (torch.clamp(d, max=hl - 1) - torch.clamp(c, min=0) + 1).clamp(min=0)
            return bw * bh

        per_it = area(mnx, mxx, mny, mxy)                       # (N,B,ty,tx)
        uni = area(mnx.amin(0), mxx.amax(0), mny.amin(0), mxy.amax(0))
        # per-pixel union span over the iterations
        sx = torch.where(hit, x0, big).amin(0), torch.where(hit, x0, -big).amax(0)
        sy = torch.where(hit, y0, big).amin(0), torch.where(hit, y0, -big).amax(0)
        none = sx[0] > sx[1]
        fit = none | ((sx[1] - sx[0] + E <= ug) & (sy[1] - sy[0] + E <= ug))
        tfit = tiles(fit, 1).amin(dim=(3, 5)) > 0
        out.append((l, per_it.float().mean().item(), uni.float().mean().item(),
                    uni.float().max().item(), tfit.float().mean().item()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--batch', type=int, default=12)
    ap.add_argument('--iters', type=int, default=12)
    a = ap.parse_args()
    dev = torch.device('cuda')
    margs = argparse.Namespace(small=False, mixed_precision=True, amp_dtype='bfloat16',
                               alternate_corr=False, dropout=0.0, corr_mode='onthefly',
                               corr_impl='auto', iters=a.iters)
    torch.manual_seed(1234)
    model = RAFT(margs).to(dev).train()
    rec = []
    orig = corr_ops.OnTheFlyVolume.lookup_nhwc

    def spy(self, coords, radius, cbuf):
        rec.append(coords.detach().float().clone())
        return orig(self, coords, radius, cbuf)
    corr_ops.OnTheFlyVolume.lookup_nhwc = spy
    g = torch.Generator(device='cpu').manual_seed(0)
    i1 = torch.rand(a.batch, 3, 368, 496, generator=g).mul(255).to(dev)
    i2 = torch.rand(a.batch, 3, 368, 496, generator=g).mul(255).to(dev)
    with torch.no_grad():
        model(i1, i2, iters=a.iters)
    print('recorded %d lookups, coords %s' % (len(rec), tuple(rec[0].shape)))
    h, w = rec[0].shape[-2:]
    d = torch.stack([(c - rec[0]).abs().amax() for c in rec]).tolist()
    print('max |coords - coords0| per iteration:', ['%.2f' % x for x in d])
    for l, pi, un, umax, fit in tile_stats([c.cpu() for c in rec], h, w, 4):
        print('level %d: mean box per iteration %.0f, union box mean %.0f max %.0f, '
              'tiles on the union-grid path %.1f%%' % (l, pi, un, umax, 100 * fit))


if __name__ == '__main__':
    main()
