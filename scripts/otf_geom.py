"""On-the-fly correlation backward geometry at the bench shape: per query tile (8x8) and level, the
union box of all iterations' windows (-> fmap2 chunks of 64 positions) and whether every pixel's
window union fits the kernel's 15x15 grid (the fast dS path).  Eager training steps as bench.py
(chairs 368x496, batch 12, corr_mode onthefly); statistics of the last step's window backward."""
import argparse
import sys

import torch

sys.path.insert(0, '.')
import pytorch_raft_amd.ops.corr as corr  # noqa: E402
from pytorch_raft_amd.models.raft import RAFT  # noqa: E402
from pytorch_raft_amd.engine.trainer import TrainState  # noqa: E402
from pytorch_raft_amd.data.synthetic import device_batches  # noqa: E402

LAST = {}


class _Ops:
    def __init__(self, real):
        self.real = real

    def __getattr__(self, k):
        f = getattr(self.real, k)
        if k != 'corr_otf_window_bwd_':
            return f

        def g(f1, f2, coords, douts, *rest):
            LAST['coords'] = [c.detach().clone() for c in coords]
            LAST['hw'] = [(t.shape[1], t.shape[2]) for t in f2]
            return f(f1, f2, coords, douts, *rest)
        return g


class _Ext:
    def __init__(self, real):
        self.real = real

    def ops(self):
        return _Ops(self.real.ops())

    def __getattr__(self, k):
        return getattr(self.real, k)


def stats(coords, hws, R=4, UG=15):
    E = 2 * R + 2
    B, _, H, W = coords[0].shape
    ty, tx = (H + 7) // 8, (W + 7) // 8
    out = []
    for l, (hl, wl) in enumerate(hws):
        x0s, y0s, hits = [], [], []
        for c in coords:
            cx = (c[:, 0] / 2 ** l).clamp(-1e6, 1e6)
            cy = (c[:, 1] / 2 ** l).clamp(-1e6, 1e6)
            x0 = torch.floor(cx).int() - R
            y0 = torch.floor(cy).int() - R
            hit = (x0 <= wl - 1) & (x0 + E - 1 >= 0) & (y0 <= hl - 1) & (y0 + E - 1 >= 0)
            x0s.append(x0)
            y0s.append(y0)
            hits.append(hit)
        X = torch.stack(x0s)  # (N,B,H,W)
        Y = torch.stack(y0s)
        Hm = torch.stack(hits)
        big = 1 << 30
        # per pixel union spread (over hitting iterations)
        mnx = torch.where(Hm, X, big).amin(0)
        mxx = torch.where(Hm, X, -big).amax(0)
        mny = torch.where(Hm, Y, big).amin(0)
        mxy = torch.where(Hm, Y, -big).amax(0)
        none = mnx > mxx
        fit = none | ((mxx - mnx + E <= UG) & (mxy - mny + E <= UG))
        # pad to tiles
        ph, pw = ty * 8 - H, tx * 8 - W

        def tile(t, val):
            t = torch.nn.functional.pad(t.float(), (0, pw, 0, ph), value=val)
            return t.view(B, ty, 8, tx, 8).permute(0, 1, 3, 2, 4).reshape(B, ty, tx, 64)
        tmnx = tile(torch.where(none, big, mnx), big).amin(-1)
        tmxx = tile(torch.where(none, -big, mxx + E - 1), -big).amax(-1)
        tmny = tile(torch.where(none, big, mny), big).amin(-1)
        tmxy = tile(torch.where(none, -big, mxy + E - 1), -big).amax(-1)
        bx0, bx1 = tmnx.clamp(min=0), tmxx.clamp(max=wl - 1)
        by0, by1 = tmny.clamp(min=0), tmxy.clamp(max=hl - 1)
        ok = (bx1 >= bx0) & (by1 >= by0)
        U = torch.where(ok, (bx1 - bx0 + 1) * (by1 - by0 + 1), torch.zeros_like(bx0))
        chunks = torch.ceil(U / 64)
        tfit = tile(fit, 1.0).amin(-1)
        out.append((l, U.mean().item(), U.max().item(), chunks.mean().item(), chunks.max().item(),
                    1.0 - tfit.mean().item(), (1 - fit.float()).mean().item()))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--batch', type=int, default=12)
    a = ap.parse_args()
    corr._ext = _Ext(corr._ext)
    dev = torch.device('cuda')
    margs = argparse.Namespace(
        small=False, mixed_precision=True, amp_dtype='bfloat16', alternate_corr=False,
        dropout=0.0, corr_mode='onthefly', corr_impl='auto', channels_last=False, lr=4e-4,
        wdecay=1e-4, epsilon=1e-8, num_steps=100000, iters=12, gamma=0.8, clip=1.0,
        add_noise=False)
    torch.manual_seed(1234)
    model = RAFT(margs).to(dev)
    model.train()
    st = TrainState(model, margs, dev, graph_ready=False)
    batches = device_batches(a.batch, 368, 496, dev, count=2, seed=0, max_flow=20.0)
    for k in range(a.steps):
        st.step(*batches[k % 2])
        torch.cuda.synchronize()
        if 'coords' in LAST:
            print('step', k, 'iters', len(LAST['coords']))
            for r in stats(LAST['coords'], LAST['hw']):
                print('  level %d  U mean %.0f max %d  chunks mean %.2f max %d  tiles-not-fit %.3f  px-not-fit %.4f' % r)
            sys.stdout.flush()


if __name__ == '__main__':
    main()
