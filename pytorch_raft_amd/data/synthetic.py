"""Synthetic frame pairs with known flow (benchmarks, smoke tests, CPU tests).

``SyntheticPairs`` renders a random smooth texture, warps it by a random smooth flow field (so the
pair is actually consistent: image2(x + f(x)) ~= image1(x)) and returns the same 4-tuple as the real
datasets: (img1 (3,H,W) float 0..255, img2, flow (2,H,W), valid (H,W)).

``device_batches`` builds a small pool of such batches directly on the GPU -- used by ``bench.py`` so
the measured step is the training step, not the host data pipeline.
"""
import torch
import torch.nn.functional as F


def _smooth_noise(g, shape, scale, device):
    n, c, h, w = shape
    lo = torch.randn(n, c, max(h // scale, 2), max(w // scale, 2), generator=g, device=device)
    return F.interpolate(lo, size=(h, w), mode='bicubic', align_corners=False)


def make_pair_batch(n, h, w, device='cpu', seed=0, max_flow=20.0):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    tex = _smooth_noise(g, (n, 3, h, w), 8, device) + 0.3 * _smooth_noise(g, (n, 3, h, w), 2, device)
    tex = (tex - tex.amin(dim=(1, 2, 3), keepdim=True))
    tex = tex / tex.amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6) * 255.0
    flow = _smooth_noise(g, (n, 2, h, w), 32, device)
    flow = flow / flow.abs().amax(dim=(1, 2, 3), keepdim=True).clamp_min(1e-6) * max_flow
    # image2 = image1 warped backwards: sample image1 at x - flow (approximate inverse warp)
    ys, xs = torch.meshgrid(torch.arange(h, device=device, dtype=torch.float32),
                            torch.arange(w, device=device, dtype=torch.float32), indexing='ij')
    gx = (xs[None] - flow[:, 0]) / max(w - 1, 1) * 2 - 1
    gy = (ys[None] - flow[:, 1]) / max(h - 1, 1) * 2 - 1
    img2 = F.grid_sample(tex, torch.stack([gx, gy], dim=-1), align_corners=True, padding_mode='border')
    valid = torch.ones(n, h, w, device=device)
    return tex.contiguous(), img2.contiguous(), flow.contiguous(), valid


class SyntheticPairs(torch.utils.data.Dataset):
    def __init__(self, size=(368, 496), length=64, seed=0, max_flow=20.0):
        self.h, self.w = size
        self.length = length
        self.seed = seed
        self.max_flow = max_flow

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        i1, i2, f, v = make_pair_batch(1, self.h, self.w, seed=self.seed * 100003 + idx,
                                       max_flow=self.max_flow)
        return i1[0], i2[0], f[0], v[0]


def device_batches(batch, h, w, device, count=2, seed=0, max_flow=20.0):
    return [make_pair_batch(batch, h, w, device=device, seed=seed + k, max_flow=max_flow)
            for k in range(count)]
