"""Small tensor utilities shared by the model, evaluation and demos.

Behavioural parity with reference `core/utils/utils.py`:

* ``InputPadder``        replicate-pad to a multiple of 8 ('sintel' centres both axes, any other mode
                         pads only the bottom for height) and ``unpad`` back (`:7-24`).
* ``forward_interpolate`` forward-splat a 1/8 flow and fill holes by nearest neighbour (`:26-54`).
                         Used for the Sintel warm start.  Implemented with a KD-tree nearest search
                         (scipy ``cKDTree``) which is what ``griddata(method='nearest')`` does.
* ``bilinear_sampler``   pixel-coordinate wrapper of ``grid_sample(align_corners=True)`` (`:57-71`).
* ``coords_grid``        (B, 2, H, W) grid, channel 0 = x, 1 = y (`:74-77`).
* ``upflow8``            8 x bilinear(align_corners=True) upsample of a flow field (`:80-82`).
"""
import numpy as np
import torch
import torch.nn.functional as F


class InputPadder:
    """Pads images such that both spatial dims are divisible by 8."""

    def __init__(self, dims, mode='sintel'):
        self.ht, self.wd = dims[-2:]
        pad_ht = (-self.ht) % 8
        pad_wd = (-self.wd) % 8
        left, right = pad_wd // 2, pad_wd - pad_wd // 2
        if mode == 'sintel':
            top, bottom = pad_ht // 2, pad_ht - pad_ht // 2
        else:
            top, bottom = 0, pad_ht
        # F.pad order: (left, right, top, bottom)
        self._pad = [left, right, top, bottom]

    def pad(self, *inputs):
        return [F.pad(x, self._pad, mode='replicate') for x in inputs]

    def unpad(self, x):
        ht, wd = x.shape[-2:]
        left, right, top, bottom = self._pad
        return x[..., top:ht - bottom, left:wd - right]


def coords_grid(batch, ht, wd, device=None, dtype=torch.float32):
    ys, xs = torch.meshgrid(torch.arange(ht, device=device, dtype=dtype),
                            torch.arange(wd, device=device, dtype=dtype), indexing='ij')
    grid = torch.stack([xs, ys], dim=0)
    return grid[None].expand(batch, 2, ht, wd).contiguous()


def bilinear_sampler(img, coords, mode='bilinear', mask=False):
    """Sample ``img`` (N, C, H, W) at pixel coords (N, h, w, 2) with x first, zero padding."""
    H, W = img.shape[-2:]
    x, y = coords[..., 0:1], coords[..., 1:2]
    gx = 2.0 * x / (W - 1) - 1.0
    gy = 2.0 * y / (H - 1) - 1.0
    grid = torch.cat([gx, gy], dim=-1)
    out = F.grid_sample(img, grid, mode=mode, align_corners=True)
    if mask:
        inside = (gx > -1) & (gy > -1) & (gx < 1) & (gy < 1)
        return out, inside.float()
    return out


def upflow8(flow, mode='bilinear'):
    size = (8 * flow.shape[2], 8 * flow.shape[3])
    return 8.0 * F.interpolate(flow, size=size, mode=mode, align_corners=True)


def forward_interpolate(flow):
    """Forward-warp a (2, H, W) flow to the next frame, filling holes with the nearest splat.

    Returns a float32 CPU tensor (2, H, W) (reference returns a CPU tensor too).
    """
    from scipy.spatial import cKDTree

    f = flow.detach().float().cpu().numpy()
    dx, dy = f[0], f[1]
    ht, wd = dx.shape
    x0, y0 = np.meshgrid(np.arange(wd), np.arange(ht))
    x1 = (x0 + dx).reshape(-1)
    y1 = (y0 + dy).reshape(-1)
    dxf, dyf = dx.reshape(-1), dy.reshape(-1)
    keep = (x1 > 0) & (x1 < wd) & (y1 > 0) & (y1 < ht)
    if not np.any(keep):
        return torch.zeros(2, ht, wd, dtype=torch.float32)
    pts = np.stack([x1[keep], y1[keep]], axis=1)
    tree = cKDTree(pts)
    q = np.stack([x0.reshape(-1), y0.reshape(-1)], axis=1).astype(np.float64)
    _, idx = tree.query(q, k=1)
    out = np.stack([dxf[keep][idx].reshape(ht, wd), dyf[keep][idx].reshape(ht, wd)], axis=0)
    return torch.from_numpy(out.astype(np.float32))
