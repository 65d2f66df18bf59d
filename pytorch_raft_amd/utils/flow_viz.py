"""Optical-flow colour coding (Baker et al., ICCV 2007 / Middlebury colour wheel).

Same public functions and output as the reference (`core/utils/flow_viz.py:20-132`):
``make_colorwheel()`` (55 x 3), ``flow_uv_to_colors(u, v, convert_to_bgr=False)`` and
``flow_to_image(flow_uv, clip_flow=None, convert_to_bgr=False)`` (normalised by the max radius).
Implemented vectorised over the three channels.
"""
import numpy as np

# hue segment lengths: red-yellow, yellow-green, green-cyan, cyan-blue, blue-magenta, magenta-red
_SEGMENTS = (15, 6, 4, 11, 13, 6)


def make_colorwheel():
    ncols = sum(_SEGMENTS)
    wheel = np.zeros((ncols, 3))
    start = 0
    # each segment ramps one channel while holding another at 255
    ramps = [  # (rising/falling channel, held channel, rising?)
        (1, 0, True), (0, 1, False), (2, 1, True), (1, 2, False), (0, 2, True), (2, 0, False)]
    for n, (ramp_ch, hold_ch, rising) in zip(_SEGMENTS, ramps):
        t = np.floor(255 * np.arange(n) / n)
        wheel[start:start + n, hold_ch] = 255
        wheel[start:start + n, ramp_ch] = t if rising else 255 - t
        start += n
    return wheel


def flow_uv_to_colors(u, v, convert_to_bgr=False):
    img = np.zeros((u.shape[0], u.shape[1], 3), np.uint8)
    wheel = make_colorwheel()
    ncols = wheel.shape[0]
    rad = np.sqrt(np.square(u) + np.square(v))
    ang = np.arctan2(-v, -u) / np.pi
    fk = (ang + 1) / 2 * (ncols - 1)
    k0 = np.floor(fk).astype(np.int32)
    k1 = k0 + 1
    k1[k1 == ncols] = 0
    f = (fk - k0)[..., None]
    col = (1 - f) * wheel[k0] / 255.0 + f * wheel[k1] / 255.0  # (H, W, 3)
    inside = (rad <= 1)[..., None]
    col = np.where(inside, 1 - rad[..., None] * (1 - col), col * 0.75)
    out = np.floor(255 * col)
    if convert_to_bgr:
        out = out[..., ::-1]
    img[...] = out
    return img


def flow_to_image(flow_uv, clip_flow=None, convert_to_bgr=False):
    assert flow_uv.ndim == 3, 'input flow must have three dimensions'
    assert flow_uv.shape[2] == 2, 'input flow must have shape [H,W,2]'
    if clip_flow is not None:
        flow_uv = np.clip(flow_uv, 0, clip_flow)
    u, v = flow_uv[:, :, 0], flow_uv[:, :, 1]
    rad_max = np.max(np.sqrt(np.square(u) + np.square(v)))
    eps = 1e-5
    return flow_uv_to_colors(u / (rad_max + eps), v / (rad_max + eps), convert_to_bgr)
