"""Host image ops for the data pipeline / demos: OpenCV-free replacements (native C++ via ctypes).

* ``resize_linear(img, fx=None, fy=None, dsize=None)`` -- ``cv2.resize(..., INTER_LINEAR)`` semantics
  (pixel-centre mapping, replicated border); float32 math, uint8 in -> uint8 out (rounded, saturated).
* ``remap_linear(img, map_xy)`` -- ``cv2.remap(img, map, None, INTER_LINEAR)`` with a constant-0 border.
* ``rgb_to_bgr`` / ``bgr_to_rgb`` channel flips.

The kernels live in ``csrc/cpu/imgproc.cpp`` (``_cpu.so``); a numpy fallback keeps CPU-only machines
without a toolchain working.
"""
import ctypes
import os

import numpy as np

_LIB = None
_LIB_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), '_cpu.so')


def _lib():
    global _LIB
    if _LIB is None:
        if os.path.exists(_LIB_PATH):
            try:
                lib = ctypes.CDLL(_LIB_PATH)
                f = ctypes.c_void_p
                i = ctypes.c_int
                lib.raft_resize_linear_f32.argtypes = [f, i, i, i, f, i, i, ctypes.c_double, ctypes.c_double]
                lib.raft_remap_linear_f32.argtypes = [f, i, i, i, f, f, i, i]
                lib.raft_png_unfilter.argtypes = [f, i, i, i, f]
                lib.raft_png_unfilter.restype = ctypes.c_int
                _LIB = lib
            except OSError:
                _LIB = False
        else:
            _LIB = False
    return _LIB or None


def native_available():
    return _lib() is not None


def _ptr(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def _as_hwc_f32(img):
    a = np.asarray(img)
    squeeze = a.ndim == 2
    if squeeze:
        a = a[..., None]
    return np.ascontiguousarray(a, dtype=np.float32), squeeze, a.dtype


def _restore(out, squeeze, dtype):
    if squeeze:
        out = out[..., 0]
    if dtype == np.uint8:
        return np.clip(np.rint(out), 0, 255).astype(np.uint8)
    if dtype == np.uint16:
        return np.clip(np.rint(out), 0, 65535).astype(np.uint16)
    return out.astype(dtype, copy=False)


def _resize_numpy(a, oh, ow, inv_sx, inv_sy):
    h, w, _ = a.shape
    ys = (np.arange(oh) + 0.5) * inv_sy - 0.5
    xs = (np.arange(ow) + 0.5) * inv_sx - 0.5
    y0 = np.floor(ys).astype(np.int64)
    x0 = np.floor(xs).astype(np.int64)
    ay = (ys - y0).astype(np.float32)
    ax = (xs - x0).astype(np.float32)
    ay[y0 < 0] = 0
    ax[x0 < 0] = 0
    y1 = np.clip(y0 + 1, 0, h - 1)
    x1 = np.clip(x0 + 1, 0, w - 1)
    y0 = np.clip(y0, 0, h - 1)
    x0 = np.clip(x0, 0, w - 1)
    ay[y0 == y1] = 0
    ax[x0 == x1] = 0
    top = a[y0][:, x0] + ax[None, :, None] * (a[y0][:, x1] - a[y0][:, x0])
    bot = a[y1][:, x0] + ax[None, :, None] * (a[y1][:, x1] - a[y1][:, x0])
    return (top + ay[:, None, None] * (bot - top)).astype(np.float32)


def resize_linear(img, fx=None, fy=None, dsize=None):
    """Resize like ``cv2.resize(img, dsize or None, fx=fx, fy=fy, interpolation=INTER_LINEAR)``.

    ``dsize`` is (width, height) like OpenCV.  With fx/fy the output size is round(size * f) and the
    sampling step is 1/f (OpenCV behaviour).
    """
    a, squeeze, dtype = _as_hwc_f32(img)
    h, w, c = a.shape
    if dsize is not None:
        ow, oh = int(dsize[0]), int(dsize[1])
        inv_sx, inv_sy = w / ow, h / oh
    else:
        ow, oh = int(round(w * fx)), int(round(h * fy))
        inv_sx, inv_sy = 1.0 / fx, 1.0 / fy
    lib = _lib()
    if lib is not None:
        out = np.empty((oh, ow, c), np.float32)
        lib.raft_resize_linear_f32(_ptr(a), h, w, c, _ptr(out), oh, ow, inv_sx, inv_sy)
    else:
        out = _resize_numpy(a, oh, ow, inv_sx, inv_sy)
    return _restore(out, squeeze, dtype)


def remap_linear(img, map_xy):
    """dst(y, x) = bilinear(img, map_xy[y, x]) with zeros outside (cv2.remap INTER_LINEAR)."""
    a, squeeze, dtype = _as_hwc_f32(img)
    h, w, c = a.shape
    m = np.ascontiguousarray(map_xy, dtype=np.float32)
    oh, ow = m.shape[:2]
    lib = _lib()
    if lib is not None:
        out = np.empty((oh, ow, c), np.float32)
        lib.raft_remap_linear_f32(_ptr(a), h, w, c, _ptr(m), _ptr(out), oh, ow)
    else:
        import torch
        import torch.nn.functional as F
        t = torch.from_numpy(a).permute(2, 0, 1)[None]
        gx = torch.from_numpy(m[..., 0]) / max(w - 1, 1) * 2 - 1
        gy = torch.from_numpy(m[..., 1]) / max(h - 1, 1) * 2 - 1
        g = torch.stack([gx, gy], -1)[None]
        out = F.grid_sample(t, g, align_corners=True, padding_mode='zeros')[0].permute(1, 2, 0).numpy()
    return _restore(out, squeeze, dtype)


def rgb_to_bgr(img):
    return np.ascontiguousarray(np.asarray(img)[..., ::-1])


bgr_to_rgb = rgb_to_bgr
