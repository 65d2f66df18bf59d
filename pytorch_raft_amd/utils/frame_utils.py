"""Flow / image file IO (reference `core/utils/frame_utils.py`).

* ``.flo``  Middlebury: float32 magic 202021.25, int32 width, int32 height, interleaved (u, v).
* ``.pfm``  'PF' (3 ch) / 'Pf' (1 ch); negative scale = little endian; rows stored bottom-up.
* KITTI flow PNG: uint16 (u, v, valid) with flow = (value - 2^15) / 64.
* KITTI disparity PNG: uint16 / 256, flow = (-disp, 0).
* ``read_gen`` dispatches on the extension like the reference (`:123-137`).

16-bit PNGs go through our own codec (utils/png.py) instead of cv2.
"""
import os
import re

import numpy as np
from PIL import Image

from .png import read_png, write_png

TAG_FLOAT = 202021.25
TAG_CHAR = np.array([TAG_FLOAT], np.float32)


def readFlow(fn):
    with open(fn, 'rb') as f:
        magic = np.fromfile(f, np.float32, count=1)
        if magic.size != 1 or magic[0] != TAG_FLOAT:
            print('Magic number incorrect. Invalid .flo file')
            return None
        w = int(np.fromfile(f, np.int32, count=1)[0])
        h = int(np.fromfile(f, np.int32, count=1)[0])
        data = np.fromfile(f, np.float32, count=2 * w * h)
    return np.resize(data, (h, w, 2))


def writeFlow(filename, uv, v=None):
    if v is None:
        uv = np.asarray(uv)
        assert uv.ndim == 3 and uv.shape[2] == 2
        u, v = uv[:, :, 0], uv[:, :, 1]
    else:
        u = np.asarray(uv)
    assert u.shape == v.shape
    h, w = u.shape
    inter = np.empty((h, w, 2), np.float32)
    inter[..., 0] = u
    inter[..., 1] = v
    with open(filename, 'wb') as f:
        TAG_CHAR.tofile(f)
        np.array(w, np.int32).tofile(f)
        np.array(h, np.int32).tofile(f)
        inter.tofile(f)


def readPFM(file):
    with open(file, 'rb') as f:
        header = f.readline().rstrip()
        if header == b'PF':
            color = True
        elif header == b'Pf':
            color = False
        else:
            raise Exception('Not a PFM file.')
        m = re.match(rb'^(\d+)\s(\d+)\s$', f.readline())
        if not m:
            raise Exception('Malformed PFM header.')
        width, height = map(int, m.groups())
        scale = float(f.readline().rstrip())
        endian = '<' if scale < 0 else '>'
        data = np.fromfile(f, endian + 'f')
    shape = (height, width, 3) if color else (height, width)
    return np.flipud(np.reshape(data, shape))


def writePFM(file, image, scale=1.0):
    image = np.asarray(image, dtype=np.float32)
    color = image.ndim == 3 and image.shape[2] == 3
    if not (color or image.ndim == 2 or (image.ndim == 3 and image.shape[2] == 1)):
        raise ValueError('PFM needs H x W x 3 or H x W')
    with open(file, 'wb') as f:
        f.write(b'PF\n' if color else b'Pf\n')
        f.write(b'%d %d\n' % (image.shape[1], image.shape[0]))
        f.write(b'%f\n' % (-abs(scale)))  # little endian
        np.flipud(image).astype('<f4').tofile(f)


def readFlowKITTI(filename):
    raw = read_png(filename).astype(np.float32)  # RGB order as stored (u, v, valid)
    flow, valid = raw[:, :, :2], raw[:, :, 2]
    flow = (flow - 2 ** 15) / 64.0
    return flow, valid


def readDispKITTI(filename):
    disp = read_png(filename).astype(np.float32) / 256.0
    if disp.ndim == 3:
        disp = disp[..., 0]
    valid = disp > 0.0
    flow = np.stack([-disp, np.zeros_like(disp)], -1)
    return flow, valid


def writeFlowKITTI(filename, uv):
    uv = 64.0 * np.asarray(uv) + 2 ** 15
    valid = np.ones([uv.shape[0], uv.shape[1], 1])
    out = np.concatenate([uv, valid], axis=-1).astype(np.uint16)
    write_png(filename, out)


def read_gen(file_name, pil=False):
    ext = os.path.splitext(file_name)[-1]
    if ext in ('.png', '.jpeg', '.ppm', '.jpg'):
        return Image.open(file_name)
    if ext in ('.bin', '.raw'):
        return np.load(file_name)
    if ext == '.flo':
        return readFlow(file_name).astype(np.float32)
    if ext == '.pfm':
        flow = readPFM(file_name).astype(np.float32)
        return flow if flow.ndim == 2 else flow[:, :, :-1]
    return []
