"""Minimal PNG codec with full 16-bit support (KITTI flow / disparity maps).

PIL cannot round-trip 16-bit RGB PNGs and OpenCV is not part of this stack, so KITTI's
``flow_occ/*.png`` (uint16 RGB: u, v, valid) are decoded here: chunks are parsed in Python, IDAT is
inflated with zlib, scanlines are un-filtered by the native ``raft_png_unfilter`` (csrc/cpu/imgproc.cpp;
numpy fallback), and big-endian samples are converted.  Non-interlaced greyscale / grey+alpha / RGB /
RGBA at 8 or 16 bits are supported -- everything the datasets use.  ``write_png`` writes
unfiltered rows (filter type 0), which every decoder reads.
"""
import struct
import zlib

import numpy as np

from .imgproc import _lib, _ptr

_SIG = b'\x89PNG\r\n\x1a\n'
_CHANNELS = {0: 1, 2: 3, 4: 2, 6: 4}


def _unfilter_numpy(raw, rows, stride, bpp):
    out = np.zeros((rows, stride), np.uint8)
    raw = raw.reshape(rows, stride + 1)
    prev = np.zeros(stride, np.int32)
    for y in range(rows):
        ft = raw[y, 0]
        line = raw[y, 1:].astype(np.int32)
        cur = np.zeros(stride, np.int32)
        if ft == 0:
            cur = line
        elif ft == 2:
            cur = (line + prev) & 0xFF
        else:
            for i in range(stride):
                a = cur[i - bpp] if i >= bpp else 0
                b = prev[i]
                c = prev[i - bpp] if i >= bpp else 0
                if ft == 1:
                    p = a
                elif ft == 3:
                    p = (a + b) >> 1
                elif ft == 4:
                    pp = a + b - c
                    pa, pb, pc = abs(pp - a), abs(pp - b), abs(pp - c)
                    p = a if (pa <= pb and pa <= pc) else (b if pb <= pc else c)
                else:
                    raise ValueError('bad PNG filter %d' % ft)
                cur[i] = (line[i] + p) & 0xFF
        out[y] = cur
        prev = cur
    return out


def read_png(path):
    """Return an (H, W[, C]) uint8 / uint16 array in file channel order (RGB[A])."""
    with open(path, 'rb') as f:
        data = f.read()
    if data[:8] != _SIG:
        raise ValueError('%s is not a PNG file' % path)
    pos = 8
    idat = []
    hdr = None
    while pos < len(data):
        n, kind = struct.unpack('>I4s', data[pos:pos + 8])
        body = data[pos + 8:pos + 8 + n]
        pos += 12 + n
        if kind == b'IHDR':
            hdr = struct.unpack('>IIBBBBB', body)
        elif kind == b'IDAT':
            idat.append(body)
        elif kind == b'IEND':
            break
    w, h, depth, ctype, _, _, interlace = hdr
    if interlace != 0 or ctype not in _CHANNELS or depth not in (8, 16):
        raise ValueError('unsupported PNG layout (depth %d, colour type %d, interlace %d)'
                         % (depth, ctype, interlace))
    ch = _CHANNELS[ctype]
    bpp = ch * depth // 8
    stride = w * bpp
    raw = np.frombuffer(zlib.decompress(b''.join(idat)), np.uint8)
    lib = _lib()
    if lib is not None:
        raw_c = np.ascontiguousarray(raw)
        out = np.empty((h, stride), np.uint8)
        if lib.raft_png_unfilter(_ptr(raw_c), h, stride, bpp, _ptr(out)) != 0:
            raise ValueError('corrupt PNG filter stream in %s' % path)
    else:
        out = _unfilter_numpy(raw, h, stride, bpp)
    if depth == 16:
        img = out.view('>u2').astype(np.uint16).reshape(h, w, ch)
    else:
        img = out.reshape(h, w, ch)
    return img[..., 0] if ch == 1 else img


def _chunk(kind, body):
    return struct.pack('>I', len(body)) + kind + body + struct.pack('>I', zlib.crc32(kind + body) & 0xFFFFFFFF)


def write_png(path, img):
    a = np.asarray(img)
    if a.dtype not in (np.uint8, np.uint16):
        raise ValueError('write_png expects uint8 or uint16')
    if a.ndim == 2:
        a = a[..., None]
    h, w, ch = a.shape
    ctype = {1: 0, 2: 4, 3: 2, 4: 6}[ch]
    depth = 16 if a.dtype == np.uint16 else 8
    rows = a.astype('>u2' if depth == 16 else np.uint8).reshape(h, -1).view(np.uint8)
    raw = np.concatenate([np.zeros((h, 1), np.uint8), rows], axis=1)
    body = zlib.compress(raw.tobytes(), 6)
    ihdr = struct.pack('>IIBBBBB', w, h, depth, ctype, 0, 0, 0)
    with open(path, 'wb') as f:
        f.write(_SIG + _chunk(b'IHDR', ihdr) + _chunk(b'IDAT', body) + _chunk(b'IEND', b''))
