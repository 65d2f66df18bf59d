"""Frames -> video without OpenCV (reference `frame2video.py` uses cv2.VideoWriter).

``MJPEGWriter`` writes a standard RIFF/AVI container with Motion-JPEG frames (encoded by PIL) and an
idx1 index -- playable by common players.  ``.gif`` output uses PIL's animated GIF encoder.  Codecs
that need an external encoder (.mp4 H.264, .ogv Theora, .flv) are written as MJPEG-AVI next to the
requested name (``<name>.avi``) with a notice, since no such encoder is available in this stack.
"""
import io
import os
import struct

from PIL import Image


def _chunk(fourcc, data):
    pad = b'\x00' if len(data) % 2 else b''
    return fourcc + struct.pack('<I', len(data)) + data + pad


def _list(kind, payload):
    return b'LIST' + struct.pack('<I', len(payload) + 4) + kind + payload


class MJPEGWriter:
    def __init__(self, path, fps, size, quality=90):
        self.path = path
        self.fps = int(round(fps))
        self.size = (int(size[0]), int(size[1]))
        self.quality = quality
        self.frames = []

    def write(self, img):
        """img: PIL image or HxWx3 uint8 RGB array."""
        if not isinstance(img, Image.Image):
            img = Image.fromarray(img)
        if img.size != self.size:
            img = img.resize(self.size, Image.BILINEAR)
        buf = io.BytesIO()
        img.convert('RGB').save(buf, format='JPEG', quality=self.quality)
        self.frames.append(buf.getvalue())

    def release(self):
        w, h = self.size
        n = len(self.frames)
        usec = int(1e6 / max(self.fps, 1))
        maxbytes = max((len(f) for f in self.frames), default=0)
        avih = struct.pack('<IIIIIIIIIIIIII', usec, maxbytes * self.fps, 0, 0x10, n, 0, 1,
                           maxbytes, w, h, 0, 0, 0, 0)
        strh = struct.pack('<4s4sIHHIIIIIIIIhhhh', b'vids', b'MJPG', 0, 0, 0, 0, 1, self.fps, 0, n,
                           maxbytes, 0xFFFFFFFF, 0, 0, 0, w, h)
        strf = struct.pack('<IiiHH4sIiiII', 40, w, h, 1, 24, b'MJPG', w * h * 3, 0, 0, 0, 0)
        hdrl = _list(b'hdrl', _chunk(b'avih', avih) + _list(b'strl', _chunk(b'strh', strh) + _chunk(b'strf', strf)))
        movi_payload = b''
        index = b''
        offset = 4
        for f in self.frames:
            c = _chunk(b'00dc', f)
            index += struct.pack('<4sIII', b'00dc', 0x10, offset, len(f))
            movi_payload += c
            offset += len(c)
        movi = _list(b'movi', movi_payload)
        body = b'AVI ' + hdrl + movi + _chunk(b'idx1', index)
        with open(self.path, 'wb') as fh:
            fh.write(b'RIFF' + struct.pack('<I', len(body)) + body)


def frames_to_video(frames, savepath, fps=24, size=(854, 480)):
    """Write ``frames`` (paths or arrays) to ``savepath``; returns the path actually written."""
    ext = os.path.splitext(savepath)[1].lower()
    if ext == '.gif':
        imgs = [(Image.open(f) if isinstance(f, str) else Image.fromarray(f)).convert('RGB').resize(size)
                for f in frames]
        if imgs:
            imgs[0].save(savepath, save_all=True, append_images=imgs[1:],
                         duration=int(1000 / max(fps, 1)), loop=0)
        return savepath
    if ext != '.avi':
        print('note: no %s encoder in this stack; writing MJPEG AVI instead' % ext)
        savepath = os.path.splitext(savepath)[0] + '.avi'
    wr = MJPEGWriter(savepath, fps, size)
    for f in frames:
        wr.write(Image.open(f) if isinstance(f, str) else f)
    wr.release()
    return savepath
