"""File formats and the native host image ops (CPU)."""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F
from PIL import Image

from pytorch_raft_amd.utils import frame_utils, imgproc, png
from pytorch_raft_amd.utils.video import MJPEGWriter, frames_to_video


def test_flo_roundtrip(tmp_path):
    flow = np.random.RandomState(0).randn(7, 11, 2).astype(np.float32)
    p = str(tmp_path / 'a.flo')
    frame_utils.writeFlow(p, flow)
    raw = open(p, 'rb').read()
    assert np.frombuffer(raw[:4], np.float32)[0] == 202021.25
    assert np.frombuffer(raw[4:12], np.int32).tolist() == [11, 7]
    assert np.array_equal(frame_utils.readFlow(p), flow)
    assert np.array_equal(frame_utils.read_gen(p), flow)
    frame_utils.writeFlow(p, flow[..., 0], flow[..., 1])
    assert np.array_equal(frame_utils.readFlow(p), flow)


def test_pfm_roundtrip(tmp_path):
    rng = np.random.RandomState(1)
    img3 = rng.randn(5, 6, 3).astype(np.float32)
    p = str(tmp_path / 'a.pfm')
    frame_utils.writePFM(p, img3)
    assert np.array_equal(frame_utils.readPFM(p), img3)
    # read_gen drops the 3rd channel of a flow PFM
    assert np.array_equal(frame_utils.read_gen(p), img3[:, :, :2])
    img1 = rng.randn(4, 3).astype(np.float32)
    frame_utils.writePFM(p, img1)
    assert np.array_equal(frame_utils.readPFM(p), img1)


def test_kitti_png16_roundtrip(tmp_path):
    rng = np.random.RandomState(2)
    flow = np.round(rng.randn(9, 13, 2) * 40 * 64) / 64
    p = str(tmp_path / 'f.png')
    frame_utils.writeFlowKITTI(p, flow)
    got, valid = frame_utils.readFlowKITTI(p)
    assert np.allclose(got, flow, atol=1 / 64)
    assert np.all(valid == 1)


@pytest.mark.parametrize('mode', ['RGB', 'L', 'RGBA'])
def test_png_codec_matches_pil_8bit(tmp_path, mode):
    rng = np.random.RandomState(3)
    ch = {'RGB': 3, 'L': 1, 'RGBA': 4}[mode]
    # smooth gradients make PIL pick Sub/Up/Paeth filters
    base = np.cumsum(rng.randint(0, 3, size=(33, 47, ch)), axis=1).astype(np.uint8)
    arr = base[..., 0] if ch == 1 else base
    p = str(tmp_path / 'x.png')
    Image.fromarray(arr, mode).save(p, optimize=True)
    assert np.array_equal(png.read_png(p), np.array(Image.open(p)))


def test_png_16bit_grey(tmp_path):
    arr = (np.arange(12 * 10).reshape(12, 10) * 517).astype(np.uint16)
    p = str(tmp_path / 'g.png')
    png.write_png(p, arr)
    assert np.array_equal(png.read_png(p), arr)


def test_native_lib_loaded():
    assert imgproc.native_available(), 'csrc/cpu/imgproc.cpp not built (python -m pytorch_raft_amd.build)'


@pytest.mark.parametrize('shape,dsize', [((20, 30, 3), (45, 40)), ((50, 64, 2), (31, 17))])
def test_resize_matches_torch_bilinear(shape, dsize):
    rng = np.random.RandomState(4)
    img = rng.rand(*shape).astype(np.float32)
    out = imgproc.resize_linear(img, dsize=dsize)
    t = torch.from_numpy(img).permute(2, 0, 1)[None]
    ref = F.interpolate(t, size=(dsize[1], dsize[0]), mode='bilinear', align_corners=False)
    ref = ref[0].permute(1, 2, 0).numpy()
    assert out.shape == ref.shape
    assert np.allclose(out, ref, atol=1e-5)


def test_resize_fx_uint8():
    img = (np.random.RandomState(5).rand(16, 16, 3) * 255).astype(np.uint8)
    out = imgproc.resize_linear(img, fx=1.5, fy=0.75)
    assert out.shape == (12, 24, 3) and out.dtype == np.uint8


def test_remap_matches_grid_sample():
    rng = np.random.RandomState(6)
    img = rng.rand(10, 12, 3).astype(np.float32)
    ys, xs = np.mgrid[0:10, 0:12]
    m = np.dstack([xs, ys]).astype(np.float32) + rng.randn(10, 12, 2).astype(np.float32) * 2
    out = imgproc.remap_linear(img, m)
    t = torch.from_numpy(img).permute(2, 0, 1)[None]
    g = torch.from_numpy(m)
    gx = g[..., 0] / 11 * 2 - 1
    gy = g[..., 1] / 9 * 2 - 1
    ref = F.grid_sample(t, torch.stack([gx, gy], -1)[None], align_corners=True)[0].permute(1, 2, 0).numpy()
    assert np.allclose(out, ref, atol=1e-5)


def test_mjpeg_avi_writer(tmp_path):
    p = str(tmp_path / 'v.avi')
    wr = MJPEGWriter(p, 10, (32, 24))
    for k in range(3):
        wr.write(np.full((24, 32, 3), k * 60, np.uint8))
    wr.release()
    data = open(p, 'rb').read()
    assert data[:4] == b'RIFF' and data[8:12] == b'AVI ' and data.count(b'00dc') >= 6
    out = frames_to_video([np.zeros((8, 8, 3), np.uint8)] * 2, str(tmp_path / 'v.mp4'), 5, (8, 8))
    assert out.endswith('.avi') and os.path.exists(out)


def test_reference_demo_frame_decodes():
    path = '/root/reference/demo-Game/frame_0016.png'
    if not os.path.exists(path):
        pytest.skip('reference demo frames not mounted')
    assert np.array_equal(png.read_png(path)[..., :3], np.array(Image.open(path).convert('RGB')))
