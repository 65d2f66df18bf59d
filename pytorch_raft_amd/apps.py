"""Shared helpers for the CLI applications (demo / warping demos / evaluate / frame2video).

Reference behaviours kept (`demo.py`, `demo_warp*.py`, `frame2video.py`):

* models are loaded through the ``module.``-prefixed checkpoint with a strict load (`demo.py:43-44`);
* ``load_image`` -> float (1,3,H,W) 0..255 on the device; ``load_image_mult8`` resizes to a multiple of
  8 like the folder demos (`demo_warp_folder_firstframe.py:46-53`);
* ``warp(x, flo)`` = backward warp output(p) = x(p + flo(p)).  The reference normalises with
  (W-1)/(H-1) (align_corners=True convention) but samples with grid_sample's default
  align_corners=False (`demo_warp.py:45-49`); that exact behaviour is the default here
  (``convention='reference'``), ``convention='exact'`` gives the geometrically consistent warp.
  On GPU both run the HIP bilinear sampler (csrc/kernels/sampler.hip).
* ``warp_cv2`` = cv2.remap(INTER_LINEAR) replacement on the host (native C++).
"""
import glob
import os

import numpy as np
import torch
from PIL import Image

from .models.raft import RAFT
from .engine import checkpoint as ckpt
from .ops.sampler import warp_image
from .utils import imgproc


def default_device():
    return 'cuda' if torch.cuda.is_available() else 'cpu'


def create_raft(args, device=None):
    device = device or default_device()
    model = RAFT(args)
    if getattr(args, 'model', None):
        ckpt.load_weights(model, args.model, strict=True)
    model.to(device).eval()
    return model


def load_image(imfile, device=None):
    img = np.array(Image.open(imfile).convert('RGB')).astype(np.uint8)
    t = torch.from_numpy(img).permute(2, 0, 1).float()
    return t[None].to(device or default_device())


def load_image_mult8(imfile, device=None):
    img = np.array(Image.open(imfile).convert('RGB')).astype(np.uint8)
    h, w = img.shape[:2]
    img = imgproc.resize_linear(img, dsize=(w // 8 * 8, h // 8 * 8))
    t = torch.from_numpy(img).permute(2, 0, 1).float()
    return t[None].to(device or default_device())


def list_frames(path, sort=True):
    exts = ('*.png', '*.jpg', '*.jpeg', '*.ppm', '*.bmp', '*.JPEG')
    files = []
    for root, _, _ in os.walk(path):
        for e in exts:
            files += glob.glob(os.path.join(root, e))
    return sorted(files) if sort else files


def warp(x, flo, convention='reference'):
    return warp_image(x, flo, convention=convention)


def warp_cv2(x, flo):
    h, w = x.shape[:2]
    ys, xs = np.mgrid[0:h, 0:w]
    pixel_map = np.dstack([xs, ys]).astype(np.float32) + np.asarray(flo, np.float32)
    return imgproc.remap_linear(x, pixel_map)


def save_rgb(path, img):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    Image.fromarray(np.clip(np.asarray(img), 0, 255).astype(np.uint8)).save(path)


def warp_name(path):
    """a/b/frame.png -> a/b/frame_warp.png (the reference's str.replace('.', '_warp.') also rewrote
    dots in directory names)."""
    root, ext = os.path.splitext(path)
    return root + '_warp' + ext


@torch.no_grad()
def flow_pair(model, image1, image2, iters=20, pad=True):
    """Full-resolution flow image1 -> image2 (test mode), returned with the padded inputs."""
    from .utils.utils import InputPadder
    if pad:
        padder = InputPadder(image1.shape)
        image1, image2 = padder.pad(image1, image2)
    _, flow_up = model(image1, image2, iters=iters, test_mode=True)
    return image1, image2, flow_up


@torch.no_grad()
def warp_pair(model, imfile1, imfile2, use_cv2=False, iters=20, mult8=False):
    """Warp frame 1 by flow(1 -> 2) like `demo_warp_folder.py:94-137`; returns uint8 HxWx3 RGB at the
    input resolution (the padded result is resized back, as the reference does)."""
    loader = load_image_mult8 if mult8 else load_image
    image1 = loader(imfile1)
    image2 = loader(imfile2)
    assert image1.shape == image2.shape
    h, w = image1.shape[-2:]
    image1, image2, flow_up = flow_pair(model, image1, image2, iters=iters, pad=not mult8)
    if use_cv2:
        img = image1[0].permute(1, 2, 0).cpu().numpy()
        fl = flow_up[0].permute(1, 2, 0).cpu().numpy()
        out = warp_cv2(img, fl)
    else:
        out = warp(image1, flow_up)[0].permute(1, 2, 0).cpu().numpy()
    out = out.astype(np.uint8)
    if out.shape[:2] != (h, w):
        out = imgproc.resize_linear(out, dsize=(w, h))
    return out


def show_or_save(img, save_path=None):
    """matplotlib window like the reference, or a file when headless / --save given."""
    if save_path:
        save_rgb(save_path, img)
        return save_path
    import matplotlib
    if os.environ.get('DISPLAY') is None:
        matplotlib.use('Agg')
    import matplotlib.pyplot as plt
    plt.imshow(np.asarray(img) / 255.0)
    plt.show()
    return None
