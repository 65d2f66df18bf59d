#!/usr/bin/env python
"""Single-pair warping demo (reference `demo_warp.py`): flow(img1 -> img2), warp img1 by it and show
a 3 x 2 mosaic [img1 | img2 | mean] over [flow | warp | warp].

    python demo_warp.py --model=models/raft-things.pth --path1 a.png --path2 b.png [--save out.png]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_raft_amd import apps  # noqa: E402
from pytorch_raft_amd.utils import flow_viz  # noqa: E402
from pytorch_raft_amd.utils.utils import InputPadder  # noqa: E402

warp = apps.warp
warp_cv2 = apps.warp_cv2


def _mosaic(img1, img2, img2_warp, flo):
    flo = flow_viz.flow_to_image(flo)
    c1 = np.concatenate([img1, flo], axis=0)
    c2 = np.concatenate([img2, img2_warp], axis=0)
    c3 = np.concatenate([(img1 + img2) / 2, img2_warp], axis=0)
    return np.concatenate([c1, c2, c3], axis=1)


def viz_warp(img1, img2, flo, save=None):
    img2_warp = warp(img1, flo)
    t = lambda x: x[0].permute(1, 2, 0).cpu().numpy()  # noqa: E731
    apps.show_or_save(_mosaic(t(img1), t(img2), t(img2_warp), t(flo)), save)
    return img2_warp


def viz_warp_cv2(img1, img2, flo, save=None):
    t = lambda x: x[0].permute(1, 2, 0).cpu().numpy()  # noqa: E731
    img1, img2, flo = t(img1), t(img2), t(flo)
    img2_warp = warp_cv2(img1, flo)
    apps.show_or_save(_mosaic(img1, img2, img2_warp, flo), save)
    return img2_warp


def demo(args):
    model = apps.create_raft(args)
    with torch.no_grad():
        image1 = apps.load_image(args.path1)
        image2 = apps.load_image(args.path2)
        assert image1.shape == image2.shape
        padder = InputPadder(image1.shape)
        image1, image2 = padder.pad(image1, image2)
        flow_low, flow_up = model(image1, image2, iters=20, test_mode=True)
        return viz_warp(image1, image2, flow_up, args.save)


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--path1', default='demo-Game/frame_0016.png')
    parser.add_argument('--path2', default='demo-Game/frame_0017.png')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--save', default=None, help='write the mosaic here instead of showing it')
    demo(parser.parse_args())
