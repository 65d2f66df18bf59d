#!/usr/bin/env python
"""Flow visualisation demo (reference `demo.py`): consecutive frame pairs of a folder -> RAFT
(iters=20, test mode) -> image stacked over its flow colour coding.

    python demo.py --model=models/raft-things.pth --path=demo-Game [--save_dir out/]

``--path`` defaults to demo-frames like the reference and falls back to demo-Game when that folder
does not exist.  Without a display (or with ``--save_dir``) the visualisations are written as PNGs.
"""
import argparse
import glob
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_raft_amd import apps  # noqa: E402
from pytorch_raft_amd.utils import flow_viz  # noqa: E402
from pytorch_raft_amd.utils.utils import InputPadder  # noqa: E402


def viz(img, flo, save_path=None):
    img = img[0].permute(1, 2, 0).cpu().numpy()
    flo = flo[0].permute(1, 2, 0).cpu().numpy()
    flo = flow_viz.flow_to_image(flo)
    img_flo = np.concatenate([img, flo], axis=0)
    return apps.show_or_save(img_flo, save_path)


def demo(args):
    model = apps.create_raft(args)
    path = args.path if os.path.isdir(args.path) else 'demo-Game'
    images = sorted(glob.glob(os.path.join(path, '*.png')) + glob.glob(os.path.join(path, '*.jpg')))
    with torch.no_grad():
        for k, (imfile1, imfile2) in enumerate(zip(images[:-1], images[1:])):
            image1 = apps.load_image(imfile1)
            image2 = apps.load_image(imfile2)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            flow_low, flow_up = model(image1, image2, iters=args.iters, test_mode=True)
            save = os.path.join(args.save_dir, 'flow_%04d.png' % k) if args.save_dir else None
            viz(image1, flow_up, save)


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--path', default='demo-frames', help='dataset for evaluation')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--iters', type=int, default=20)
    parser.add_argument('--save_dir', default=None, help='write visualisations here instead of showing')
    demo(parser.parse_args())
