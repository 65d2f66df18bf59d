#!/usr/bin/env python
"""Warp an explicit list of (frame1, frame2) pairs (reference `demo_warp_imglist.py`); each warped
frame 1 is saved as ``<frame2>_warp.<ext>``.  (The reference ``demo()`` crashes on a NameError,
`:98-102`; both paths work here.)
"""
import argparse
import ast
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_raft_amd import apps  # noqa: E402

DEFAULT_PAIRS = [['demo-Game/frame_0016.png', 'demo-Game/frame_0017.png'],
                 ['demo-Game/frame_0018.png', 'demo-Game/frame_0019.png']]


def demo(model, imfile1, imfile2, use_cv2=False, out_dir=None):
    out = apps.warp_pair(model, imfile1, imfile2, use_cv2=use_cv2)
    dst = apps.warp_name(imfile2)
    if out_dir:
        dst = os.path.join(out_dir, os.path.basename(dst))
    apps.save_rgb(dst, out)
    return dst


def demo_cv2(model, imfile1, imfile2, out_dir=None):
    return demo(model, imfile1, imfile2, use_cv2=True, out_dir=out_dir)


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--pathlist', default=DEFAULT_PAIRS, type=ast.literal_eval,
                        help='python list of [frame1, frame2] pairs')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--out_dir', default=None)
    args = parser.parse_args()
    model = apps.create_raft(args)
    for a, b in args.pathlist:
        print(a, b)
        demo_cv2(model, a, b, args.out_dir)
