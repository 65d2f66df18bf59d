#!/usr/bin/env python
"""Warp consecutive frames listed in a FlyingThings3D split file (reference
`demo_warp_imglist_FlyingThings3D.py`): each line of ``--txt_path`` holds 9-10 frame names; every
consecutive pair (f_j, f_j+1) read from ``--read_path`` is warped and written to ``--save_path`` as
``<f_j>_warp.<ext>``.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_raft_amd import apps  # noqa: E402


def text_readlines(filename):
    try:
        with open(filename, 'r') as f:
            return [line.rstrip('\n') for line in f]
    except IOError:
        return []


def build_pairs(lines):
    pairs = []
    for line in lines:
        names = [n for n in line.split(' ') if n]
        pairs += [[names[j], names[j + 1]] for j in range(len(names) - 1)]
    return pairs


def demo_cv2(args, model, imfile1, imfile2):
    out = apps.warp_pair(model, os.path.join(args.read_path, imfile1),
                         os.path.join(args.read_path, imfile2), use_cv2=True)
    dst = os.path.join(args.save_path, apps.warp_name(imfile1))
    apps.save_rgb(dst, out)
    return dst


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--txt_path', default='txt/FlyingThings3D_subset_train_split.txt')
    parser.add_argument('--read_path', default='datasets/FlyingThings3D_subset/train/image_clean/left')
    parser.add_argument('--save_path', default='datasets/FlyingThings3D_subset/train/image_clean/left_warp')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    args = parser.parse_args()
    pairs = build_pairs(text_readlines(args.txt_path))
    os.makedirs(args.save_path, exist_ok=True)
    model = apps.create_raft(args)
    for a, b in pairs:
        print(a, b)
        demo_cv2(args, model, a, b)
