#!/usr/bin/env python
"""Chain-warp the first frame of a folder (reference `demo_warp_folder_firstframe.py`).

Frames are resized to a multiple of 8, flows of all consecutive pairs are computed, then the first
frame is repeatedly warped by -flow_i (`:144-167`) and every intermediate result is written to
``result4/<i+1>.png`` (``--torch_warp`` uses the GPU sampler and ``result/`` like ``warp_folder``).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_raft_amd import apps  # noqa: E402
from pytorch_raft_amd.utils import imgproc  # noqa: E402


@torch.no_grad()
def compute_flows(model, frames, iters=20):
    flows = []
    for prev, nxt in zip(frames[:-1], frames[1:]):
        print(prev, nxt)
        i1 = apps.load_image_mult8(prev)
        i2 = apps.load_image_mult8(nxt)
        _, _, flow_up = apps.flow_pair(model, i1, i2, iters=iters, pad=False)
        flows.append(flow_up)
    return flows


@torch.no_grad()
def warp_folder(source_path, flow_list, savepath='result'):
    os.makedirs(savepath, exist_ok=True)
    source = apps.load_image_mult8(source_path)
    h, w = source.shape[-2:]
    for i, flow_up in enumerate(flow_list):
        source = apps.warp(source, -flow_up)
        img = source[0].permute(1, 2, 0).cpu().numpy().astype(np.uint8)
        apps.save_rgb(os.path.join(savepath, '%d.png' % (i + 1)), imgproc.resize_linear(img, dsize=(w, h)))


@torch.no_grad()
def warp_folder_cv2(source_path, flow_list, savepath='result4'):
    os.makedirs(savepath, exist_ok=True)
    source = apps.load_image_mult8(source_path)
    h, w = source.shape[-2:]
    source = source[0].permute(1, 2, 0).cpu().numpy()
    for i, flow_up in enumerate(flow_list):
        fl = flow_up[0].permute(1, 2, 0).cpu().numpy()
        source = apps.warp_cv2(source, -fl)
        img = source.astype(np.uint8)
        apps.save_rgb(os.path.join(savepath, '%d.png' % (i + 1)), imgproc.resize_linear(img, dsize=(w, h)))


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--folderlist', default='demo-Cat', help='folder of frames')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--torch_warp', action='store_true')
    parser.add_argument('--out_dir', default=None)
    args = parser.parse_args()
    frames = apps.list_frames(args.folderlist)
    model = apps.create_raft(args)
    flows = compute_flows(model, frames)
    if args.torch_warp:
        warp_folder(frames[0], flows, args.out_dir or 'result')
    else:
        warp_folder_cv2(frames[0], flows, args.out_dir or 'result4')
