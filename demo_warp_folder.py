#!/usr/bin/env python
"""Folder warping demo (reference `demo_warp_folder.py`): for every consecutive pair (i, i+1) of a
folder, warp frame i by flow(i -> i+1) and save it next to frame i+1 as ``<name>_warp.<ext>``.

Frames are processed in sorted order (the reference discards the result of ``sorted()``, `:152`).
``--out_dir`` writes results elsewhere instead of next to the inputs.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_raft_amd import apps  # noqa: E402

get_files = apps.list_frames


def run(args):
    frames = get_files(args.folderlist)
    model = apps.create_raft(args)
    outs = []
    for prev, nxt in zip(frames[:-1], frames[1:]):
        print(prev, nxt)
        out = apps.warp_pair(model, prev, nxt, use_cv2=not args.torch_warp)
        dst = apps.warp_name(nxt)
        if args.out_dir:
            dst = os.path.join(args.out_dir, os.path.basename(dst))
        apps.save_rgb(dst, out)
        outs.append(dst)
    return outs


if __name__ == '__main__':
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', default='models/raft-things.pth', help='restore checkpoint')
    parser.add_argument('--folderlist', default='demo-Cat', help='folder of frames')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--torch_warp', action='store_true', help='GPU sampler instead of the remap path')
    parser.add_argument('--out_dir', default=None)
    run(parser.parse_args())
