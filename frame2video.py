#!/usr/bin/env python
"""Frames of a folder -> video (reference `frame2video.py`).

    python frame2video.py --readpath ./demo-imgs --savepath ./result.avi --fps 30 --size 960 540

Writes MJPEG-AVI (or animated GIF) through ``pytorch_raft_amd.utils.video`` (no OpenCV); frames are
collected recursively and processed in sorted order.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from pytorch_raft_amd.utils.video import frames_to_video  # noqa: E402

image_format = ['.jpg', '.JPEG', '.png', '.bmp']


def get_files(path):
    ret = []
    for root, _, files in os.walk(path):
        for name in files:
            p = os.path.join(root, name)
            if os.path.splitext(p)[1] in image_format:
                ret.append(p)
    return sorted(ret)


def frame2video(readpath, savepath, fps=24, size=(854, 480)):
    return frames_to_video(get_files(readpath), savepath, fps=fps, size=size)


if __name__ == '__main__':
    ap = argparse.ArgumentParser()
    ap.add_argument('--readpath', default='./demo-imgs')
    ap.add_argument('--savepath', default='./result.avi')
    ap.add_argument('--fps', type=int, default=30)
    ap.add_argument('--size', type=int, nargs=2, default=[960, 540])
    a = ap.parse_args()
    print(frame2video(a.readpath, a.savepath, a.fps, tuple(a.size)))
