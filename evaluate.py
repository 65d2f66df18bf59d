#!/usr/bin/env python
"""Evaluation CLI (reference `evaluate.py:169-196`).

    python evaluate.py --model=models/raft-things.pth --dataset=sintel [--mixed_precision]

Additive flags: ``--submission {sintel,kitti}`` (leaderboard files), ``--warm_start``,
``--root`` (dataset root), ``--iters`` override.
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import torch  # noqa: E402

from pytorch_raft_amd import apps  # noqa: E402
from pytorch_raft_amd.engine.evaluate import (  # noqa: E402,F401
    validate_chairs, validate_sintel, validate_kitti, create_sintel_submission,
    create_kitti_submission)


def main():
    parser = argparse.ArgumentParser()
    parser.add_argument('--model', help='restore checkpoint')
    parser.add_argument('--dataset', help='dataset for evaluation')
    parser.add_argument('--small', action='store_true', help='use small model')
    parser.add_argument('--mixed_precision', action='store_true', help='use mixed precision')
    parser.add_argument('--alternate_corr', action='store_true', help='use efficent correlation implementation')
    parser.add_argument('--submission', choices=['sintel', 'kitti'], default=None)
    parser.add_argument('--warm_start', action='store_true')
    parser.add_argument('--root', default=None)
    parser.add_argument('--iters', type=int, default=None)
    args = parser.parse_args()

    model = apps.create_raft(args)
    kw = {}
    if args.root:
        kw['root'] = args.root
    if args.iters:
        kw['iters'] = args.iters
    with torch.no_grad():
        if args.submission == 'sintel':
            create_sintel_submission(model, warm_start=args.warm_start, **kw)
        elif args.submission == 'kitti':
            create_kitti_submission(model, **kw)
        elif args.dataset == 'chairs':
            validate_chairs(model, **kw)
        elif args.dataset == 'sintel':
            validate_sintel(model, **kw)
        elif args.dataset == 'kitti':
            validate_kitti(model, **kw)


if __name__ == '__main__':
    main()
