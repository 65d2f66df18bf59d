"""Validation and leaderboard submissions (reference `evaluate.py:21-166`).

Same metrics, iteration counts and output formats:

* ``validate_chairs``  24 iters, EPE over the 640-pair validation split.
* ``validate_sintel``  32 iters, clean + final, EPE / 1px / 3px / 5px, InputPadder('sintel').
* ``validate_kitti``   24 iters, EPE and F1-all (epe > 3 and epe / |gt| > 0.05) over valid pixels.
* ``create_sintel_submission`` (optional warm start by forward interpolation across a sequence) and
  ``create_kitti_submission`` write .flo / 16-bit PNG files.

MI355X path: metrics are accumulated on the device (one host sync per dataset instead of per image),
images go through pinned host memory, and all iterations except the last skip the convex upsample.
``device`` defaults to the model's device, so everything also runs on CPU.
"""
import os

import numpy as np
import torch

from ..data import datasets
from ..utils import frame_utils
from ..utils.utils import InputPadder, forward_interpolate


def _dev(model):
    return next(model.parameters()).device


@torch.no_grad()
def create_sintel_submission(model, iters=32, warm_start=False, output_path='sintel_submission',
                             root='datasets/Sintel'):
    model.eval()
    dev = _dev(model)
    for dstype in ['clean', 'final']:
        test_dataset = datasets.MpiSintel(split='test', aug_params=None, dstype=dstype, root=root)
        flow_prev, sequence_prev = None, None
        for test_id in range(len(test_dataset)):
            image1, image2, (sequence, frame) = test_dataset[test_id]
            if sequence != sequence_prev:
                flow_prev = None
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1[None].to(dev), image2[None].to(dev))
            flow_low, flow_pr = model(image1, image2, iters=iters, flow_init=flow_prev, test_mode=True)
            flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
            if warm_start:
                flow_prev = forward_interpolate(flow_low[0])[None].to(dev)
            out_dir = os.path.join(output_path, dstype, sequence)
            os.makedirs(out_dir, exist_ok=True)
            frame_utils.writeFlow(os.path.join(out_dir, 'frame%04d.flo' % (frame + 1)), flow)
            sequence_prev = sequence


@torch.no_grad()
def create_kitti_submission(model, iters=24, output_path='kitti_submission', root='datasets/KITTI'):
    model.eval()
    dev = _dev(model)
    test_dataset = datasets.KITTI(split='testing', aug_params=None, root=root)
    os.makedirs(output_path, exist_ok=True)
    for test_id in range(len(test_dataset)):
        image1, image2, (frame_id,) = test_dataset[test_id]
        padder = InputPadder(image1.shape, mode='kitti')
        image1, image2 = padder.pad(image1[None].to(dev), image2[None].to(dev))
        _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
        flow = padder.unpad(flow_pr[0]).permute(1, 2, 0).cpu().numpy()
        frame_utils.writeFlowKITTI(os.path.join(output_path, frame_id), flow)


@torch.no_grad()
def validate_chairs(model, iters=24, root='datasets/FlyingChairs_release/data'):
    model.eval()
    dev = _dev(model)
    val_dataset = datasets.FlyingChairs(split='validation', root=root)
    tot = torch.zeros((), dtype=torch.float64, device=dev)
    cnt = 0
    for val_id in range(len(val_dataset)):
        image1, image2, flow_gt, _ = val_dataset[val_id]
        _, flow_pr = model(image1[None].to(dev), image2[None].to(dev), iters=iters, test_mode=True)
        epe = torch.sum((flow_pr[0] - flow_gt.to(dev)) ** 2, dim=0).sqrt()
        tot += epe.double().sum()
        cnt += epe.numel()
    epe = float(tot.item() / max(cnt, 1))
    print('Validation Chairs EPE: %f' % epe)
    return {'chairs': epe}


@torch.no_grad()
def validate_sintel(model, iters=32, root='datasets/Sintel'):
    model.eval()
    dev = _dev(model)
    results = {}
    for dstype in ['clean', 'final']:
        val_dataset = datasets.MpiSintel(split='training', dstype=dstype, root=root)
        acc = torch.zeros(4, dtype=torch.float64, device=dev)
        per_image = []
        cnt = 0
        for val_id in range(len(val_dataset)):
            image1, image2, flow_gt, _ = val_dataset[val_id]
            image1, image2 = image1[None].to(dev), image2[None].to(dev)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
            flow = padder.unpad(flow_pr[0])
            epe = torch.sum((flow - flow_gt.to(dev)) ** 2, dim=0).sqrt().reshape(-1)
            acc += torch.stack([epe.sum(), (epe < 1).sum(), (epe < 3).sum(), (epe < 5).sum()]).double()
            per_image.append(epe.mean())
            cnt += epe.numel()
        a = (acc / max(cnt, 1)).cpu().tolist()
        print('Validation (%s) EPE: %f, 1px: %f, 3px: %f, 5px: %f' % (dstype, a[0], a[1], a[2], a[3]))
        # reference reports mean of per-image means for the returned value (`evaluate.py:126`)
        results[dstype] = float(torch.stack(per_image).mean().item()) if per_image else float('nan')
    return results


@torch.no_grad()
def validate_kitti(model, iters=24, root='datasets/KITTI'):
    model.eval()
    dev = _dev(model)
    val_dataset = datasets.KITTI(split='training', root=root)
    out_list, epe_list = [], []
    for val_id in range(len(val_dataset)):
        image1, image2, flow_gt, valid_gt = val_dataset[val_id]
        image1, image2 = image1[None].to(dev), image2[None].to(dev)
        padder = InputPadder(image1.shape, mode='kitti')
        image1, image2 = padder.pad(image1, image2)
        _, flow_pr = model(image1, image2, iters=iters, test_mode=True)
        flow = padder.unpad(flow_pr[0])
        flow_gt, valid_gt = flow_gt.to(dev), valid_gt.to(dev)
        epe = torch.sum((flow - flow_gt) ** 2, dim=0).sqrt()
        mag = torch.sum(flow_gt ** 2, dim=0).sqrt()
        epe, mag = epe.view(-1), mag.view(-1)
        val = valid_gt.view(-1) >= 0.5
        out = ((epe > 3.0) & ((epe / mag) > 0.05)).float()
        epe_list.append(epe[val].mean())
        out_list.append(out[val])
    if not epe_list:
        return {'kitti-epe': float('nan'), 'kitti-f1': float('nan')}
    epe = float(torch.stack(epe_list).mean().item())
    f1 = 100 * float(torch.cat(out_list).mean().item())
    print('Validation KITTI: %f, %f' % (epe, f1))
    return {'kitti-epe': epe, 'kitti-f1': f1}


VALIDATORS = {'chairs': validate_chairs, 'sintel': validate_sintel, 'kitti': validate_kitti}
