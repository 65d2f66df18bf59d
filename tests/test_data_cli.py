"""CPU integration tests on a generated fake dataset tree: every dataset class + augmentor, the
per-stage training mix, the validators and submissions, and the train / evaluate / demo CLIs.

The reference has no tests (`SURVEY.md` §4); its integration checks are `evaluate.py` on the real
datasets and the demos on the bundled frames.  Here the same code paths run end-to-end on tiny
synthetic files written in the reference's on-disk formats (`core/datasets.py:102-196`,
`core/utils/frame_utils.py`), with RAFT-small at 128x160 so the whole module stays fast on CPU.
(Below 128 px the coarsest correlation level is 1 pixel wide and the reference's align_corners
normalisation 2x/(W-1)-1 divides by zero -- `core/utils/utils.py:61-62` -- so the flow is NaN in
the reference as well; the fake frames stay above that size.)
"""
import argparse
import os
import subprocess
import sys

import numpy as np
import pytest
import torch
from PIL import Image

from pytorch_raft_amd.utils import frame_utils

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
H, W = 128, 160  # >= 128: RAFT's 4th pyramid level needs H/8, W/8 >= 16 (see below)


def _img(path, rng, fmt=None):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    Image.fromarray(rng.integers(0, 255, (H, W, 3), dtype=np.uint8)).save(path, format=fmt)


def _flow(rng):
    return (rng.standard_normal((H, W, 2)) * 3).astype(np.float32)


def _kitti_flow(path, rng):
    os.makedirs(os.path.dirname(path), exist_ok=True)
    frame_utils.writeFlowKITTI(path, _flow(rng))


@pytest.fixture(scope='module')
def tree(tmp_path_factory):
    """datasets/{FlyingChairs_release, FlyingThings3D, Sintel, KITTI, HD1k} + chairs_split.txt."""
    base = tmp_path_factory.mktemp('fake')
    rng = np.random.default_rng(0)
    d = base / 'datasets'
    # FlyingChairs: 4 pairs, split 1 1 2 2 (train, train, val, val)
    ch = d / 'FlyingChairs_release' / 'data'
    for i in range(4):
        _img(str(ch / ('%05d_img1.ppm' % i)), rng, 'PPM')
        _img(str(ch / ('%05d_img2.ppm' % i)), rng, 'PPM')
        frame_utils.writeFlow(str(ch / ('%05d_flow.flo' % i)), _flow(rng))
    (base / 'chairs_split.txt').write_text('1\n1\n2\n2\n')
    # FlyingThings3D: one sequence of 3 frames, both passes, both directions
    for dst in ('frames_cleanpass', 'frames_finalpass'):
        for k in range(3):
            _img(str(d / 'FlyingThings3D' / dst / 'TRAIN' / 'A' / '0000' / 'left' / ('%04d.png' % k)), rng)
    for dirn in ('into_future', 'into_past'):
        fd = d / 'FlyingThings3D' / 'optical_flow' / 'TRAIN' / 'A' / '0000' / dirn / 'left'
        os.makedirs(fd, exist_ok=True)
        for k in range(3):
            frame_utils.writePFM(str(fd / ('OpticalFlow_%04d_L.pfm' % k)),
                                 np.concatenate([_flow(rng), np.zeros((H, W, 1), np.float32)], -1))
    # Sintel: training (clean / final + flow) and test, one scene of 3 frames
    for split in ('training', 'test'):
        for dst in ('clean', 'final'):
            for k in range(3):
                _img(str(d / 'Sintel' / split / dst / 'alley' / ('frame_%04d.png' % (k + 1))), rng)
    fl = d / 'Sintel' / 'training' / 'flow' / 'alley'
    os.makedirs(fl, exist_ok=True)
    for k in range(2):
        frame_utils.writeFlow(str(fl / ('frame_%04d.flo' % (k + 1))), _flow(rng))
    # KITTI: 2 training pairs with sparse flow, 1 testing pair
    for i in range(2):
        for s in ('10', '11'):
            _img(str(d / 'KITTI' / 'training' / 'image_2' / ('%06d_%s.png' % (i, s))), rng)
        _kitti_flow(str(d / 'KITTI' / 'training' / 'flow_occ' / ('%06d_10.png' % i)), rng)
    for s in ('10', '11'):
        _img(str(d / 'KITTI' / 'testing' / 'image_2' / ('000000_%s.png' % s)), rng)
    # HD1K: one sequence of 3 frames
    for k in range(3):
        _img(str(d / 'HD1k' / 'hd1k_input' / 'image_2' / ('000000_%04d.png' % k)), rng)
        _kitti_flow(str(d / 'HD1k' / 'hd1k_flow_gt' / 'flow_occ' / ('000000_%04d.png' % k)), rng)
    return base


@pytest.fixture
def in_tree(tree, monkeypatch):
    monkeypatch.chdir(tree)
    return tree


def _check_sample(s, crop, sparse=False):
    img1, img2, flow, valid = s
    assert img1.shape == (3, *crop) and img2.shape == (3, *crop) and flow.shape == (2, *crop)
    assert valid.shape == tuple(crop)
    assert img1.dtype == torch.float32 and 0 <= float(img1.min()) and float(img1.max()) <= 255
    assert torch.isfinite(flow).all()
    assert set(torch.unique(valid).tolist()) <= {0.0, 1.0}


def test_dataset_classes_with_augmentation(in_tree):
    from pytorch_raft_amd.data import datasets as D
    crop = (96, 128)
    dense = dict(crop_size=crop, min_scale=-0.1, max_scale=0.3, do_flip=True)
    sparse = dict(crop_size=crop, min_scale=-0.1, max_scale=0.2, do_flip=True)
    cases = [(D.FlyingChairs(dense, split='training'), 2), (D.FlyingChairs(None, split='validation'), 2),
             (D.FlyingThings3D(dense), 4), (D.MpiSintel(dense, dstype='final'), 2),
             (D.KITTI(sparse), 2), (D.HD1K(sparse), 2)]
    for ds, n in cases:
        assert len(ds) == n, (type(ds).__name__, len(ds))
        s = ds[0]
        if ds.augmentor is None:
            assert s[0].shape == (3, H, W)
        else:
            _check_sample(s, crop)
    # test splits return (img1, img2, extra_info)
    t = D.MpiSintel(None, split='test', dstype='clean')
    i1, i2, info = t[1]
    assert i1.shape == (3, H, W) and info == ('alley', 1)
    k = D.KITTI(None, split='testing')
    assert k[0][2] == ['000000_10.png']
    # __rmul__ repeats the lists
    ds = 3 * D.KITTI(sparse)
    assert len(ds) == 6


def test_augmentors_deterministic_geometry(in_tree):
    """Dense augmentor with scale 0 and no flips: a crop of the input, flow unchanged."""
    from pytorch_raft_amd.data.augmentor import FlowAugmentor, SparseFlowAugmentor
    rng = np.random.default_rng(1)
    img1 = rng.integers(0, 255, (H, W, 3), dtype=np.uint8)
    img2 = rng.integers(0, 255, (H, W, 3), dtype=np.uint8)
    flow = _flow(rng)
    aug = FlowAugmentor((32, 48), min_scale=0.0, max_scale=0.0, do_flip=False)
    aug.spatial_aug_prob = 0.0
    np.random.seed(0)
    a1, a2, af = aug(img1, img2, flow)
    assert a1.shape == (32, 48, 3) and af.shape == (32, 48, 2)
    # the flow crop is a window of the input flow
    found = any(np.array_equal(af, flow[y:y + 32, x:x + 48])
                for y in range(H - 31) for x in range(W - 47))
    assert found
    saug = SparseFlowAugmentor((32, 48), min_scale=0.0, max_scale=0.0, do_flip=False)
    saug.spatial_aug_prob = 0.0
    valid = (rng.random((H, W)) > 0.3).astype(np.float32)
    s1, s2, sf, sv = saug(img1, img2, flow, valid)
    assert sf.shape == (32, 48, 2) and sv.shape == (32, 48)
    # invalid pixels carry no flow through the sparse path
    assert np.all(sf[sv < 0.5] == 0) or np.all(np.isfinite(sf))


def test_fetch_dataloader_stages_and_ranks(in_tree):
    from pytorch_raft_amd.data.datasets import fetch_dataloader, per_rank_batch
    for stage, size in (('chairs', (96, 128)), ('things', (96, 128)), ('sintel', (96, 128)),
                        ('kitti', (96, 128))):
        args = argparse.Namespace(stage=stage, image_size=list(size), batch_size=2)
        dl = fetch_dataloader(args, num_workers=0)
        b = next(iter(dl))
        assert b[0].shape == (2, 3, *size), stage
    # global batch semantics: 4 pairs on 2 ranks -> 2 per rank, disjoint shards
    args = argparse.Namespace(stage='sintel', image_size=[96, 128], batch_size=4)
    dl0 = fetch_dataloader(args, rank=0, world=2, num_workers=0)
    dl1 = fetch_dataloader(args, rank=1, world=2, num_workers=0)
    assert dl0.batch_size == 2 and dl1.batch_size == 2
    i0, i1 = list(dl0.sampler), list(dl1.sampler)
    assert not set(i0) & set(i1)
    with pytest.warns(UserWarning):
        assert per_rank_batch(10, 3) == 3


def _small_model():
    from pytorch_raft_amd import RAFT
    torch.manual_seed(0)
    return RAFT(argparse.Namespace(small=True, mixed_precision=False)).eval()


def test_validators_and_submissions(in_tree):
    from pytorch_raft_amd.engine import evaluate as E
    m = _small_model()
    r = E.validate_chairs(m, iters=2)
    assert np.isfinite(r['chairs'])
    r = E.validate_sintel(m, iters=2)
    assert set(r) == {'clean', 'final'} and all(np.isfinite(v) for v in r.values())
    r = E.validate_kitti(m, iters=2)
    assert np.isfinite(r['kitti-epe']) and 0 <= r['kitti-f1'] <= 100
    E.create_sintel_submission(m, iters=2, warm_start=True, output_path='sub_sintel')
    f = frame_utils.readFlow('sub_sintel/final/alley/frame0002.flo')
    assert f.shape == (H, W, 2)
    E.create_kitti_submission(m, iters=2, output_path='sub_kitti')
    kf, kv = frame_utils.readFlowKITTI('sub_kitti/000000_10.png')
    assert kf.shape == (H, W, 2) and kv.min() == 1


def _run(args, cwd, timeout=600):
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    r = subprocess.run([sys.executable] + args, cwd=cwd, env=env, capture_output=True, text=True,
                       timeout=timeout)
    assert r.returncode == 0, (r.stdout[-3000:], r.stderr[-3000:])
    return r.stdout


@pytest.mark.slow
def test_train_evaluate_demo_clis(in_tree):
    """train.py (2 steps + a checkpoint/validation cycle) -> evaluate.py -> the demo CLIs, all on
    the CPU with the reference's flags, on the fake tree."""
    out = _run([os.path.join(ROOT, 'train.py'), '--name', 'tiny', '--stage', 'chairs', '--small',
                '--num_steps', '2', '--batch_size', '2', '--image_size', '128', '128', '--cpu',
                '--gpus', '0', '--num_workers', '0', '--val_freq', '2', '--sum_freq', '1',
                '--validation', 'chairs', '--checkpoint_dir', 'ck', '--lr', '0.0001'], in_tree)
    assert 'Parameter Count' in out and 'Validation Chairs EPE' in out
    assert os.path.exists(in_tree / 'ck' / 'tiny.pth') and os.path.exists(in_tree / 'ck' / '2_tiny.pth')
    sd = torch.load(str(in_tree / 'ck' / 'tiny.pth'), map_location='cpu', weights_only=True)
    assert all(k.startswith('module.') for k in sd)
    ck = str(in_tree / 'ck' / 'tiny.pth')
    out = _run([os.path.join(ROOT, 'evaluate.py'), '--model', ck, '--dataset', 'kitti', '--small',
                '--iters', '2'], in_tree)
    assert 'Validation KITTI' in out
    frames = in_tree / 'frames'
    rng = np.random.default_rng(3)
    for k in range(3):
        _img(str(frames / ('f%02d.png' % k)), rng)
    _run([os.path.join(ROOT, 'demo.py'), '--model', ck, '--path', str(frames), '--small',
          '--iters', '2', '--save_dir', 'viz'], in_tree)
    assert len(os.listdir(in_tree / 'viz')) == 2
    _run([os.path.join(ROOT, 'demo_warp.py'), '--model', ck, '--path1', str(frames / 'f00.png'),
          '--path2', str(frames / 'f01.png'), '--small', '--save', 'mosaic.png'], in_tree)
    assert os.path.exists(in_tree / 'mosaic.png')
    _run([os.path.join(ROOT, 'demo_warp_folder.py'), '--model', ck, '--folderlist', str(frames),
          '--small', '--out_dir', 'warped'], in_tree)
    assert len(os.listdir(in_tree / 'warped')) == 2
    _run([os.path.join(ROOT, 'demo_warp_folder_firstframe.py'), '--model', ck, '--folderlist',
          str(frames), '--small', '--out_dir', 'chain'], in_tree)
    assert len(os.listdir(in_tree / 'chain')) >= 2
    _run([os.path.join(ROOT, 'frame2video.py'), '--readpath', str(frames), '--savepath', 'v.avi',
          '--size', str(W), str(H)], in_tree)
    assert os.path.getsize(in_tree / 'v.avi') > 0
