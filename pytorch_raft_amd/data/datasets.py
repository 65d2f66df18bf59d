"""Optical-flow datasets and the per-stage training mix (reference `core/datasets.py`).

Classes keep the reference constructor signatures, default roots and on-disk conventions:

=================  ==========================================================  ==========
class              layout                                                      GT
=================  ==========================================================  ==========
MpiSintel          Sintel/{split}/{clean|final}/<scene>/*.png consecutive       .flo dense
FlyingChairs       FlyingChairs_release/data/*.ppm|*.flo + chairs_split.txt     .flo dense
FlyingThings3D     {dstype}/TRAIN/*/*/left, optical_flow/TRAIN/*/*/{dir}/left    .pfm dense
KITTI              {split}/image_2/*_10.png,*_11.png, flow_occ/*_10.png          PNG16 sparse
HD1K               hd1k_input/image_2/%06d_*.png, hd1k_flow_gt/flow_occ          PNG16 sparse
=================  ==========================================================  ==========

``fetch_dataloader(args)`` reproduces the stage table (`core/datasets.py:199-234`).  Multi-process
training gets a ``DistributedSampler`` so each rank reads a disjoint shard with a per-rank batch of
``batch_size / world`` (the reference's ``--batch_size`` is the global DataParallel batch).
``chairs_split.txt`` is looked up in the CWD, then ``txt/`` and the repo root (the reference only
looks in the CWD although the file ships in ``txt/``).
"""
import os
import os.path as osp
import random
from glob import glob

import numpy as np
import torch
import torch.utils.data as data

from ..utils import frame_utils
from .augmentor import FlowAugmentor, SparseFlowAugmentor

_REPO = osp.dirname(osp.dirname(osp.dirname(osp.abspath(__file__))))

# Worker RNG seed = _WORKER_SEED_BASE + worker id.  The reference seeds worker k with k
# (`core/datasets.py:45-51`), which under one-process-per-GPU data parallelism would give worker k
# of EVERY rank the same crop / flip / jitter / eraser stream; ``fetch_dataloader`` sets the base to
# rank * num_workers inside each worker (``_seed_worker``) so every (rank, worker) pair is distinct.
_WORKER_SEED_BASE = 0


class _seed_worker:
    """Picklable DataLoader ``worker_init_fn``: records this rank's seed base in the worker."""

    def __init__(self, base):
        self.base = int(base)

    def __call__(self, worker_id):
        global _WORKER_SEED_BASE
        _WORKER_SEED_BASE = self.base


def per_rank_batch(global_batch, world, rank=0):
    """Per-rank batch for a GLOBAL ``--batch_size`` (reference DataParallel semantics).  A batch
    that does not divide by the world size is rounded down; rank 0 says so, since the effective
    global batch (and with it the gradient scale per step) differs from the one asked for."""
    per = max(1, global_batch // world)
    if per * world != global_batch and rank == 0:
        import warnings
        warnings.warn('--batch_size %d is not divisible by %d ranks: training with %d pairs per rank '
                      '(effective global batch %d)' % (global_batch, world, per, per * world))
    return per


class FlowDataset(data.Dataset):
    def __init__(self, aug_params=None, sparse=False):
        self.augmentor = None
        self.sparse = sparse
        if aug_params is not None:
            self.augmentor = SparseFlowAugmentor(**aug_params) if sparse else FlowAugmentor(**aug_params)
        self.is_test = False
        self.init_seed = False
        self.flow_list = []
        self.image_list = []
        self.extra_info = []

    @staticmethod
    def _rgb(img):
        img = np.array(img).astype(np.uint8)
        if img.ndim == 2:
            return np.tile(img[..., None], (1, 1, 3))
        return img[..., :3]

    def __getitem__(self, index):
        if self.is_test:
            img1 = self._rgb(frame_utils.read_gen(self.image_list[index][0]))
            img2 = self._rgb(frame_utils.read_gen(self.image_list[index][1]))
            img1 = torch.from_numpy(img1).permute(2, 0, 1).float()
            img2 = torch.from_numpy(img2).permute(2, 0, 1).float()
            return img1, img2, self.extra_info[index]

        if not self.init_seed:
            info = torch.utils.data.get_worker_info()
            if info is not None:
                seed = _WORKER_SEED_BASE + info.id
                torch.manual_seed(seed)
                np.random.seed(seed)
                random.seed(seed)
                self.init_seed = True

        index = index % len(self.image_list)
        valid = None
        if self.sparse:
            flow, valid = frame_utils.readFlowKITTI(self.flow_list[index])
        else:
            flow = frame_utils.read_gen(self.flow_list[index])
        img1 = self._rgb(frame_utils.read_gen(self.image_list[index][0]))
        img2 = self._rgb(frame_utils.read_gen(self.image_list[index][1]))
        flow = np.array(flow).astype(np.float32)

        if self.augmentor is not None:
            if self.sparse:
                img1, img2, flow, valid = self.augmentor(img1, img2, flow, valid)
            else:
                img1, img2, flow = self.augmentor(img1, img2, flow)

        img1 = torch.from_numpy(np.ascontiguousarray(img1)).permute(2, 0, 1).float()
        img2 = torch.from_numpy(np.ascontiguousarray(img2)).permute(2, 0, 1).float()
        flow = torch.from_numpy(np.ascontiguousarray(flow)).permute(2, 0, 1).float()
        if valid is not None:
            valid = torch.from_numpy(np.ascontiguousarray(valid))
        else:
            valid = (flow[0].abs() < 1000) & (flow[1].abs() < 1000)
        return img1, img2, flow, valid.float()

    def __rmul__(self, v):
        self.flow_list = v * self.flow_list
        self.image_list = v * self.image_list
        return self

    def __len__(self):
        return len(self.image_list)


class MpiSintel(FlowDataset):
    def __init__(self, aug_params=None, split='training', root='datasets/Sintel', dstype='clean'):
        super().__init__(aug_params)
        flow_root = osp.join(root, split, 'flow')
        image_root = osp.join(root, split, dstype)
        if split == 'test':
            self.is_test = True
        scenes = sorted(os.listdir(image_root)) if osp.isdir(image_root) else []
        for scene in scenes:
            images = sorted(glob(osp.join(image_root, scene, '*.png')))
            for i in range(len(images) - 1):
                self.image_list.append([images[i], images[i + 1]])
                self.extra_info.append((scene, i))
            if split != 'test':
                self.flow_list += sorted(glob(osp.join(flow_root, scene, '*.flo')))


def _find_split_file(name='chairs_split.txt'):
    for cand in (name, osp.join('txt', name), osp.join(_REPO, 'txt', name), osp.join(_REPO, name)):
        if osp.exists(cand):
            return cand
    raise FileNotFoundError(name)


class FlyingChairs(FlowDataset):
    def __init__(self, aug_params=None, split='train', root='datasets/FlyingChairs_release/data'):
        super().__init__(aug_params)
        images = sorted(glob(osp.join(root, '*.ppm')))
        flows = sorted(glob(osp.join(root, '*.flo')))
        assert len(images) // 2 == len(flows)
        split_list = np.loadtxt(_find_split_file(), dtype=np.int32)
        for i in range(len(flows)):
            xid = split_list[i]
            if (split == 'training' and xid == 1) or (split == 'validation' and xid == 2):
                self.flow_list.append(flows[i])
                self.image_list.append([images[2 * i], images[2 * i + 1]])


class FlyingThings3D(FlowDataset):
    def __init__(self, aug_params=None, root='datasets/FlyingThings3D', dstype='frames_cleanpass'):
        super().__init__(aug_params)
        for cam in ['left']:
            for direction in ['into_future', 'into_past']:
                image_dirs = sorted(osp.join(f, cam) for f in glob(osp.join(root, dstype, 'TRAIN/*/*')))
                flow_dirs = sorted(osp.join(f, direction, cam)
                                   for f in glob(osp.join(root, 'optical_flow/TRAIN/*/*')))
                for idir, fdir in zip(image_dirs, flow_dirs):
                    images = sorted(glob(osp.join(idir, '*.png')))
                    flows = sorted(glob(osp.join(fdir, '*.pfm')))
                    for i in range(len(flows) - 1):
                        if direction == 'into_future':
                            self.image_list.append([images[i], images[i + 1]])
                            self.flow_list.append(flows[i])
                        else:
                            self.image_list.append([images[i + 1], images[i]])
                            self.flow_list.append(flows[i + 1])


class KITTI(FlowDataset):
    def __init__(self, aug_params=None, split='training', root='datasets/KITTI'):
        super().__init__(aug_params, sparse=True)
        if split == 'testing':
            self.is_test = True
        root = osp.join(root, split)
        images1 = sorted(glob(osp.join(root, 'image_2/*_10.png')))
        images2 = sorted(glob(osp.join(root, 'image_2/*_11.png')))
        for img1, img2 in zip(images1, images2):
            self.extra_info.append([osp.basename(img1)])
            self.image_list.append([img1, img2])
        if split == 'training':
            self.flow_list = sorted(glob(osp.join(root, 'flow_occ/*_10.png')))


class HD1K(FlowDataset):
    def __init__(self, aug_params=None, root='datasets/HD1k'):
        super().__init__(aug_params, sparse=True)
        seq = 0
        while True:
            flows = sorted(glob(osp.join(root, 'hd1k_flow_gt', 'flow_occ/%06d_*.png' % seq)))
            images = sorted(glob(osp.join(root, 'hd1k_input', 'image_2/%06d_*.png' % seq)))
            if len(flows) == 0:
                break
            for i in range(len(flows) - 1):
                self.flow_list.append(flows[i])
                self.image_list.append([images[i], images[i + 1]])
            seq += 1


STAGE_AUG = {
    'chairs': dict(min_scale=-0.1, max_scale=1.0, do_flip=True),
    'things': dict(min_scale=-0.4, max_scale=0.8, do_flip=True),
    'sintel': dict(min_scale=-0.2, max_scale=0.6, do_flip=True),
    'kitti': dict(min_scale=-0.2, max_scale=0.4, do_flip=False),
}


def build_train_dataset(args, TRAIN_DS='C+T+K+S+H'):
    crop = args.image_size
    aug = dict(crop_size=crop, **STAGE_AUG[args.stage]) if args.stage in STAGE_AUG else None
    if args.stage == 'chairs':
        return FlyingChairs(aug, split='training')
    if args.stage == 'things':
        return (FlyingThings3D(aug, dstype='frames_cleanpass')
                + FlyingThings3D(aug, dstype='frames_finalpass'))
    if args.stage == 'sintel':
        things = FlyingThings3D(aug, dstype='frames_cleanpass')
        clean = MpiSintel(aug, split='training', dstype='clean')
        final = MpiSintel(aug, split='training', dstype='final')
        if TRAIN_DS == 'C+T+K+S+H':
            kitti = KITTI({'crop_size': crop, 'min_scale': -0.3, 'max_scale': 0.5, 'do_flip': True})
            hd1k = HD1K({'crop_size': crop, 'min_scale': -0.5, 'max_scale': 0.2, 'do_flip': True})
            return 100 * clean + 100 * final + 200 * kitti + 5 * hd1k + things
        return 100 * clean + 100 * final + things
    if args.stage == 'kitti':
        return KITTI(aug, split='training')
    raise ValueError('unknown stage %r' % (args.stage,))


def fetch_dataloader(args, TRAIN_DS='C+T+K+S+H', rank=0, world=1, num_workers=4):
    """Per-stage training loader.  ``args.batch_size`` is the GLOBAL batch (reference semantics)."""
    ds = build_train_dataset(args, TRAIN_DS)
    per_rank = per_rank_batch(args.batch_size, world, rank)
    sampler = None
    if world > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=world, rank=rank,
                                                                  shuffle=True, drop_last=True)
    loader = data.DataLoader(ds, batch_size=per_rank, pin_memory=torch.cuda.is_available(),
                             shuffle=sampler is None, sampler=sampler, num_workers=num_workers,
                             drop_last=True, persistent_workers=num_workers > 0,
                             worker_init_fn=_seed_worker(rank * max(1, num_workers)))
    if rank == 0:
        print('Training with %d image pairs (global batch %d = %d ranks x %d)'
              % (len(ds), per_rank * world, world, per_rank))
    return loader
