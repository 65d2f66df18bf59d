"""pytorch_raft_amd -- MI355X-native RAFT optical-flow training / inference engine.

Package layout
  models/    RAFT model family (state-dict compatible with the reference checkpoints)
  ops/       autograd wrappers of the hand-written gfx950 HIP kernels (csrc/) + torch oracles
  parallel/  one-process-per-GPU data parallelism over RCCL (torch.distributed 'nccl')
  data/      datasets, augmentation, synthetic pairs, loaders
  engine/    loss / optimizer / logger / checkpoint / training loop / evaluation
  utils/     padding, sampling, flow IO (.flo / PFM / KITTI PNG), flow visualisation, warping
"""
__version__ = '0.1.0'

from .models.raft import RAFT  # noqa: E402,F401
