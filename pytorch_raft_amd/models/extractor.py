"""Feature / context encoders.

Behavioural parity with the reference encoders (`core/extractor.py:6-267`):

* ``BasicEncoder``  (full model)  conv7x7/s2 3->64, norm, ReLU, 3 stages of two residual blocks
  (64, 96/s2, 128/s2) and a 1x1 projection (`core/extractor.py:118-192`).
* ``SmallEncoder``  (small model) same skeleton with bottleneck blocks 32 -> 32 -> 64 -> 96
  (`core/extractor.py:195-267`).
* A list/tuple input is run as ONE batched call and split back (`core/extractor.py:171-174,189-190`),
  which is what lets fnet see both frames in a single set of kernel launches.

State-dict schema is kept identical (`SURVEY.md` §2.5), including the strided residual block that
registers the same norm module as both ``norm3`` and ``downsample.1`` (`core/extractor.py:26,44-45`).

MI355X notes: on the GPU under bf16 autocast the forward runs the channels-last fast path of
``pytorch_raft_amd.ops.encoder``: the stride-1 convs on our MFMA implicit-GEMM kernels, the strided
ones on NHWC MIOpen convs, each norm + ReLU (and residual add + ReLU) one fused HIP autograd node,
conv biases folded into the norms.  An fp32 model (the reference's default schedule) runs its
stride-1 convs as split-bf16 MFMA products (``MfmaConv2d`` -> ``ops/conv_fp32.py``, ~2^-16
relative) while ``conv_fp32.enabled()`` is active; only the three strided convs stay on MIOpen.
"""
import os

import torch
import torch.nn as nn

from .update import MfmaConv2d


def make_norm(kind, channels, groups=None):
    """Normalisation factory used by every block (`core/extractor.py:14-36`)."""
    if kind == 'group':
        return nn.GroupNorm(num_groups=groups if groups is not None else channels // 8,
                            num_channels=channels)
    if kind == 'batch':
        return nn.BatchNorm2d(channels)
    if kind == 'instance':
        return nn.InstanceNorm2d(channels)
    if kind == 'none':
        return nn.Sequential()
    raise ValueError('unknown norm_fn %r' % (kind,))


class ResidualBlock(nn.Module):
    """Two 3x3 convs + identity / strided 1x1 shortcut (`core/extractor.py:6-56`)."""

    def __init__(self, in_planes, planes, norm_fn='group', stride=1):
        super().__init__()
        self.conv1 = MfmaConv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = MfmaConv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = make_norm(norm_fn, planes, g)
        self.norm2 = make_norm(norm_fn, planes, g)
        if stride == 1:
            self.downsample = None
        else:
            # the same module object under two names -> both key sets appear in state_dict
            self.norm3 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(
                MfmaConv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class BottleneckBlock(nn.Module):
    """1x1 -> 3x3 (strided) -> 1x1 bottleneck (`core/extractor.py:60-116`)."""

    def __init__(self, in_planes, planes, norm_fn='group', stride=1):
        super().__init__()
        mid = planes // 4
        self.conv1 = MfmaConv2d(in_planes, mid, kernel_size=1, padding=0)
        self.conv2 = MfmaConv2d(mid, mid, kernel_size=3, padding=1, stride=stride)
        self.conv3 = MfmaConv2d(mid, planes, kernel_size=1, padding=0)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = make_norm(norm_fn, mid, g)
        self.norm2 = make_norm(norm_fn, mid, g)
        self.norm3 = make_norm(norm_fn, planes, g)
        if stride == 1:
            self.downsample = None
        else:
            self.norm4 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(
                MfmaConv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm4)

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        y = self.relu(self.norm3(self.conv3(y)))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class _Encoder(nn.Module):
    """Shared skeleton of both encoders: stem, three 2-block stages, 1x1 head."""

    block = None
    widths = ()

    def __init__(self, output_dim=128, norm_fn='batch', dropout=0.0):
        super().__init__()
        self.norm_fn = norm_fn
        stem = self.widths[0]
        self.norm1 = make_norm(norm_fn, stem, 8)
        self.conv1 = MfmaConv2d(3, stem, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)

        self.in_planes = stem
        self.layer1 = self._make_layer(self.widths[1], stride=1)
        self.layer2 = self._make_layer(self.widths[2], stride=2)
        self.layer3 = self._make_layer(self.widths[3], stride=2)
        self.conv2 = MfmaConv2d(self.widths[3], output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        self._init_weights()

    def _init_weights(self):
        # kaiming(fan_out) convs, unit/zero affine norms (`core/extractor.py:150-157`)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode='fan_out', nonlinearity='relu')
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim, stride=1):
        first = self.block(self.in_planes, dim, self.norm_fn, stride=stride)
        second = self.block(dim, dim, self.norm_fn, stride=1)
        self.in_planes = dim
        return nn.Sequential(first, second)

    def _chunk_images(self, x):
        """Images per call so that the largest activation (the stem output at 1/2 resolution)
        stays under 2 GiB -- the int32 byte-offset range of MIOpen's kernels and of our buffer
        descriptors.  Past it MIOpen falls back to solvers that did not finish one batch-192
        training step (384 fnet images, a 2.24 GB stem output) in 10 minutes (profiles/r3/cfg).
        Only per-image norms may be chunked: batch norm in training mode couples the images
        (0 = no chunking); frozen batch norm (`freeze_bn`, every stage after chairs) is per-image."""
        if self.norm_fn == 'batch' and any(
                m.training for m in self.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)):
            return 0
        limit = int(os.environ.get('RAFT_ENC_CHUNK_BYTES', str(2 ** 31 - 1)))
        es = 2 if torch.is_autocast_enabled(x.device.type) else x.element_size()
        per_img = self.widths[0] * ((x.shape[2] + 1) // 2) * ((x.shape[3] + 1) // 2) * es
        n = max(1, limit // per_img)
        return n if x.shape[0] > n else 0

    def forward(self, x):
        batched = isinstance(x, (list, tuple))
        if batched:
            n = x[0].shape[0]
            x = torch.cat(x, dim=0)
        chunk = self._chunk_images(x)
        if chunk:
            # equal chunks (the same kernel configs for every chunk)
            k = -(-x.shape[0] // chunk)
            size = -(-x.shape[0] // k)
            x = torch.cat([self._run(c) for c in torch.split(x, size, dim=0)], dim=0)
        else:
            x = self._run(x)
        if batched:
            x = torch.split(x, [n, n], dim=0)
        return x

    def _run(self, x):
        from ..ops import encoder as fast
        if fast.fast_path_ok(self, x):
            # channels-last MIOpen convs + fused HIP norm/ReLU/residual nodes (ops/encoder.py)
            x = fast.encoder_forward(self, x)
        else:
            x = self.relu1(self.norm1(self.conv1(x)))
            x = self.layer3(self.layer2(self.layer1(x)))
            x = self.conv2(x)
            if self.training and self.dropout is not None:
                x = self.dropout(x)
        return x


class BasicEncoder(_Encoder):
    block = ResidualBlock
    widths = (64, 64, 96, 128)


class SmallEncoder(_Encoder):
    block = BottleneckBlock
    widths = (32, 32, 64, 96)
