"""Recurrent update operator: motion encoder, (Sep)ConvGRU, flow head, convex-upsampling mask head.

Parity map (reference `core/update.py`):

==========================  =====================================  =========================
module                      reference lines                        state-dict prefix
==========================  =====================================  =========================
FlowHead                    6-14                                   flow_head.conv{1,2}
ConvGRU (small)             16-31                                  gru.conv{z,r,q}
SepConvGRU (full)           33-60                                  gru.conv{z,r,q}{1,2}
SmallMotionEncoder          62-77                                  encoder.conv{c1,f1,f2,}
BasicMotionEncoder          79-97                                  encoder.conv{c1,c2,f1,f2,}
SmallUpdateBlock            99-112
BasicUpdateBlock            114-136 (mask scaled by 0.25 at :135)  mask.{0,2}
==========================  =====================================  =========================

These modules are the weight containers AND the eager/CPU reference implementation.  The MI355X
hot path (``pytorch_raft_amd.ops.update_hip``) reads the very same parameters and runs the
iteration with fused HIP kernels; it never changes the checkpoint layout.
"""
import torch
import torch.nn as nn
import torch.nn.functional as F


class MfmaConv2d(nn.Conv2d):
    """nn.Conv2d (same parameters and state-dict keys) whose fp32 GPU forward runs on the bf16
    MFMA conv kernels as a split-bf16 product (``ops/conv_fp32.py``) while an fp32 model's update
    block is active (``conv_fp32.enabled()``); everything else is the plain nn.Conv2d path."""

    def forward(self, x):
        from ..ops import conv_fp32
        if (conv_fp32.active_for(x, self.weight) and self.stride == (1, 1) and
                self.dilation == (1, 1) and self.groups == 1 and self.padding_mode == 'zeros' and
                conv_fp32.fits(x, self.out_channels)):
            return conv_fp32.module_conv2d(self, x)
        return super().forward(x)


def _gru_gate_update(h, z, q):
    # h' = (1-z) h + z q  written as one lerp (same value, one fewer temporary)
    return torch.lerp(h, q, z)


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = MfmaConv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = MfmaConv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


class ConvGRU(nn.Module):
    """3x3 convolutional GRU (small model)."""

    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz = MfmaConv2d(cin, hidden_dim, 3, padding=1)
        self.convr = MfmaConv2d(cin, hidden_dim, 3, padding=1)
        self.convq = MfmaConv2d(cin, hidden_dim, 3, padding=1)

    def forward(self, h, x):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(self.convz(hx))
        r = torch.sigmoid(self.convr(hx))
        q = torch.tanh(self.convq(torch.cat([r * h, x], dim=1)))
        return _gru_gate_update(h, z, q)


class SepConvGRU(nn.Module):
    """Separable GRU: a (1x5) horizontal half-step then a (5x1) vertical one (full model)."""

    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz1 = MfmaConv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = MfmaConv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = MfmaConv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = MfmaConv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = MfmaConv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = MfmaConv2d(cin, hidden_dim, (5, 1), padding=(2, 0))

    @staticmethod
    def _half_step(h, x, cz, cr, cq):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(cz(hx))
        r = torch.sigmoid(cr(hx))
        q = torch.tanh(cq(torch.cat([r * h, x], dim=1)))
        return _gru_gate_update(h, z, q)

    def forward(self, h, x):
        h = self._half_step(h, x, self.convz1, self.convr1, self.convq1)
        h = self._half_step(h, x, self.convz2, self.convr2, self.convq2)
        return h


class SmallMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = MfmaConv2d(cor_planes, 96, 1, padding=0)
        self.convf1 = MfmaConv2d(2, 64, 7, padding=3)
        self.convf2 = MfmaConv2d(64, 32, 3, padding=1)
        self.conv = MfmaConv2d(128, 80, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc1(corr))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class BasicMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = MfmaConv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = MfmaConv2d(256, 192, 3, padding=1)
        self.convf1 = MfmaConv2d(2, 128, 7, padding=3)
        self.convf2 = MfmaConv2d(128, 64, 3, padding=1)
        self.conv = MfmaConv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow], dim=1)


class SmallUpdateBlock(nn.Module):
    def __init__(self, args, hidden_dim=96):
        super().__init__()
        self.encoder = SmallMotionEncoder(args)
        self.gru = ConvGRU(hidden_dim=hidden_dim, input_dim=82 + 64)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=128)

    def forward(self, net, inp, corr, flow):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        return net, None, self.flow_head(net)


class BasicUpdateBlock(nn.Module):
    MASK_SCALE = 0.25  # "scale mask to balance gradients" (`core/update.py:134-135`)

    def __init__(self, args, hidden_dim=128, input_dim=128):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(
            MfmaConv2d(128, 256, 3, padding=1),
            nn.ReLU(inplace=True),
            MfmaConv2d(256, 64 * 9, 1, padding=0))

    def forward(self, net, inp, corr, flow, upsample=True):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        delta_flow = self.flow_head(net)
        mask = self.MASK_SCALE * self.mask(net)
        return net, mask, delta_flow
