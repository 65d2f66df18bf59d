"""CPU dry run of the GPU-only orchestration: every HIP op replaced by a schema-checking stub.

Catches Python-side errors of the fused paths (argument order / counts / types against the
TORCH_LIBRARY schemas, autograd plumbing of the token nodes, buffer bookkeeping) without a GPU.
Numerics are covered by the GPU tests.
"""
import argparse
import os

import pytest
import torch

from pytorch_raft_amd.ops import _ext, update_hip

if not os.path.exists(_ext.LIB_PATH):
    pytest.skip('native library not built', allow_module_level=True)


def _returns():
    def corr_build(f1, f2, levels):
        b, c, h, w = f1.shape
        out = []
        for _ in range(levels):
            out.append(torch.zeros(b, h * w if not out else out[0].shape[1], h, w))
            h, w = h // 2, w // 2
        return out

    def corr_build_bf16(f1, f2, levels, pyr_bf16=False):
        b, h, w, c = f1.shape
        return corr_build(f1.permute(0, 3, 1, 2), f2, levels)

    def lookup(pyr, coords, r):
        b, _, h, w = coords.shape
        return torch.zeros(b, len(pyr) * (2 * r + 1) ** 2, h, w)

    def reduce(g, s):
        b, n = g[0].shape[:2]
        return torch.zeros(b, n, n)

    def cup_fwd(flow, mask, nhwc=False):
        b, _, h, w = flow.shape
        return torch.zeros(b, 2, 8 * h, 8 * w)

    def cup_bwd(flow, mask, dout, nhwc=False):
        return [torch.zeros_like(flow), torch.zeros_like(mask)]

    def loss_fwd(preds, gt, valid, g, m):
        return torch.ones(6)

    def loss_bwd(preds, gt, valid, dl, g, m):
        return [torch.zeros_like(p) for p in preds]

    def win_grad(coords, dout, levels, r):
        b, _, h, w = coords.shape
        return torch.zeros(b, h * w, levels, 2 * r + 2, 2 * r + 2)

    def tap_reduce(coords, douts, h, w, levels, r, s, bf16=False, pitch=0, split=False,
                   split_out=False):
        ld = (h * w + pitch - 1) // pitch * pitch if pitch else h * w
        if split_out:
            return torch.zeros(2, coords[0].shape[0], h * w, ld, dtype=torch.bfloat16)
        return torch.zeros(coords[0].shape[0], h * w, ld,
                           dtype=torch.bfloat16 if bf16 else torch.float32)

    def bwd_fmaps(dc, f1, f2):
        return [torch.zeros_like(f1), torch.zeros_like(f2)]

    def bwd_fmaps_split(dc2, f1, f2):
        b, c, h, w = f1.shape
        return [torch.zeros(b, h, w, c), torch.zeros(b, h, w, c)]

    def win_reduce(coords, wgs, h, w, levels, r, s, bf16=False):
        return torch.zeros(coords[0].shape[0], h * w, h * w,
                           dtype=torch.bfloat16 if bf16 else torch.float32)

    return {'corr_build': corr_build, 'corr_build_bf16': corr_build_bf16, 'corr_lookup_fwd': lookup, 'corr_pyr_grad_reduce': reduce,
            'corr_window_grad': win_grad, 'corr_window_reduce': win_reduce,
            'corr_tap_reduce': tap_reduce, 'corr_bwd_fmaps': bwd_fmaps,
            'corr_bwd_fmaps_split': bwd_fmaps_split,
            'convex_up_fwd': cup_fwd, 'convex_up_bwd': cup_bwd, 'seq_loss_fwd': loss_fwd,
            'seq_loss_bwd': loss_bwd}


@pytest.mark.parametrize('alternate', [False, True])
def test_dry_run_fused_training_step(alternate):
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip',
                              alternate_corr=alternate)
    torch.manual_seed(0)
    m = RAFT(args).train()
    i1, i2, flow, valid = make_pair_batch(2, 128, 160)
    with _ext.dry_run(_returns()) as ops:
        preds = m(i1, i2, iters=2)
        loss, metrics = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
    names = set(ops.calls)
    assert {'conv_fwd_', 'conv_dgrad_', 'conv_wgrad_taps_',
            'f1_patch_', 'fh2_fwd_', 'fh2_dgrad_', 'fh2_wgrad_', 'convex_up_fwd',
            'convex_up_bwd', 'seq_loss_fwd'} <= names, names
    # the motion encoder's ReLU backward rides in the last input-gradient conv's epilogue (gate 3)
    assert ('relu_bwd_' in names) == (not update_hip._GATES_FUSED)
    if not alternate:
        assert {'corr_build', 'corr_lookup_nhwc_', 'corr_tap_reduce'} <= names
    else:
        assert {'corr_otf_fwd_', 'corr_otf_window_bwd_'} <= names
    # every update-block parameter received a gradient through the fused backward
    for n, p in m.named_parameters():
        if n.startswith('update_block'):
            assert p.grad is not None and p.grad.shape == p.shape, n


def test_dry_run_small_model_training_step():
    """RAFT-small through the fused ConvGRU path (ops/update_hip_small.py): schema-checked ops,
    every update-block parameter gets a gradient of its own shape."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    args = argparse.Namespace(small=True, mixed_precision=True, corr_impl='hip', update_impl='hip')
    torch.manual_seed(0)
    m = RAFT(args).train()
    i1, i2, flow, valid = make_pair_batch(2, 128, 160)
    with _ext.dry_run(_returns()) as ops:
        preds = m(i1, i2, iters=2)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
    names = set(ops.calls)
    assert {'conv_fwd_', 'conv_dgrad_', 'conv_wgrad_taps_', 'gru_q_bwd_', 'gru_zr_bwd_', 'relu_bwd_',
            'f1_patch_', 'corr_lookup_nhwc_'} <= names, names
    for n, p in m.named_parameters():
        if n.startswith('update_block'):
            assert p.grad is not None and p.grad.shape == p.shape, n


def test_dry_run_inference():
    from pytorch_raft_amd import RAFT
    args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip')
    m = RAFT(args).eval()
    x = torch.rand(1, 3, 128, 128) * 255
    with _ext.dry_run(_returns()) as ops, torch.no_grad():
        lo, up = m(x, x, iters=3, test_mode=True)
    assert up.shape == (1, 2, 128, 128) and lo.shape == (1, 2, 16, 16)
    assert ops.calls.count('convex_up_fwd') == 1  # only after the last iteration


@pytest.mark.parametrize('alternate,small', [(False, False), (True, False), (False, True), (True, True)])
def test_dry_run_fp32_fused_training_step(alternate, small):
    """fp32 schedule (no mixed precision) through the fused block on split-fp32 operands: the
    conv schemas take the split flags, the flow head runs on the MFMA convs (no fh2_* VALU ops),
    and every update-block parameter gets a gradient of its own shape."""
    from pytorch_raft_amd import RAFT
    from pytorch_raft_amd.ops.loss import sequence_loss
    from pytorch_raft_amd.data.synthetic import make_pair_batch
    args = argparse.Namespace(small=small, mixed_precision=False, corr_impl='hip', update_impl='hip',
                              alternate_corr=alternate)
    torch.manual_seed(0)
    m = RAFT(args).train()
    i1, i2, flow, valid = make_pair_batch(2, 128, 160)
    with _ext.dry_run(_returns()) as ops:
        preds = m(i1, i2, iters=2)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
    names = set(ops.calls)
    assert {'conv_fwd_', 'conv_dgrad_', 'conv_wgrad_taps_', 'f1_patch_', 'split_hilo_'} <= names, names
    assert not ({'fh2_fwd_', 'fh2_dgrad_', 'fh2_wgrad_'} & names), names
    for n, p in m.named_parameters():
        if n.startswith('update_block'):
            assert p.grad is not None and p.grad.shape == p.shape, n
