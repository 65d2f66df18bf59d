"""CPU parity against the read-only reference implementation (used as an executable oracle).

The reference modules are imported from /root/reference/core when present (skipped otherwise);
random init is seeded identically, so both models hold bit-identical weights.
"""
import argparse
import importlib
import sys

import numpy as np
import pytest
import torch

from pytorch_raft_amd import RAFT
from pytorch_raft_amd.models.corr import (CorrBlock, torch_corr_pyramid, torch_corr_lookup,
                                          torch_onthefly_corr)
from pytorch_raft_amd.ops.upsample import torch_convex_upsample
from pytorch_raft_amd.utils import utils as U
from pytorch_raft_amd.utils import flow_viz


def _ref(module):
    return importlib.import_module(module)


@pytest.mark.parametrize('small', [False, True])
def test_raft_forward_matches_reference(reference_core, small):
    RefRAFT = _ref('raft').RAFT
    torch.manual_seed(0)
    ref = RefRAFT(argparse.Namespace(small=small, mixed_precision=False)).eval()
    torch.manual_seed(0)
    ours = RAFT(argparse.Namespace(small=small, mixed_precision=False, corr_impl='torch')).eval()
    for (k1, a), (k2, b) in zip(ref.state_dict().items(), ours.state_dict().items()):
        assert k1 == k2 and torch.equal(a, b)
    g = torch.Generator().manual_seed(1)
    x1 = torch.rand(1, 3, 128, 160, generator=g) * 255
    x2 = torch.rand(1, 3, 128, 160, generator=g) * 255
    with torch.no_grad():
        a = ref(x1, x2, iters=3)
        b = ours(x1, x2, iters=3)
        la, ua = ref(x1, x2, iters=3, test_mode=True)
        lb, ub = ours(x1, x2, iters=3, test_mode=True)
    for p, q in zip(a, b):
        torch.testing.assert_close(q, p, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(lb, la, atol=1e-4, rtol=1e-4)
    torch.testing.assert_close(ub, ua, atol=1e-4, rtol=1e-4)


def test_raft_train_mode_grads_match_reference(reference_core):
    RefRAFT = _ref('raft').RAFT
    torch.manual_seed(0)
    ref = RefRAFT(argparse.Namespace(small=False, mixed_precision=False)).train()
    torch.manual_seed(0)
    ours = RAFT(argparse.Namespace(small=False, mixed_precision=False, corr_impl='torch')).train()
    g = torch.Generator().manual_seed(2)
    x1 = torch.rand(1, 3, 128, 128, generator=g) * 255
    x2 = torch.rand(1, 3, 128, 128, generator=g) * 255
    ref(x1, x2, iters=2)[-1].square().mean().backward()
    ours(x1, x2, iters=2)[-1].square().mean().backward()
    ga = torch.cat([p.grad.reshape(-1) for p in ref.parameters()])
    gb = torch.cat([p.grad.reshape(-1) for p in ours.parameters()])
    assert ((ga - gb).norm() / ga.norm()) < 1e-4


def test_corrblock_matches_reference(reference_core):
    RefCorr = _ref('corr').CorrBlock
    g = torch.Generator().manual_seed(3)
    f1 = torch.randn(2, 64, 16, 20, generator=g)
    f2 = torch.randn(2, 64, 16, 20, generator=g)
    coords = U.coords_grid(2, 16, 20) + 3 * torch.randn(2, 2, 16, 20, generator=g)
    a = RefCorr(f1, f2, radius=4)(coords)
    b = CorrBlock(f1, f2, radius=4, impl='torch')(coords)
    torch.testing.assert_close(b, a, atol=1e-5, rtol=1e-5)


def test_onthefly_oracle_equals_allpairs():
    g = torch.Generator().manual_seed(4)
    f1 = torch.randn(2, 32, 16, 24, generator=g)
    f2 = torch.randn(2, 32, 16, 24, generator=g)
    coords = U.coords_grid(2, 16, 24) + 5 * torch.randn(2, 2, 16, 24, generator=g)
    coords[:, :, 0, 0] = -40.0
    for r in (3, 4):
        pyr = torch_corr_pyramid(f1, f2, 4)
        a = torch_corr_lookup(pyr, coords, r)
        p2 = [f2]
        for _ in range(3):
            p2.append(torch.nn.functional.avg_pool2d(p2[-1], 2, 2))
        b = torch_onthefly_corr(p2, f1, coords, r)
        torch.testing.assert_close(b, a, atol=1e-5, rtol=1e-4)


def test_convex_upsample_matches_reference(reference_core):
    RefRAFT = _ref('raft').RAFT
    m = RefRAFT(argparse.Namespace(small=False, mixed_precision=False))
    g = torch.Generator().manual_seed(5)
    flow = torch.randn(2, 2, 6, 7, generator=g)
    mask = torch.randn(2, 576, 6, 7, generator=g)
    torch.testing.assert_close(torch_convex_upsample(flow, mask), m.upsample_flow(flow, mask))


def test_utils_match_reference(reference_core):
    RU = _ref('utils.utils')
    for shape in [(1, 3, 436, 1024), (1, 3, 375, 1242), (2, 3, 368, 496)]:
        for mode in ('sintel', 'kitti'):
            a, b = RU.InputPadder(shape, mode=mode), U.InputPadder(shape, mode=mode)
            assert a._pad == b._pad
            x = torch.randn(*shape)
            pa, pb = a.pad(x)[0], b.pad(x)[0]
            assert torch.equal(pa, pb)
            assert torch.equal(b.unpad(pb), x)
    assert torch.equal(RU.coords_grid(2, 5, 7, 'cpu'), U.coords_grid(2, 5, 7, 'cpu'))
    f = torch.randn(1, 2, 5, 6)
    torch.testing.assert_close(U.upflow8(f), RU.upflow8(f))
    img = torch.randn(3, 1, 9, 11)
    c = torch.rand(3, 4, 4, 2) * 12 - 1
    torch.testing.assert_close(U.bilinear_sampler(img, c), RU.bilinear_sampler(img, c))


def test_forward_interpolate_matches_reference(reference_core):
    RU = _ref('utils.utils')
    g = torch.Generator().manual_seed(6)
    flow = 3 * torch.randn(2, 12, 17, generator=g)
    torch.testing.assert_close(U.forward_interpolate(flow), RU.forward_interpolate(flow))


def test_flow_viz_matches_reference(reference_core):
    RV = _ref('utils.flow_viz')
    assert np.array_equal(flow_viz.make_colorwheel(), RV.make_colorwheel())
    rng = np.random.RandomState(0)
    f = rng.randn(20, 30, 2).astype(np.float32) * 5
    assert np.array_equal(flow_viz.flow_to_image(f), RV.flow_to_image(f))
    assert np.array_equal(flow_viz.flow_to_image(f, convert_to_bgr=True),
                          RV.flow_to_image(f, convert_to_bgr=True))
