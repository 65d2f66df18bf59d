"""Native multi-source gather + cast (csrc/kernels/gather.hip) vs torch.cat + index_select + cast."""
import pytest
import torch

from pytorch_raft_amd.ops.conv import gather_index

pytestmark = pytest.mark.gpu
DEV = 'cuda'


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16, torch.float32])
@pytest.mark.parametrize('n_out', [1, 7, 4099, 300001])
def test_gather_cast_matches_index_select(ext_ops, dt, n_out):
    g = torch.Generator().manual_seed(n_out)
    numels = [int(x) for x in torch.randint(1, 5000, (23,), generator=g)]
    srcs = [torch.randn(n, generator=g).to(DEV) for n in numels]
    total = sum(numels)
    ids = torch.randint(0, total + 1, (n_out,), generator=g)   # total = the zero slot
    ids[0] = total
    flat = torch.cat([s for s in srcs] + [torch.zeros(1, device=DEV)])
    ref = flat.index_select(0, ids.to(DEV)).to(dt)
    out = torch.full((n_out,), 7.0, device=DEV, dtype=dt)
    ext_ops.gather_cast_(srcs, gather_index(ids, numels).to(DEV), out)
    assert torch.equal(out, ref)
    assert out[0].item() == 0.0


@pytest.mark.parametrize('st', [torch.bfloat16, torch.float16])
def test_gather_16bit_sources_to_fp32(ext_ops, st):
    g = torch.Generator().manual_seed(1)
    numels = [300, 17, 4096, 5]
    srcs = [torch.randn(n, generator=g).to(DEV).to(st) for n in numels]
    total = sum(numels)
    ids = torch.randperm(total, generator=g)
    flat = torch.cat(srcs).float()
    out = torch.empty(total, device=DEV)
    ext_ops.gather_cast_(srcs, gather_index(ids, numels).to(DEV), out)
    assert torch.equal(out, flat[ids.to(DEV)])


def test_gather_rejects_bad_args(ext_ops):
    src = [torch.randn(10, device=DEV)]
    idx = torch.zeros(4, dtype=torch.int32, device=DEV)
    with pytest.raises(RuntimeError):
        ext_ops.gather_cast_(src, idx, torch.empty(5, device=DEV))            # size mismatch
    with pytest.raises(RuntimeError):
        ext_ops.gather_cast_(src, idx.long(), torch.empty(4, device=DEV))     # int64 index
    with pytest.raises(RuntimeError):
        ext_ops.gather_cast_([s.double() for s in src], idx, torch.empty(4, device=DEV))
    with pytest.raises(RuntimeError):    # 16-bit -> 16-bit is not a packing direction
        ext_ops.gather_cast_([s.half() for s in src], idx, torch.empty(4, device=DEV).half())


@pytest.mark.parametrize('dt', [torch.bfloat16, torch.float16, torch.float32])
def test_image_prep_matches_eager(ext_ops, dt):
    """image_prep_: both frames -> 2 * (x / 255) - 1 -> one channels_last batch, bitwise the
    eager chain (ATen's scalar division = multiply by the float reciprocal)."""
    g = torch.Generator().manual_seed(0)
    a = (torch.rand(3, 3, 37, 53, generator=g) * 255).to(DEV)
    b = (torch.rand(3, 3, 37, 53, generator=g) * 255).to(DEV)
    ref = torch.cat([2 * (a / 255.0) - 1.0, 2 * (b / 255.0) - 1.0]).to(dt)
    out = torch.empty(6, 3, 37, 53, device=DEV, dtype=dt, memory_format=torch.channels_last)
    ext_ops.image_prep_(a, b, out)
    assert torch.equal(out, ref)


def test_gather_split_residual_sources(ext_ops):
    """lo_from: sources from that index on yield bf16(v - bf16(v)) -- the split-fp32 weight packs'
    w_lo -- while the others yield bf16(v)."""
    g = torch.Generator().manual_seed(2)
    numels = [500, 37, 1200]
    srcs = [torch.randn(n, generator=g).to(DEV) for n in numels]
    total = sum(numels)
    ids = torch.randint(0, 2 * total + 1, (20000,), generator=g)
    out = torch.empty(ids.numel(), device=DEV, dtype=torch.bfloat16)
    ext_ops.gather_cast_(srcs + srcs, gather_index(ids, numels + numels).to(DEV), out, len(srcs))
    flat = torch.cat(srcs)
    hi = flat.to(torch.bfloat16)
    lo = (flat - hi.float()).to(torch.bfloat16)
    ref = torch.cat([hi, lo, torch.zeros(1, device=DEV, dtype=torch.bfloat16)])[ids.to(DEV)]
    assert torch.equal(out, ref)
