"""Encoders with per-image norms run huge batches in image chunks (the stem output must stay under
the 2 GiB byte-offset range, models/extractor.py:_chunk_images).  Chunked == unchunked, forward and
backward, on the CPU (fp32) with a tiny limit; batch norm is never chunked."""
import pytest
import torch

from pytorch_raft_amd.models.extractor import BasicEncoder, SmallEncoder


@pytest.mark.parametrize('cls,dim', [(BasicEncoder, 256), (SmallEncoder, 128)])
def test_instance_norm_encoder_chunked_matches_whole(monkeypatch, cls, dim):
    torch.manual_seed(0)
    enc = cls(output_dim=dim, norm_fn='instance').train()
    x1 = torch.randn(3, 3, 32, 40, requires_grad=True)
    x2 = torch.randn(3, 3, 32, 40, requires_grad=True)
    f1, f2 = enc([x1, x2])
    (f1.square().mean() + f2.mean()).backward()
    ref = [f1.detach(), f2.detach(), x1.grad.clone(), x2.grad.clone(),
           enc.conv1.weight.grad.clone()]
    enc.zero_grad()
    x1.grad = x2.grad = None
    per_img = enc.widths[0] * 16 * 20 * 4
    monkeypatch.setenv('RAFT_ENC_CHUNK_BYTES', str(2 * per_img + 1))  # 2 images per call
    assert enc._chunk_images(torch.cat([x1, x2])) == 2
    g1, g2 = enc([x1, x2])
    (g1.square().mean() + g2.mean()).backward()
    got = [g1.detach(), g2.detach(), x1.grad, x2.grad, enc.conv1.weight.grad]
    for a, b in zip(got, ref):
        torch.testing.assert_close(a, b, atol=1e-5, rtol=1e-5)


def test_batch_norm_encoder_chunked_only_when_frozen(monkeypatch):
    torch.manual_seed(1)
    enc = BasicEncoder(output_dim=256, norm_fn='batch').train()
    monkeypatch.setenv('RAFT_ENC_CHUNK_BYTES', '1')
    x = torch.randn(4, 3, 32, 40)
    assert enc._chunk_images(x) == 0  # training-mode batch statistics couple the images
    enc.eval()  # frozen statistics: per-image, chunkable (one image per call here)
    assert enc._chunk_images(x) == 1
    got = enc(x)
    monkeypatch.setenv('RAFT_ENC_CHUNK_BYTES', str(2 ** 31 - 1))
    torch.testing.assert_close(got, enc(x), atol=1e-5, rtol=1e-5)


def test_default_limit_keeps_headline_batches_whole():
    # chairs 368x496, bf16 stem: 5.84 MB per image -> 367 images per call; batch 96 (192 fnet
    # images) stays one call, batch 192 (384) becomes two calls of 192
    enc = BasicEncoder(output_dim=256, norm_fn='instance')
    with torch.autocast('cpu', dtype=torch.bfloat16):
        assert enc._chunk_images(torch.empty(1, 3, 368, 496).expand(192, -1, -1, -1)) == 0
        assert enc._chunk_images(torch.empty(1, 3, 368, 496).expand(384, -1, -1, -1)) == 367


@pytest.mark.parametrize('stride,k', [(1, 3), (2, 3), (2, 7), (2, 1)])
def test_fast_path_conv_chunks_oversized_batches(monkeypatch, stride, k):
    """A training-mode batch-norm encoder cannot be chunked as a whole; instead each conv whose
    input or output passes the 2 GiB offset range runs as equal image chunks (ops/encoder.py:
    _conv) -- same output and gradients as one call (CPU, bf16 channels_last, tiny limit)."""
    from pytorch_raft_amd.ops import encoder as fast
    torch.manual_seed(2)
    conv = torch.nn.Conv2d(8, 16, k, stride=stride, padding=k // 2)
    x = torch.randn(5, 8, 12, 14).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    ps = fast._Pass({}, {}, {})
    y0 = fast._conv(ps, x, conv)
    g = torch.randn_like(y0)
    (y0.float() * g).sum().backward()
    ref = (y0.detach().clone(), x.grad.clone(), conv.weight.grad.clone())
    x.grad = None
    conv.weight.grad = None
    monkeypatch.setattr(fast, '_CONV_BYTES', 2 * 16 * 12 * 14 * 2)   # two images per call
    y1 = fast._conv(ps, x, conv)
    assert y1.is_contiguous(memory_format=torch.channels_last)
    (y1.float() * g).sum().backward()
    torch.testing.assert_close(y1, ref[0], atol=0, rtol=0)
    torch.testing.assert_close(x.grad, ref[1], atol=0, rtol=0)
    # the weight gradient sums per-chunk bf16 gradients (autograd accumulation): bf16 rounding
    scale = ref[2].abs().max().item()
    torch.testing.assert_close(conv.weight.grad, ref[2], atol=2e-2 * scale, rtol=0)
