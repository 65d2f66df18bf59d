"""CPU checks of the split-bf16 fp32 conv helpers (ops/conv_fp32.py): the hi/lo pair of an
fp32 tensor, and the packed [w_hi | w_hi | w_lo] weight whose virtual-concat product with
[x_hi | x_lo | x_hi] reproduces an fp32 conv to ~2^-16."""
import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import conv as C
from pytorch_raft_amd.ops import conv_fp32


def test_split_pair_is_exact_to_2e16():
    torch.manual_seed(0)
    x = torch.randn(2, 70, 5, 6) * 10
    buf = conv_fp32._split_nhwc(x, 128)
    assert buf.shape == (2, 5, 6, 256) and buf.dtype == torch.bfloat16
    hi, lo = buf[..., :70].float(), buf[..., 128:198].float()
    rec = (hi + lo).permute(0, 3, 1, 2)
    assert ((rec - x).abs() <= x.abs() * 2 ** -15).all()
    assert torch.all(buf[..., 70:128] == 0) and torch.all(buf[..., 198:] == 0)


def test_three_product_conv_matches_fp32():
    """The packed three-segment product, evaluated with a plain conv on the same bf16 operands,
    equals the fp32 conv to split-bf16 accuracy (what the MFMA kernel computes)."""
    torch.manual_seed(1)
    cin, cout, k = 96, 40, (3, 3)
    x = torch.randn(2, cin, 9, 11)
    w = torch.randn(cout, cin, *k) / 30
    cp = C.round_up(cin, 64)
    xs = conv_fp32._split_nhwc(x, cp).float()
    xin = torch.cat([xs[..., :cp], xs[..., cp:], xs[..., :cp]], -1).permute(0, 3, 1, 2)
    wpk = conv_fp32._pack3(w, cp).float()[:cout]                  # (cout, kh*kw*3cp)
    w3 = wpk.view(cout, k[0], k[1], 3 * cp).permute(0, 3, 1, 2)
    got = F.conv2d(xin, w3, padding=1)
    ref = F.conv2d(x.double(), w.double(), padding=1)
    rel = ((got.double() - ref).norm() / ref.norm()).item()
    assert rel < 3e-5, rel
