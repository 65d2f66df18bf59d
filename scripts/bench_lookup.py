"""Time the bf16 all-pairs pyramid build (corr_build_bf16) and the NHWC
pyramid lookup (corr_lookup_nhwc_; RAFT_LOOKUP_TPV=4|8|16 pixels per workgroup) at the chairs
training shape (B=12, 46x62, 4 levels, r=4).  Prints us per call
and a checksum (variants must agree bit for bit)."""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import _ext  # noqa: E402


def main():
    ops = _ext.ops()
    b, h, w, c = 12, 46, 62, 256
    g = torch.Generator(device='cpu').manual_seed(0)
    f1 = torch.randn(b, h, w, c, generator=g).to(torch.bfloat16).cuda()
    f2 = torch.randn(b, h, w, c, generator=g).to(torch.bfloat16).cuda()
    pyr = ops.corr_build_bf16(f1, f2, 4, True)
    ys, xs = torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing='ij')
    coords = (torch.stack([xs, ys])[None].repeat(b, 1, 1, 1) + 4 * torch.randn(b, 2, h, w, generator=g)).cuda()
    out = torch.empty(b, h, w, 384, device='cuda', dtype=torch.bfloat16)
    for _ in range(3):
        ops.corr_lookup_nhwc_(pyr, coords, 4, out)
        pyr = ops.corr_build_bf16(f1, f2, 4, True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        pyr = ops.corr_build_bf16(f1, f2, 4, True)
    e1.record()
    torch.cuda.synchronize()
    print('corr_build_bf16 %.1f us/call  checksum %.6f' % (e0.elapsed_time(e1) * 100,
                                                          sum(float(p.float().sum()) for p in pyr)), flush=True)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 20
    e0.record()
    for _ in range(n):
        ops.corr_lookup_nhwc_(pyr, coords, 4, out)
    e1.record()
    torch.cuda.synchronize()
    print('corr_lookup_nhwc %.1f us/call  checksum %.6f' % (e0.elapsed_time(e1) * 1000 / n,
                                                           out.float().sum().item()), flush=True)


if __name__ == '__main__':
    main()
