"""Micro-benchmark of the all-pairs correlation backward fold (chairs shape, 12 iterations)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_raft_amd.ops import _ext
ops = _ext.ops()
B, H, W, L, R, K = 12, 46, 62, 4, 4, 12
g = torch.Generator(device='cuda').manual_seed(0)
ys, xs = torch.meshgrid(torch.arange(H, device='cuda').float(), torch.arange(W, device='cuda').float(), indexing='ij')
coords = [(torch.stack([xs, ys])[None].repeat(B, 1, 1, 1) + 3 * torch.randn(B, 2, H, W, device='cuda', generator=g)).contiguous() for _ in range(K)]
douts = [torch.randn(B, H, W, 384, device='cuda', generator=g).to(torch.bfloat16) for _ in range(K)]
for _ in range(3):
    out = ops.corr_tap_reduce(coords, douts, H, W, L, R, 1 / 16, True)
torch.cuda.synchronize()
t = time.perf_counter()
n = 10
for _ in range(n):
    out = ops.corr_tap_reduce(coords, douts, H, W, L, R, 1 / 16, True)
torch.cuda.synchronize()
print('corr_tap_reduce: %.1f us' % ((time.perf_counter() - t) / n * 1e6))
