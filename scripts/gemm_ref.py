"""Library bar for the update-block conv GEMM shapes: hipBLASLt (torch.matmul, bf16) on the same
M x N x K as each implicit-GEMM conv (M = 12 x 46 x 62 pixels, K = taps x Cin)."""
import torch

from scripts.conv_bench import GEOS, timeit  # noqa: E402

M = 12 * 46 * 62
for name, cout, k, segs in GEOS:
    K = k[0] * k[1] * sum(segs)
    a = torch.randn(M, K, device='cuda', dtype=torch.bfloat16)
    b = torch.randn(K, cout, device='cuda', dtype=torch.bfloat16)
    t = timeit(lambda: a @ b, 30)
    print(f'{name:5s} M {M} N {cout} K {K}: {t:6.1f} us  {2 * M * K * cout / t / 1e6:6.1f} TF/s', flush=True)
