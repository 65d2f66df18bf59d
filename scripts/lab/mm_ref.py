"""Library GEMM reference points for the update-block conv shapes (as plain GEMMs, im2col
ignored): what hipBLASLt / rocBLAS reach at M = 34,224 on MI355X."""
import torch
import time

dev = torch.device('cuda')
shapes = [('zr', 256, 1280), ('q', 128, 1280), ('c2', 192, 2304), ('head', 512, 1152),
          ('conv', 128, 2304), ('m2', 576, 256), ('c1', 256, 384)]
M = 34224
for name, N, K in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(3):
        e0.record()
        for _ in range(20):
            c = a @ b
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / 20 * 1e3)
    print('%-5s M %d N %d K %d: %.1f us  %.0f TF/s' % (name, M, N, K, best, 2 * M * N * K / best * 1e-6), flush=True)
