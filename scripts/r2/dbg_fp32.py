"""Time the split-bf16 fp32 conv pieces at bench size (batch 12, 46x62)."""
import sys
import time
import torch
sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv_fp32, conv as C  # noqa: E402

dev = 'cuda'
B, H, W = 12, 46, 62
for cin, cout, k in [(384, 256, (1, 5)), (256, 192, (3, 3)), (128, 256, (3, 3))]:
    pad = (k[0] // 2, k[1] // 2)
    x = torch.randn(B, cin, H, W, device=dev, requires_grad=True)
    w = (torch.randn(cout, cin, *k, device=dev) * 0.02).requires_grad_()
    b = torch.zeros(cout, device=dev, requires_grad=True)
    for rep in range(3):
        torch.cuda.synchronize(); t0 = time.time()
        y = conv_fp32.conv2d(x, w, b, pad)
        torch.cuda.synchronize(); t1 = time.time()
        y.backward(torch.ones_like(y))
        torch.cuda.synchronize(); t2 = time.time()
        print(cin, cout, k, 'rep', rep, 'fwd %.2f ms  bwd %.2f ms' % ((t1 - t0) * 1e3, (t2 - t1) * 1e3), flush=True)
    cp = C.round_up(cin, 64)
    xs = conv_fp32._split_nhwc(x.detach(), cp)
    cop = C.round_up(cout, 64)
    gs = conv_fp32._split_nhwc(torch.ones(B, cout, H, W, device=dev), cop)
    d1 = torch.zeros(cout, k[0] * k[1] * 2 * cp, device=dev)
    for rep in range(2):
        torch.cuda.synchronize(); t0 = time.time()
        C.conv_wgrad(gs, 0, [(xs, 0, cp), (xs, cp, cp)], k, pad, cout, d1)
        torch.cuda.synchronize(); t1 = time.time()
        print('   wgrad hi x [hi|lo] %.2f ms' % ((t1 - t0) * 1e3), flush=True)
