"""Run one update-block conv shape N times (for rocprofv3 PMC runs).  usage: conv_one.py <layer> [n]"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from pytorch_raft_amd.ops import conv as C  # noqa: E402

SH = {'zr': (384, 256, (1, 5)), 'zr2': (256, 256, (1, 5)), 'q': (384, 128, (5, 1)), 'c2': (256, 192, (3, 3)),
      'head': (128, 512, (3, 3)), 'conv': (256, 126, (3, 3)), 'm2': (256, 576, (1, 1))}
name = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 20
cin, cout, k = SH[name]
B, H, W = 12, 46, 62
dev = 'cuda'
x = torch.randn(B, H, W, cin, device=dev).to(torch.bfloat16)
w = torch.randn(cout, cin, *k, device=dev) / 30
b = torch.randn(cout, device=dev)
wpk = C.pack_weight(w, [cin], [cin])
out = torch.empty(B, H, W, cout, device=dev, dtype=torch.bfloat16)
pad = (k[0] // 2, k[1] // 2)
for _ in range(n):
    C.conv_fwd([(x, 0, cin)], wpk, b, k, pad, cout, C.EPI_BF16, [out], [0])
torch.cuda.synchronize()
print(name, 'cfg', os.environ.get('RAFT_CONV_CFG'), torch.ops.raft_amd.conv_tune_table())
