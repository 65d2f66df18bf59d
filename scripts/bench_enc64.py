"""conv_enc64 (the encoders' 64 -> 64 stride-1 3x3 conv, conv_enc64.hip) at the chairs layer1
shapes: time per call of the kernel selected by RAFT_ENC64_KERNEL (pipe: producer / MFMA waves, the
default; half: channel halves at two workgroups per CU; wg1: one workgroup per CU) and the error vs
an fp32 F.conv2d of the same bf16 operands.
usage: RAFT_ENC64_KERNEL=pipe|half|wg1 PYTHONPATH=. python scripts/bench_enc64.py"""
import os

import torch
import torch.nn.functional as F

from pytorch_raft_amd.ops import _ext
from scripts.conv_bench import timeit

dev = torch.device('cuda')
ops = _ext.ops()
v1 = os.environ.get('RAFT_ENC64_KERNEL', 'pipe')
for name, B, H, W in [('fnet.l1', 24, 184, 248), ('cnet.l1', 12, 184, 248), ('odd', 3, 37, 45)]:
    torch.manual_seed(0)
    x = torch.randn(B, H, W, 64, device=dev).to(torch.bfloat16)
    w = (torch.randn(64, 64, 3, 3, device=dev) / 24.0).to(torch.bfloat16)
    wpk = w.permute(0, 2, 3, 1).reshape(64, 576).contiguous()
    out = torch.empty(B, H, W, 64, device=dev, dtype=torch.bfloat16)
    t = timeit(lambda: ops.conv_enc64_(x, wpk, out), 30)
    ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.float(), None, 1, 1).permute(0, 2, 3, 1)
    err = ((out.float() - ref).abs().max() / ref.abs().max()).item()
    tf = 2 * B * H * W * 64 * 576 / t / 1e6
    ck = out.view(torch.int16).double().sum().item()  # bitwise fingerprint: the variants must agree
    print(f'{v1} {name}: {t:7.1f} us  {tf:6.1f} TF/s  err {err:.1e}  ck {ck:.0f}', flush=True)
