"""Bisect the split-bf16 fp32 encoder against fp64: the split conv enabled for ONE module at a
time (input-gradient error per module), then for all modules (error per parameter gradient)."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv_fp32  # noqa: E402
from pytorch_raft_amd.models import update as U  # noqa: E402
from pytorch_raft_amd.models.extractor import BasicEncoder  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main(norm):
    torch.manual_seed(0)
    enc = BasicEncoder(output_dim=256, norm_fn=norm).cuda().train()
    x0 = torch.randn(3, 3, 96, 128, device='cuda')
    gout = torch.randn(3, 256, 12, 16, device='cuda')

    def run(m, x, g, on=False):
        m.zero_grad(set_to_none=True)
        x = x.clone().requires_grad_(True)
        with conv_fp32.enabled(on):
            y = m(x)
        (y * g).sum().backward()
        return {'out': y.detach().double().cpu(), 'dx': x.grad.detach().double().cpu(),
                **{n: p.grad.detach().double().cpu() for n, p in m.named_parameters()}}

    ref = run(copy.deepcopy(enc).double().cpu(), x0.double().cpu(), gout.double().cpu())
    names = [n for n, m in enc.named_modules() if isinstance(m, U.MfmaConv2d)]
    orig = U.MfmaConv2d.forward
    for only in names:
        target = dict(enc.named_modules())[only]

        def fwd(self, x, _t=target):
            if self is _t:
                return orig(self, x)
            return torch.nn.Conv2d.forward(self, x)
        U.MfmaConv2d.forward = fwd
        r = run(enc, x0, gout, True)
        U.MfmaConv2d.forward = orig
        print('%s only %-22s out %.2e dx %.2e' % (norm, only, rel(r['out'], ref['out']), rel(r['dx'], ref['dx'])),
              flush=True)
    r = run(enc, x0, gout, True)
    m = run(enc, x0, gout, False)
    for n in ref:
        print('%s all  %-28s split %.2e  miopen %.2e' % (norm, n, rel(r[n], ref[n]), rel(m[n], ref[n])), flush=True)


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'instance')
