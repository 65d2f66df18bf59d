"""For one split-bf16 encoder conv inside the fp32 encoder: capture the output gradient it receives
and the input gradient it returns, and compare that input gradient with fp64 on the same output
gradient (is the conv wrong, or what it is given?)."""
import sys

import torch

sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv_fp32  # noqa: E402
from pytorch_raft_amd.models.extractor import BasicEncoder  # noqa: E402


def rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    torch.manual_seed(0)
    enc = BasicEncoder(output_dim=256, norm_fn='instance').cuda().train()
    x0 = torch.randn(3, 3, 96, 128, device='cuda')
    gout = torch.randn(3, 256, 12, 16, device='cuda')
    mods = dict(enc.named_modules())
    cap = {}
    for name in ('layer1.0.conv1', 'layer2.0.conv2', 'layer2.1.conv1', 'layer3.1.conv1'):
        m = mods[name]

        def fhook(mod, inp, out, _n=name):
            cap[_n] = {'x': inp[0].detach().clone(), 'w': mod.weight.detach().clone()}

            def nhook(grad_inputs, grad_outputs, _n=_n):
                cap[_n]['g'] = grad_outputs[0].detach().clone()
                cap[_n]['dx'] = grad_inputs[0].detach().clone()
            out.grad_fn.register_hook(nhook)
        m.register_forward_hook(fhook)
    x = x0.clone().requires_grad_(True)
    with conv_fp32.enabled(True):
        y = enc(x)
    (y * gout).sum().backward()
    for n, c in cap.items():
        g, dx, w = c['g'], c['dx'], c['w']
        ref = torch.nn.grad.conv2d_input(tuple(c['x'].shape), w.double().cpu(), g.double().cpu(),
                                         padding=w.shape[-1] // 2)
        mi = torch.nn.grad.conv2d_input(tuple(c['x'].shape), w, g, padding=w.shape[-1] // 2)
        print('%-16s g %s strides %s  |g| %.3e  split dx err %.2e  miopen dx err %.2e  ref norm %.3e' % (
            n, tuple(g.shape), g.stride(), g.norm().item(), rel(dx.double().cpu(), ref),
            rel(mi.double().cpu(), ref), ref.norm().item()), flush=True)
        # same g through the standalone split conv path
        xg = c['x'].clone().requires_grad_(True)
        yy = conv_fp32.conv2d(xg, w, None, (w.shape[-1] // 2,) * 2)
        dx2, = torch.autograd.grad(yy, xg, g)
        print('%-16s standalone split dx err %.2e; g absmax %.3e absmin(nonzero) %.3e' % (
            n, rel(dx2.double().cpu(), ref), g.abs().max().item(), g.abs()[g != 0].min().item()), flush=True)


if __name__ == '__main__':
    main()
