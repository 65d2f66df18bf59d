"""fp64 conditioning of the encoder gradient: relative change of the output / input gradient when
every stride-1 conv output (forward) or its gradient (backward) gets 4e-6 relative noise.
usage: python scripts/fp32_enc_conditioning.py instance|batch"""
import torch, sys
sys.path.insert(0,'.')
from pytorch_raft_amd.models.extractor import BasicEncoder
from pytorch_raft_amd.models import update as U
torch.manual_seed(0)
enc = BasicEncoder(output_dim=256, norm_fn=sys.argv[1]).train().double()
x0 = torch.randn(3, 3, 96, 128).double()
gout = torch.randn(3, 256, 12, 16).double()
def run(eps_f=0.0, eps_b=0.0, only=None):
    hs=[]
    gen = torch.Generator().manual_seed(5)
    for n,m in enc.named_modules():
        if isinstance(m, U.MfmaConv2d) and m.stride==(1,1) and (only is None or n==only):
            def fh(mod, inp, out):
                if eps_f: out = out + eps_f*out.abs().mean()*torch.randn(out.shape, generator=gen, dtype=out.dtype)
                if eps_b:
                    out.register_hook(lambda g: g + eps_b*g.abs().mean()*torch.randn(g.shape, generator=gen, dtype=g.dtype))
                return out
            hs.append(m.register_forward_hook(fh))
    x = x0.clone().requires_grad_(True)
    y = enc(x); (y*gout).sum().backward()
    for h in hs: h.remove()
    return y.detach(), x.grad.detach()
y0, d0 = run()
rel=lambda a,b: ((a-b).norm()/b.norm()).item()
for ef, eb in ((4e-6,0),(0,4e-6)):
    y1,d1 = run(ef,eb)
    print(sys.argv[1], 'fwd noise %.0e bwd noise %.0e -> out %.2e dx %.2e' % (ef, eb, rel(y1,y0), rel(d1,d0)))
