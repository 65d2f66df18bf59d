"""fp64 emulation of the split-bf16 encoder forward (exact backward): gradient deviation caused by
the scheme itself.  usage: python scripts/fp32_enc_split_emulation.py instance|batch 3|4|f32
(3 = three bf16 products, 4 = with lo*lo, f32 = an fp32 forward instead)"""
import torch, sys
import torch.nn.functional as F
sys.path.insert(0,'.')
from pytorch_raft_amd.models.extractor import BasicEncoder
from pytorch_raft_amd.models import update as U
torch.manual_seed(0)
norm = sys.argv[1]; mode = sys.argv[2]
enc = BasicEncoder(output_dim=256, norm_fn=norm).train().double()
x0 = torch.randn(3, 3, 96, 128).double()
gout = torch.randn(3, 256, 12, 16).double()
def bf(t): return t.float().to(torch.bfloat16).double()
def split_conv(x, w, b, pad):
    xh = bf(x); xl = bf(x - xh); wh = bf(w); wl = bf(w - wh)
    y = F.conv2d(xh, wh, None, padding=pad) + F.conv2d(xl, wh, None, padding=pad) + F.conv2d(xh, wl, None, padding=pad)
    if mode == '4': y = y + F.conv2d(xl, wl, None, padding=pad)
    if mode == 'f32': y = F.conv2d(x.float(), w.float(), None, padding=pad).double()
    return y + b.view(1,-1,1,1)
class SF(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, pad):
        ctx.save_for_backward(x, w); ctx.pad = pad
        return split_conv(x, w, b, pad)
    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        dx = torch.nn.grad.conv2d_input(x.shape, w, g, padding=ctx.pad)
        dw = torch.nn.grad.conv2d_weight(x, w.shape, g, padding=ctx.pad)
        return dx, dw, g.sum((0,2,3)), None
def run(sim):
    orig = U.MfmaConv2d.forward
    if sim:
        def fwd(self, x):
            if self.stride == (1,1): return SF.apply(x, self.weight, self.bias, self.padding)
            return torch.nn.Conv2d.forward(self, x)
        U.MfmaConv2d.forward = fwd
    enc.zero_grad()
    x = x0.clone().requires_grad_(True)
    y = enc(x); (y*gout).sum().backward()
    U.MfmaConv2d.forward = orig
    return y.detach(), x.grad.detach(), {n: p.grad.clone() for n,p in enc.named_parameters()}
y0,d0,g0 = run(False); y1,d1,g1 = run(True)
rel=lambda a,b: ((a-b).norm()/b.norm()).item()
print(norm, mode, 'out %.2e dx %.2e layer1.0.conv1.w %.2e layer3.0.conv1.w %.2e' % (rel(y1,y0), rel(d1,d0), rel(g1['layer1.0.conv1.weight'], g0['layer1.0.conv1.weight']), rel(g1['layer3.0.conv1.weight'], g0['layer3.0.conv1.weight'])))
