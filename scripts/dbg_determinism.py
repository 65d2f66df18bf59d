"""Locate forward non-determinism: run each stage of the fused RAFT forward twice on identical
inputs and print per-item max |diff| (0.0 everywhere = deterministic)."""
import argparse, sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from pytorch_raft_amd import RAFT
from pytorch_raft_amd.data.synthetic import make_pair_batch
from pytorch_raft_amd.models.corr import CorrBlock
from pytorch_raft_amd.ops import update_hip, conv as C
from pytorch_raft_amd.ops.update_hip import HipUpdateBlock, CORR_BUF

torch.manual_seed(0)
args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip')
m = RAFT(args).cuda().eval()
i1, i2, _, _ = make_pair_batch(2, 128, 160, device='cuda')
i1 = 2 * (i1 / 255) - 1; i2 = 2 * (i2 / 255) - 1


def d(name, a, b):
    if isinstance(a, (list, tuple)):
        for k, (x, y) in enumerate(zip(a, b)):
            d('%s[%d]' % (name, k), x, y)
        return
    if a is None:
        return
    print('%-14s' % name, ['%.3g' % float((a[k].float() - b[k].float()).abs().max()) for k in range(a.shape[0])], flush=True)


with torch.no_grad():
    def enc():
        with torch.autocast('cuda', dtype=torch.bfloat16):
            f1, f2 = m.fnet([i1, i2])
            c = m.cnet(i1)
        return f1.float().contiguous(), f2.float().contiguous(), c
    A, B = enc(), enc()
    d('fmap1', A[0], B[0]); d('fmap2', A[1], B[1]); d('cnet', A[2], B[2])
    f1, f2, c = A
    def corr():
        cb = CorrBlock(f1, f2, radius=4, impl='hip', precision='bf16')
        coords = m.initialize_flow(i1)[1] + torch.randn(2, 2, 16, 20, device='cuda')
        torch.manual_seed(1)
        return cb.lookup_nhwc(coords, CORR_BUF), cb
    torch.manual_seed(5); ca, cba = corr()
    torch.manual_seed(5); cb_, cbb = corr()
    d('corr lookup', ca, cb_)
    net, inp = torch.split(c, [128, 128], dim=1)
    h = torch.tanh(net).to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    x = torch.relu(inp).to(torch.bfloat16).permute(0, 2, 3, 1).contiguous()
    flow = torch.randn(2, 2, 16, 20, device='cuda')
    hub = HipUpdateBlock(m.update_block)
    outs = [hub(h, x, ca, flow, need_mask=True) for _ in range(2)]
    d('h', outs[0][0], outs[1][0]); d('delta', outs[0][1], outs[1][1]); d('mask', outs[0][2], outs[1][2])
    # per conv: run _iter_forward's convs individually
    pk = hub.state.packed
    sh = (2, 16, 20)
    def run_conv(name, segs, epi, cout_buf, aux=(), split=0, outs_n=1):
        s = update_hip.SPEC[name]
        res = []
        for _ in range(2):
            os_ = [torch.zeros(sh + (cout_buf,), device='cuda', dtype=torch.bfloat16) for _ in range(outs_n)]
            C.conv_fwd(segs, pk.w[name], pk.b[name], s.k, s.pad, s.cout, epi, os_, [0] * outs_n,
                       list(aux), [0] * len(aux), scale=s.scale, split=split, cin_small=2 if s.small else 0)
            res.append(os_)
        d('conv ' + name, res[0], res[1])
    run_conv('c1', [(ca, 0, CORR_BUF)], C.EPI_RELU_BF16, 256)
    c1 = torch.randn(sh + (256,), device='cuda').to(torch.bfloat16)
    run_conv('c2', [(c1, 0, 256)], C.EPI_RELU_BF16, 192)
    run_conv('conv', [(c1, 0, 256)], C.EPI_RELU_BF16, 128)
    mf = torch.randn(sh + (128,), device='cuda').to(torch.bfloat16)
    run_conv('zr1', [(h, 0, 128), (x, 0, 128), (mf, 0, 128)], C.EPI_GRU_ZR, 128, aux=[h], split=128, outs_n=3)
    run_conv('zr2', [(h, 0, 128), (x, 0, 128), (mf, 0, 128)], C.EPI_GRU_ZR, 128, aux=[h], split=128, outs_n=3)
    run_conv('head', [(h, 0, 128)], C.EPI_RELU_BF16, 512)
    fm = torch.relu(torch.randn(sh + (512,), device='cuda')).to(torch.bfloat16)
    run_conv('m2', [(fm, 256, 256)], C.EPI_BF16, 576)
