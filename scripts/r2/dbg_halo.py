"""Debug: dgrad-epilogue conv per forced config vs an fp32 reference."""
import sys
import torch
import torch.nn.functional as F
sys.path.insert(0, '.')
from pytorch_raft_amd.ops import conv as C, _ext  # noqa: E402

ops = _ext.ops()
dev = 'cuda'
torch.manual_seed(6)
B, H, W, hd = 2, 10, 14, 128
for (k, segs_out) in [((1, 5), [128, 128]), ((1, 5), [256]), ((3, 3), [128, 128])]:
    cin_g = 256
    cout = sum(segs_out)
    wf = torch.randn(cin_g, cout, *k, device=dev) / 40  # forward weight (Cout_f=256 x Cin_f=cout)
    g = torch.randn(B, cin_g, H, W, device=dev).to(torch.bfloat16)
    pad = (k[0] // 2, k[1] // 2)
    ref = F.conv_transpose2d(g.float(), wf.to(torch.bfloat16).float(), padding=pad)  # (B, cout, H, W)
    wd = C.pack_weight_dgrad(wf, [cin_g], [cin_g])
    gn = g.permute(0, 2, 3, 1).contiguous()
    for cfg in [-1, 10, 30, 31, 32, 33]:
        outs = [torch.zeros(B, H, W, c, device=dev) for c in segs_out]
        ops.conv_set_forced_cfg(cfg)
        try:
            ops.conv_dgrad_([gn], [0], [cin_g], wd, k[0], k[1], pad[0], pad[1], 0, 1.0, outs,
                            [0] * len(outs), segs_out, segs_out, [0] * len(outs), outs,
                            [0] * len(outs), [], [])
            torch.cuda.synchronize()
            got = torch.cat(outs, 3).permute(0, 3, 1, 2)
            err = (got - ref).abs().max().item()
            bad = ((got - ref).abs() > 1e-2).nonzero()
            print(k, segs_out, 'cfg', cfg, 'maxerr %.4g' % err, 'nbad', bad.shape[0],
                  bad[:4].tolist(), flush=True)
        except RuntimeError as e:
            print(k, segs_out, 'cfg', cfg, 'ERR', str(e)[:80])
        finally:
            ops.conv_set_forced_cfg(-1)
