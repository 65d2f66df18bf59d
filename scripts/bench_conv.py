"""Microbenchmark: update-block conv shapes, our MFMA implicit-GEMM kernel vs MIOpen (torch conv2d).

Chairs training shape: B=12, 46x62 feature grid (P = 34,224 pixels).  Reports TFLOP/s per conv.
"""
import sys
import os
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from pytorch_raft_amd.ops import conv as C  # noqa: E402

SHAPES = [  # name, cin, cout, k, epi
    ('convc1 1x1 324->256', 384, 256, (1, 1), C.EPI_RELU_BF16),
    ('convc2 3x3 256->192', 256, 192, (3, 3), C.EPI_RELU_BF16),
    ('convf2 3x3 128->64', 128, 64, (3, 3), C.EPI_RELU_BF16),
    ('conv   3x3 256->126', 256, 126, (3, 3), C.EPI_RELU_BF16),
    ('gru zr 1x5 384->256', 384, 256, (1, 5), C.EPI_BF16),
    ('gru q  5x1 384->128', 384, 128, (5, 1), C.EPI_BF16),
    ('head   3x3 128->512', 128, 512, (3, 3), C.EPI_RELU_BF16),
    ('flow2  3x3 256->2', 256, 2, (3, 3), C.EPI_F32),
    ('mask2  1x1 256->576', 256, 576, (1, 1), C.EPI_F32),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def main():
    B, H, W = 12, 46, 62
    dev = 'cuda'
    torch.backends.cudnn.benchmark = True
    tot_ours = tot_miopen = tot_wg = 0.0
    print('%-22s %10s %10s %10s %10s %10s %10s' % ('conv', 'ours_us', 'ours_TF', 'miopen_us',
                                                   'miopen_TF', 'wgrad_us', 'wgrad_TF'))
    for name, cin, cout, k, epi in SHAPES:
        pad = (k[0] // 2, k[1] // 2)
        x = torch.randn(B, cin, H, W, device=dev, dtype=torch.bfloat16)
        w = torch.randn(cout, cin, *k, device=dev) / 30
        b = torch.randn(cout, device=dev)
        flops = 2.0 * B * H * W * cout * cin * k[0] * k[1]
        xb = C.nhwc(x)
        wpk = C.pack_weight(w, [cin], [cin])
        f32 = epi in (C.EPI_F32, C.EPI_ACC_F32)
        out = torch.empty(B, H, W, cout, device=dev, dtype=torch.float32 if f32 else torch.bfloat16)
        t_ours = timeit(lambda: C.conv_fwd([(xb, 0, cin)], wpk, b, k, pad, cout, epi, [out], [0]))
        xcl = x.contiguous(memory_format=torch.channels_last)
        wcl = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bb = b.to(torch.bfloat16)
        t_mi = timeit(lambda: F.conv2d(xcl, wcl, bb, padding=pad))
        g = torch.randn(B, H, W, C.round_up(cout, 8), device=dev, dtype=torch.bfloat16)
        dw = torch.zeros(cout, wpk.shape[1], device=dev)
        db = torch.zeros(cout, device=dev)
        t_wg = timeit(lambda: C.conv_wgrad(g, 0, [(xb, 0, cin)], k, pad, cout, dw, db))
        tot_ours += t_ours
        tot_miopen += t_mi
        tot_wg += t_wg
        print('%-22s %10.1f %10.1f %10.1f %10.1f %10.1f %10.1f' % (
            name, t_ours * 1e6, flops / t_ours / 1e12, t_mi * 1e6, flops / t_mi / 1e12,
            t_wg * 1e6, flops / t_wg / 1e12))
    print('total per update-block forward: ours %.3f ms, MIOpen(NHWC) %.3f ms; wgrad %.3f ms' % (
        tot_ours * 1e3, tot_miopen * 1e3, tot_wg * 1e3))




def print_tuned():
    t = torch.ops.raft_amd.conv_tune_table()
    print('autotuned conv configs: P H W KH KW cin cout small epi_class cfg BM BN')
    for i in range(0, len(t), 12):
        print('  ', t[i:i + 12])


if __name__ == '__main__':
    main()
    print_tuned()
