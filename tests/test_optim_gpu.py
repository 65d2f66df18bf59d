"""FusedAdamW (native multi-tensor AdamW with the global-norm clip folded in) vs torch's AdamW +
clip_grad_norm_ (reference `train.py:158-181`)."""
import pytest
import torch

from pytorch_raft_amd.engine.optim import FusedAdamW

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _rel(a, b):
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('lr_tensor', [False, True])
@pytest.mark.parametrize('max_norm', [None, 1.0, 1e3])
def test_fused_adamw_matches_torch(ext_ops, lr_tensor, max_norm):
    """Several steps over tensors of odd sizes (chunk tails, tensors smaller than a chunk, one
    spanning many chunks), a parameter without gradient, clipping active / inactive / off, and a
    float or device-tensor learning rate."""
    g = torch.Generator(device='cpu').manual_seed(0)
    shapes = [(7,), (4096,), (4097,), (3, 5, 7), (256, 128, 3, 3), (1,), (130, 1000)]
    ref = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    mine = [t.clone() for t in ref]
    pr = [torch.nn.Parameter(t) for t in ref]
    pm = [torch.nn.Parameter(t) for t in mine]
    lr = 2e-3
    o_ref = torch.optim.AdamW(pr, lr=lr, weight_decay=1e-4, eps=1e-8)
    o_my = FusedAdamW(pm, lr=torch.tensor(lr, device=DEV) if lr_tensor else lr, weight_decay=1e-4,
                      eps=1e-8)
    for step in range(5):
        for a, b in zip(pr, pm):
            gr = torch.randn(a.shape, generator=g).to(DEV) * 3
            a.grad = gr.clone()
            b.grad = gr.clone()
        pr[2].grad = pm[2].grad = None   # a parameter without a gradient this step
        if max_norm is not None:
            torch.nn.utils.clip_grad_norm_([p for p in pr if p.grad is not None], max_norm)
        o_ref.step()
        o_my.step(max_norm=max_norm)
        torch.cuda.synchronize()
        for a, b in zip(pr, pm):
            assert _rel(b.detach(), a.detach()) < 1e-6, step
    for a, b in zip(pr, pm):
        if o_ref.state.get(a):
            assert _rel(o_my.state[b]['exp_avg'], o_ref.state[a]['exp_avg']) < 1e-5
            assert _rel(o_my.state[b]['exp_avg_sq'], o_ref.state[a]['exp_avg_sq']) < 1e-5
    if max_norm is not None:
        # the reported total norm is the pre-clip gradient norm of the last step
        assert o_my.last_norm.shape == (2,)
