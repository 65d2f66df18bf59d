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
        if step % 2 == 0:
            # gradients on even steps only: its step count (bias correction) lags the others'
            pr[5].grad = pm[5].grad = None
        if max_norm is not None:
            torch.nn.utils.clip_grad_norm_([p for p in pr if p.grad is not None], max_norm)
        o_ref.step()
        o_my.step(max_norm=max_norm)
        torch.cuda.synchronize()
        for a, b in zip(pr, pm):
            assert _rel(b.detach(), a.detach()) < 1e-6, step
            if a.grad is not None:
                # the clipped gradient is written back, as clip_grad_norm_ leaves it
                assert _rel(b.grad, a.grad) < 1e-6, step
    for a, b in zip(pr, pm):
        if o_ref.state.get(a):
            assert _rel(o_my.state[b]['exp_avg'], o_ref.state[a]['exp_avg']) < 1e-5
            assert _rel(o_my.state[b]['exp_avg_sq'], o_ref.state[a]['exp_avg_sq']) < 1e-5
    if max_norm is not None:
        # the reported total norm is the pre-clip gradient norm of the last step
        assert o_my.last_norm.shape == (2,)


def test_fused_adamw_channels_last_params(ext_ops):
    """A channels_last model's conv weights (bench.py / train.py --channels_last): parameter,
    gradient and moments are walked flat in the parameter's own dense layout -- including a
    contiguous gradient and moments loaded before the model was re-laid out."""
    g = torch.Generator(device='cpu').manual_seed(1)
    shapes = [(64, 3, 7, 7), (128, 64, 3, 3), (96,)]
    ref = [torch.randn(s, generator=g).to(DEV) for s in shapes]
    pr = [torch.nn.Parameter(t.clone()) for t in ref]
    pm = [torch.nn.Parameter(t.clone().contiguous(memory_format=torch.channels_last) if t.dim() == 4
                             else t.clone()) for t in ref]
    o_ref = torch.optim.AdamW(pr, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    o_my = FusedAdamW(pm, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    for step in range(4):
        for a, b in zip(pr, pm):
            gr = torch.randn(a.shape, generator=g).to(DEV)
            a.grad = gr.clone()
            b.grad = gr.clone()   # contiguous gradient of a channels_last weight
        if step == 2:   # state laid out contiguously (as a loaded checkpoint's)
            for b in pm:
                for k in ('exp_avg', 'exp_avg_sq'):
                    o_my.state[b][k] = o_my.state[b][k].contiguous()
        torch.nn.utils.clip_grad_norm_(pr, 1.0)
        o_ref.step()
        o_my.step(max_norm=1.0)
        torch.cuda.synchronize()
        for a, b in zip(pr, pm):
            assert b.stride() == (b.contiguous(memory_format=torch.channels_last).stride()
                                  if b.dim() == 4 else b.stride())
            assert _rel(b.detach(), a.detach()) < 1e-6, step
            assert _rel(b.grad, a.grad) < 1e-6, step


def test_fused_adamw_global_norm_over_groups(ext_ops):
    """Two parameter groups (different lr / weight decay): the clip coefficient comes from the
    norm over ALL groups, as clip_grad_norm_ over every parameter."""
    g = torch.Generator(device='cpu').manual_seed(1)
    shapes = [(300,), (17, 9), (5000,)]
    ref = [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    groups = lambda ps: [dict(params=ps[:2], lr=1e-3, weight_decay=1e-2),   # noqa: E731
                         dict(params=ps[2:], lr=5e-3, weight_decay=0.0)]
    o_ref = torch.optim.AdamW(groups(ref), eps=1e-8)
    o_my = FusedAdamW(groups(mine), eps=1e-8)
    for step in range(3):
        for a, b in zip(ref, mine):
            gr = torch.randn(a.shape, generator=g).to(DEV) * (10.0 if step == 1 else 1.0)
            a.grad, b.grad = gr.clone(), gr.clone()
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        o_ref.step()
        o_my.step(max_norm=1.0)
        torch.cuda.synchronize()
        for a, b in zip(ref, mine):
            assert _rel(b.detach(), a.detach()) < 1e-6, step


def test_fused_adamw_gradscaler_unscale_clip_skip(ext_ops):
    """fp16 AMP step (reference `train.py:175-181`): FusedAdamW.step(max_norm, scaler) == torch's
    scaler.unscale_ + clip_grad_norm_ + scaler.step + scaler.update, including an overflow step
    (an inf gradient: the step is skipped, moments / step counts untouched, the scale backs off)
    -- all on the device."""
    g = torch.Generator(device='cpu').manual_seed(2)
    shapes = [(7,), (4097,), (64, 3, 3)]
    ref = [torch.nn.Parameter(torch.randn(s, generator=g).to(DEV)) for s in shapes]
    mine = [torch.nn.Parameter(p.detach().clone()) for p in ref]
    o_ref = torch.optim.AdamW(ref, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    o_my = FusedAdamW(mine, lr=1e-3, weight_decay=1e-4, eps=1e-8)
    s_ref = torch.amp.GradScaler('cuda', init_scale=2.0 ** 10, growth_interval=2)
    s_my = torch.amp.GradScaler('cuda', init_scale=2.0 ** 10, growth_interval=2)
    one = torch.ones((), device=DEV)
    s_ref.scale(one)
    s_my.scale(one)    # lazy scale / growth-tracker init, as the scaled backward does
    for step in range(6):
        S = float(s_ref.get_scale())
        assert S == float(s_my.get_scale()), step
        for a, b in zip(ref, mine):
            gr = torch.randn(a.shape, generator=g).to(DEV) * S
            if step == 3:
                gr[0] = float('inf')       # overflow: skipped step
            a.grad, b.grad = gr.clone(), gr.clone()
        s_ref.unscale_(o_ref)
        torch.nn.utils.clip_grad_norm_(ref, 1.0)
        s_ref.step(o_ref)
        s_ref.update()
        o_my.step(max_norm=1.0, scaler=s_my)
        torch.cuda.synchronize()
        for a, b in zip(ref, mine):
            assert _rel(b.detach(), a.detach()) < 1e-6, step
        assert float(s_my.get_scale()) == float(s_ref.get_scale()), step
    for a, b in zip(ref, mine):
        assert float(o_my.state[b]['step']) == float(o_ref.state[a]['step']) == 5.0
        assert _rel(o_my.state[b]['exp_avg_sq'], o_ref.state[a]['exp_avg_sq']) < 1e-5
