"""Fused HIP update block (forward + hand-written backward) vs the eager PyTorch update block."""
import argparse

import pytest
import torch

from pytorch_raft_amd import RAFT
from pytorch_raft_amd.data.synthetic import make_pair_batch
from pytorch_raft_amd.ops.loss import sequence_loss

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _model(update_impl, mixed=True):
    args = argparse.Namespace(small=False, mixed_precision=mixed, corr_impl='hip',
                              update_impl=update_impl)
    torch.manual_seed(0)
    return RAFT(args).to(DEV)


def _cos(a, b):
    a, b = a.reshape(-1).double(), b.reshape(-1).double()
    return (a @ b / (a.norm() * b.norm() + 1e-30)).item()


def _slope(a, ref):
    """Least-squares gain of a on ref: bf16 rounding noise averages out of it, a systematic
    scale error (a mis-scaled gate, a dropped bias) does not."""
    a, ref = a.reshape(-1).double(), ref.reshape(-1).double()
    return (a @ ref / (ref @ ref + 1e-30)).item()


def test_fused_forward_matches_eager(ext_ops):
    i1, i2, _, _ = make_pair_batch(2, 128, 160, device=DEV)
    ref = _model('torch', mixed=False).eval()   # fp32 eager reference
    hip = _model('hip').eval()
    hip.load_state_dict(ref.state_dict())
    with torch.no_grad():
        lr, ur = ref(i1, i2, iters=4, test_mode=True)
        lh, uh = hip(i1, i2, iters=4, test_mode=True)
    err = (lh - lr).abs().max().item()
    scale = lr.abs().max().item()
    assert err < 0.05 * max(scale, 1.0), (err, scale)
    assert _cos(uh, ur) > 0.995
    # no systematic error: the gain of the fused flow on the fp32 one is 1 to well under 1 %
    k, kl = _slope(uh, ur), _slope(lh, lr)
    print('flow gain %.5f, low-res %.5f' % (k, kl))
    assert abs(k - 1) < 5e-3 and abs(kl - 1) < 5e-3, (k, kl)


def test_fused_training_grads_match_eager(ext_ops):
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    grads = {}
    losses = {}
    for impl, mixed in (('torch', False), ('hip', True)):
        m = _model(impl, mixed=mixed).train()
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        losses[impl] = loss.item()
        grads[impl] = {n: p.grad.detach().clone() for n, p in m.named_parameters()}
    assert abs(losses['hip'] - losses['torch']) < 0.02 * abs(losses['torch'])
    bad = []
    for n, g in grads['torch'].items():
        if not n.startswith('update_block'):
            continue
        c = _cos(grads['hip'][n], g)
        k = _slope(grads['hip'][n], g)
        if c < 0.98 or abs(k - 1) > 3e-2:
            bad.append((n, c, k))
    print('loss', losses, 'worst gains', sorted((abs(_slope(grads['hip'][n], g) - 1), n)
                                                 for n, g in grads['torch'].items()
                                                 if n.startswith('update_block'))[-3:])
    assert not bad, bad
    # encoder grads flow back through corr / net / inp
    # (bf16 encoder activations: the stem's gradient sits ~0.95 cos from fp32 under eager bf16
    # autocast too -- see tests/test_encoder_gpu.py)
    for n, lim in (('fnet.conv2.weight', 0.97), ('cnet.conv2.weight', 0.97), ('fnet.conv1.weight', 0.93)):
        assert _cos(grads['hip'][n], grads['torch'][n]) > lim, n


def test_fused_train_step_bf16(ext_ops):
    from pytorch_raft_amd.engine.trainer import TrainState
    args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', update_impl='hip',
                              lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100, iters=4,
                              gamma=0.8, clip=1.0, add_noise=False)
    torch.manual_seed(0)
    m = RAFT(args).to(DEV).train()
    st = TrainState(m, args, torch.device(DEV))
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    losses = [st.step(i1, i2, flow, valid)[0].item() for _ in range(6)]
    assert st.check_finite()
    assert losses[-1] < losses[0]


@pytest.mark.parametrize('cs,shape', [(512, (2, 11, 13)), (256, (3, 46, 62)), (512, (1, 7, 70))])
def test_flow_head2_kernels_match_fp32(ext_ops, cs, shape):
    """flow_head.conv2 (3x3, 256 -> 2) fwd / ReLU-gated dgrad / multi-item wgrad vs torch fp32."""
    import torch.nn.functional as F
    B, H, W = shape
    g = torch.Generator(device=DEV).manual_seed(3)
    w = torch.randn(2, 256, 3, 3, device=DEV, generator=g) * 0.05
    b = torch.randn(2, device=DEV, generator=g)
    fm = torch.relu(torch.randn(B, H, W, cs, device=DEV, generator=g)).to(torch.bfloat16)
    x = fm[..., :256].float().permute(0, 3, 1, 2)
    # forward
    out = torch.empty(B, 2, H, W, device=DEV)
    wb = w.to(torch.bfloat16)
    wf = wb.permute(2, 3, 0, 1).contiguous()        # bf16 pair tables: [t][o][c]
    wd = wb.permute(2, 3, 1, 0).contiguous()        # [t][c][o]
    ext_ops.fh2_fwd_(fm, wf, b, out)
    ref = F.conv2d(x, w, b, padding=1)
    # bf16 weights (v_dot2_f32_bf16), fp32 accumulation: ~0.2 % relative per product
    torch.testing.assert_close(out, ref, atol=3e-2, rtol=1e-2)
    # the iteration's coordinate update in the same launch: bitwise the eager fp32 ops
    from pytorch_raft_amd.utils.utils import coords_grid
    c0 = coords_grid(B, H, W, device=DEV)
    c1 = c0 + torch.randn(B, 2, H, W, device=DEV, generator=g) * 20
    out2, cn, fn = (torch.empty_like(out) for _ in range(3))
    ext_ops.fh2_fwd_(fm, wf, b, out2, c1, cn, fn)
    assert torch.equal(out2, out)
    assert torch.equal(cn, c1 + out) and torch.equal(fn, (c1 + out) - c0)
    # input gradient, gated by fm > 0, written into channels 0..255 of a cs-wide buffer
    gout = torch.randn(B, 2, H, W, device=DEV, generator=g)
    dx = torch.full((B, H, W, cs), 7.0, device=DEV, dtype=torch.bfloat16)
    ext_ops.fh2_dgrad_(gout, wd, fm, dx)
    xr = x.clone().requires_grad_(True)
    F.conv2d(xr, w, b, padding=1).backward(gout)
    dref = (xr.grad * (x > 0)).permute(0, 2, 3, 1)
    torch.testing.assert_close(dx[..., :256].float(), dref, atol=2e-2, rtol=1e-2)
    if cs > 256:
        assert (dx[..., 256:] == 7.0).all(), 'wrote past channel 255'
    # weight / bias gradient summed over 3 items, accumulated into existing values
    gouts = [gout, gout * 0.5, -gout]
    ins = [fm, fm, (fm.float() * 0.25).to(torch.bfloat16)]
    part = torch.full((5, 2 * 9 * 256 + 2), float('nan'), device=DEV)
    ext_ops.fh2_wgrad_(gouts, ins, part)                # every row fully written
    ps = part.sum(0)
    dw, db = ps[:-2].view(2, 9 * 256) + 1.0, ps[-2:] + 1.0
    wr = w.clone().requires_grad_(True)
    br = b.clone().requires_grad_(True)
    for go, xi in zip(gouts, ins):
        F.conv2d(xi[..., :256].float().permute(0, 3, 1, 2), wr, br, padding=1).backward(go)
    dw_ref = wr.grad.permute(0, 2, 3, 1).reshape(2, 9 * 256) + 1.0  # k = tap * 256 + c
    torch.testing.assert_close(dw, dw_ref, atol=1e-2, rtol=1e-3)
    torch.testing.assert_close(db, br.grad + 1.0, atol=1e-3, rtol=1e-4)


def test_inference_mask_skip_and_graph_match_eager(ext_ops):
    """Test-mode forward without the non-final mask heads, eager and hipGraph-replayed, equals
    the training-path forward (every iteration computes its mask)."""
    from pytorch_raft_amd.engine.inference import FlowInference
    torch.manual_seed(0)
    m = _model('hip').eval()
    i1, i2, _, _ = make_pair_batch(2, 124, 156, device=DEV)   # padded to 128 x 160
    with torch.no_grad():
        full = m(*[torch.nn.functional.pad(t, (2, 2, 2, 2), mode='replicate') for t in (i1, i2)],
                 iters=5)
    ref_up = full[-1][..., 2:-2, 2:-2]
    eager = FlowInference(m, iters=5)
    lo_e, up_e = eager(i1, i2)
    # the flow-only head conv may run a different tile config than the fused 512-wide one
    torch.testing.assert_close(up_e, ref_up, atol=5e-2, rtol=1e-3)
    graphed = FlowInference(m, iters=5, graph=True)
    lo_g, up_g = graphed(i1, i2)
    lo_g2, up_g2 = graphed(i2, i1)          # replay with new inputs
    lo_e2, up_e2 = eager(i2, i1)
    # MIOpen's encoder convs are not bitwise deterministic run to run (~1e-3 on the flow), so the
    # replay is compared with a tolerance far below the flow change caused by swapping the inputs
    swap = (up_e2 - up_e).abs().max().item()
    assert swap > 0.1, swap
    for a, b in ((up_g, up_e), (up_g2, up_e2), (lo_g2, lo_e2)):
        assert (a - b).abs().max().item() < 0.05 * swap


def test_f1_patch_matches_unfold(ext_ops):
    """convf1 im2col: patch[..., t*2 + c] = flow_c at 7x7 tap t (zero padded), 98.. zero; the
    flow is also written into the motion-feature slot."""
    import torch.nn.functional as F
    B, H, W = 2, 9, 13
    flow = torch.randn(B, 2, H, W, device=DEV) * 4
    patch = torch.full((B, H, W, 128), 5.0, device=DEV, dtype=torch.bfloat16)
    slot = torch.zeros(B, H, W, 128, device=DEV, dtype=torch.bfloat16)
    ext_ops.f1_patch_(flow, patch, slot, 126)
    u = F.unfold(flow, 7, padding=3).view(B, 2, 49, H, W)        # (c, tap)
    ref = u.permute(0, 3, 4, 2, 1).reshape(B, H, W, 98).to(torch.bfloat16)
    assert torch.equal(patch[..., :98], ref)
    assert (patch[..., 98:] == 0).all()
    assert torch.equal(slot[..., 126:], flow.permute(0, 2, 3, 1).to(torch.bfloat16))
    assert (slot[..., :126] == 0).all()


def test_fused_iterations_match_eager_bf16_same_precision(ext_ops):
    """The fused HIP update block (bf16 activations, fp32 MFMA accumulation) vs the eager
    BasicUpdateBlock under bf16 autocast (`core/update.py:114-136`) -- the same precision -- and
    both vs an fp32 eager oracle, chained over 3 GRU iterations.

    * forward: per-iteration h / delta / mask within 1e-2 (norm-relative) of eager bf16;
    * backward: every parameter gradient and the h0 / inp / corr gradients at least as close to
      the fp32 oracle as eager bf16 autocast is (x1.5 + 1e-2 slack).  Eager autocast rounds every
      intermediate gradient to bf16 while the fused backward keeps the accumulating gradients
      (dh, d inp, d motion features) in fp32, so eager bf16 itself sits several % from fp32 on
      the deepest (motion-encoder) gradients -- a bound of 1e-2 against eager bf16 would test
      eager's rounding, not the kernels."""
    from pytorch_raft_amd.models.update import BasicUpdateBlock
    from pytorch_raft_amd.ops.update_hip import HipUpdateBlock, CORR_BUF
    args = argparse.Namespace(corr_levels=4, corr_radius=4)
    torch.manual_seed(0)
    ub = BasicUpdateBlock(args, hidden_dim=128).to(DEV)
    B, H, W, T = 2, 23, 31, 3
    g = torch.Generator(device=DEV).manual_seed(5)
    h0 = torch.tanh(torch.randn(B, 128, H, W, device=DEV, generator=g)).to(torch.bfloat16)
    inp = torch.relu(torch.randn(B, 128, H, W, device=DEV, generator=g)).to(torch.bfloat16)
    corrs = [torch.randn(B, 324, H, W, device=DEV, generator=g).to(torch.bfloat16) for _ in range(T)]
    flows = [torch.randn(B, 2, H, W, device=DEV, generator=g) * 3 for _ in range(T)]
    Rh = [torch.randn(B, 128, H, W, device=DEV, generator=g) for _ in range(T)]
    Rd = [torch.randn(B, 2, H, W, device=DEV, generator=g) for _ in range(T)]
    Rm = [torch.randn(B, 576, H, W, device=DEV, generator=g) for _ in range(T)]

    def run(mode):
        ub.zero_grad(set_to_none=True)
        dt = torch.float32 if mode == 'fp32' else torch.bfloat16
        h = h0.detach().to(dt).clone().requires_grad_(True)
        x = inp.detach().to(dt).clone().requires_grad_(True)
        cs = [c.detach().to(dt).clone().requires_grad_(True) for c in corrs]
        outs, loss = [], 0.0
        if mode == 'fused':
            hub = HipUpdateBlock(ub)
            hh = h.permute(0, 2, 3, 1).contiguous()
            xx = x.permute(0, 2, 3, 1).contiguous()
            for t in range(T):
                cb = torch.nn.functional.pad(cs[t].permute(0, 2, 3, 1), (0, CORR_BUF - 324))
                hh, delta, mask = hub(hh, xx, cb.contiguous(), flows[t])
                outs.append((hh.permute(0, 3, 1, 2).float(), delta.float(),
                             mask.permute(0, 3, 1, 2).float()))
        else:
            hh = h
            for t in range(T):
                with torch.autocast('cuda', dtype=torch.bfloat16, enabled=(mode == 'bf16')):
                    hh, mask, delta = ub(hh, x, cs[t], flows[t])
                outs.append((hh.float(), delta.float(), mask.float()))
        for t, (hn, d, mk) in enumerate(outs):
            loss = loss + (hn * Rh[t]).sum() + (d * Rd[t]).sum() + (mk * Rm[t]).sum()
        loss.backward()
        grads = {n: p.grad.detach().float().clone() for n, p in ub.named_parameters()}
        grads['d_h0'] = h.grad.float()
        grads['d_inp'] = x.grad.float()
        for t in range(T):
            grads['d_corr%d' % t] = cs[t].grad.float()
        return outs, grads

    o_32, g_32 = run('fp32')
    o_bf, g_bf = run('bf16')
    o_fu, g_fu = run('fused')

    def rel(a, b):
        return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()

    bad, report = [], []
    for t in range(T):
        for k, name in enumerate(('h', 'delta', 'mask')):
            r = rel(o_fu[t][k], o_bf[t][k])
            report.append(('iter%d.%s vs eager-bf16' % (t, name), round(r, 5)))
            if r > 1e-2:
                bad.append(report[-1])
    for n in g_32:
        e_fu, e_bf = rel(g_fu[n], g_32[n]), rel(g_bf[n], g_32[n])
        report.append((n, 'fused %.4f / eager-bf16 %.4f vs fp32' % (e_fu, e_bf)))
        if e_fu > 1.5 * e_bf + 1e-2:
            bad.append(report[-1])
    print('\n'.join('%s: %s' % r for r in report))
    assert not bad, '\n'.join('%s: %s' % r for r in bad)


@pytest.mark.parametrize('amp', ['bfloat16', 'float16'])
def test_small_model_fused_matches_eager_bf16(ext_ops, amp):
    """RAFT-small on the fused ConvGRU path (ops/update_hip_small.py) vs the eager small model
    under bf16 / fp16 autocast (`core/update.py:16-31,62-77,99-112`; fp16 is the reference's
    --mixed_precision): same loss, flow and gradients within 16-bit tolerance, and the fused
    path is the one that ran."""
    from pytorch_raft_amd.ops import update_hip_small
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    outs = {}
    for impl in ('torch', 'hip'):
        args = argparse.Namespace(small=True, mixed_precision=True, corr_impl='hip',
                                  update_impl=impl, amp_dtype=amp)
        torch.manual_seed(0)
        m = RAFT(args).to(DEV).train()
        assert m._use_fused_update(i1) == (impl == 'hip')
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        outs[impl] = (loss.item(), preds[-1].detach(),
                      {n: p.grad.detach().clone() for n, p in m.named_parameters()})
    (le, fe, ge), (lh, fh, gh) = outs['torch'], outs['hip']
    assert abs(lh - le) < 0.02 * abs(le), (lh, le)
    assert _cos(fh, fe) > 0.995
    bad = [(n, _cos(gh[n], g)) for n, g in ge.items()
           if n.startswith('update_block') and _cos(gh[n], g) < 0.98]
    assert not bad, bad
    # eval / test mode through the fused path
    m.eval()
    with torch.no_grad():
        lo, up = m(i1, i2, iters=4, test_mode=True)
    assert up.shape == (2, 2, 128, 160) and torch.isfinite(up).all()
    assert update_hip_small.SMALL.spec['zr'].row_pad == 128


def test_fused_gate_epilogues_match_elementwise_kernels(ext_ops, monkeypatch):
    """ConvGRU gate backward fused into the dgrad epilogues (OSeg.gate) vs the separate
    gru_q_bwd / gru_zr_bwd kernels: the same fp32 algebra on the same values, so every
    update-block gradient and the encoder-output gradients agree to fp32 rounding (measured:
    bit-identical).  Both runs decode the SAME encoder outputs (the encoders' MIOpen solvers are
    not run-to-run deterministic: profiles/r2/diag_gates.log)."""
    from pytorch_raft_amd.ops import update_hip
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    m = _model('hip').train()
    with torch.no_grad():
        feats = [f.detach() for f in m.encode(i1, i2)]
    res = []
    for fused in (False, True):
        monkeypatch.setattr(update_hip, '_GATES_FUSED', fused)
        m.zero_grad(set_to_none=True)
        leaves = [f.clone().requires_grad_(True) for f in feats]
        preds = m.decode(*leaves, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        g = {n: p.grad.detach().clone() for n, p in m.named_parameters()
             if p.grad is not None and n.startswith('update_block')}
        g.update({'leaf%d' % k: t.grad.detach().float().clone() for k, t in enumerate(leaves)})
        res.append(g)
    ref, got = res
    assert ref.keys() == got.keys() and len(ref) > 4
    for n in ref:
        torch.testing.assert_close(got[n], ref[n],
                                   atol=1e-5 * max(ref[n].abs().max().item(), 1e-6),
                                   rtol=1e-4, msg=lambda msg: n + ': ' + msg)
