"""End-to-end RAFT on the GPU: HIP path vs stock-ops path, training step, native code really used."""
import argparse

import pytest
import torch

from pytorch_raft_amd import RAFT
from pytorch_raft_amd.data.synthetic import make_pair_batch

pytestmark = pytest.mark.gpu
DEV = 'cuda'


def _model(impl, small=False, alternate=False, mixed=False):
    args = argparse.Namespace(small=small, mixed_precision=mixed, alternate_corr=alternate,
                              corr_impl=impl)
    torch.manual_seed(0)
    return RAFT(args).to(DEV)


@pytest.mark.parametrize('small', [False, True])
@pytest.mark.parametrize('alternate', [False, True])
def test_hip_matches_torch_forward_fp32(ext_ops, small, alternate):
    i1, i2, _, _ = make_pair_batch(2, 128, 160, device=DEV)
    ref = _model('torch', small).eval()
    hip = _model('hip', small, alternate).eval()
    hip.load_state_dict(ref.state_dict())
    with torch.no_grad():
        lr, ur = ref(i1, i2, iters=4, test_mode=True)
        lh, uh = hip(i1, i2, iters=4, test_mode=True)
    torch.testing.assert_close(lh, lr, atol=2e-3, rtol=1e-3)
    torch.testing.assert_close(uh, ur, atol=2e-2, rtol=1e-3)


def test_hip_training_grads_match_torch(ext_ops):
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    from pytorch_raft_amd.ops.loss import sequence_loss
    grads = {}
    for impl in ('torch', 'hip'):
        m = _model(impl).train()
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8, impl=impl)
        loss.backward()
        grads[impl] = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    a, b = grads['torch'], grads['hip']
    rel = (a - b).norm() / a.norm()
    # fp32 model: the HIP path runs the update block AND the encoders' stride-1 convs as split-bf16
    # products (~4e-6 per conv); the encoders' early-layer gradients amplify a forward
    # perturbation of that size ~1000x even in fp64 (profiles/r4/fp32_encoder_conditioning.txt)
    assert rel < 3e-3, rel


def test_train_step_bf16_runs(ext_ops):
    """The HIP training step learns: 12 AdamW steps on one batch (`train.py:161-181`, no noise)
    must lower the sequence loss -- the last three steps' mean clearly below the first three's.
    The 2,000-step synthetic-flow run against the stock ops is profiles/r6/parity/."""
    from pytorch_raft_amd.engine.trainer import TrainState
    args = argparse.Namespace(small=False, mixed_precision=True, corr_impl='hip', lr=4e-4,
                              wdecay=1e-4, epsilon=1e-8, num_steps=20, iters=3, gamma=0.8,
                              clip=1.0, add_noise=False)
    torch.manual_seed(0)
    m = RAFT(args).to(DEV).train()
    st = TrainState(m, args, torch.device(DEV))
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    losses = []
    for _ in range(12):
        loss, metrics = st.step(i1, i2, flow, valid)
        losses.append(loss.item())
    assert st.check_finite()
    first, last = sum(losses[:3]) / 3, sum(losses[-3:]) / 3
    assert losses[-1] < losses[0] and last < 0.95 * first, losses


def test_native_library_loaded(ext_ops):
    import os
    from pytorch_raft_amd.ops import _ext
    assert _ext.loaded()
    maps = open('/proc/self/maps').read()
    assert os.path.basename(_ext.LIB_PATH) in maps


def test_alternate_training_grads_match_allpairs(ext_ops):
    """On-the-fly (MFMA, bf16 backward operands) vs all-pairs HIP path: same loss gradients."""
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    from pytorch_raft_amd.ops.loss import sequence_loss
    grads = {}
    for alt in (False, True):
        m = _model('hip', alternate=alt).train()
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        grads[alt] = torch.cat([p.grad.reshape(-1) for p in m.parameters()])
    rel = (grads[True] - grads[False]).norm() / grads[False].norm()
    assert rel < 2e-2, rel


def test_wgrad_overlap_matches_inline(ext_ops):
    """Side-stream weight-gradient flush (end-of-backward join) == in-graph gradients, up to the
    run-to-run noise of the float-atomic split-K reductions (measured with overlap off twice)."""
    from pytorch_raft_amd.ops import update_hip
    from pytorch_raft_amd.ops.loss import sequence_loss
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    runs = []
    try:
        for overlap in (False, False, True):
            update_hip.set_wgrad_overlap(overlap)
            m = _model('hip', mixed=True).train()
            preds = m(i1, i2, iters=3)
            loss, _ = sequence_loss(preds, flow, valid, 0.8, impl='hip')
            loss.backward()
            torch.cuda.synchronize()
            runs.append([p.grad.clone() for p in m.update_block.parameters()])
    finally:
        update_hip.set_wgrad_overlap(False)
    # MIOpen's encoder convs are not bitwise reproducible from run to run (solver choice), which
    # moves every update-block gradient by up to ~1 % between identical runs; a lost or stale
    # weight-gradient contribution on the side stream would be far larger than that
    # (norm-wise: a near-cancelling fp32 atomic sum such as a tiny bias gradient can move by a few
    # % of its max element when only the atomics' order changes)
    # The side stream's autotune timings run beside the encoder backward and may pick another
    # split-K tile (another reduction order), so a tensor whose gradient nearly cancels (a bias
    # two orders below the block's gradient) can move by a few % of its own norm; bound that by
    # the block's gradient norm too.  A lost / stale contribution moves whole tensors by O(1).
    gscale = torch.cat([a.reshape(-1) for a in runs[0]]).norm().item()
    for a, a2, b in zip(*runs):
        noise = (a - a2).norm().item()
        scale = a.norm().item()
        diff = (a - b).norm().item()
        assert diff <= 4 * noise + 3e-2 * scale + 2e-3 * gscale + 1e-7, (diff, noise, scale, gscale)
        if scale > 1e-2 * gscale:
            cos = torch.nn.functional.cosine_similarity(a.reshape(1, -1), b.reshape(1, -1)).item()
            assert cos > 0.999, cos


def test_auto_corr_mode_switches_on_budget(ext_ops, monkeypatch):
    """corr_mode='auto': all-pairs while the pyramid fits the HBM budget, on-the-fly past it --
    same flow either way (the two blocks compute the same windows)."""
    i1, i2, _, _ = make_pair_batch(2, 128, 160, device=DEV)
    m = _model('hip').eval()
    with torch.no_grad():
        lo_ap, up_ap = m(i1, i2, iters=4, test_mode=True)
        assert m.last_corr == 'all-pairs'
        monkeypatch.setenv('RAFT_CORR_BUDGET_GB', '1e-6')   # 1 KiB: any pyramid exceeds it
        lo_ot, up_ot = m(i1, i2, iters=4, test_mode=True)
        assert m.last_corr == 'on-the-fly'
    torch.testing.assert_close(lo_ot, lo_ap, atol=2e-3, rtol=1e-3)
    torch.testing.assert_close(up_ot, up_ap, atol=2e-2, rtol=1e-3)


def _fp16_args(**kw):
    a = dict(small=False, mixed_precision=True, amp_dtype='float16', corr_impl='hip', lr=4e-4,
             wdecay=1e-4, epsilon=1e-8, num_steps=100, iters=3, gamma=0.8, clip=1.0,
             add_noise=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_fp16_gradscaler_grads_match_fp32(ext_ops):
    """The reference's --mixed_precision (`train.py:154,175-181`): fp16 autocast + GradScaler.
    Unscaled fp16 gradients vs the fp32 model's on the same weights (BN frozen: no batch-stat
    coupling), and the fp16 path must not lose to bf16 (more mantissa, same step)."""
    from pytorch_raft_amd.ops.loss import sequence_loss
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    grads = {}
    for prec in ('fp32', 'fp16', 'bf16'):
        args = _fp16_args(mixed_precision=prec != 'fp32',
                          amp_dtype='float16' if prec == 'fp16' else 'bfloat16')
        torch.manual_seed(0)
        m = RAFT(args).to(DEV).train()
        m.freeze_bn()
        scaler = torch.amp.GradScaler('cuda', init_scale=2.0 ** 12, enabled=prec == 'fp16')
        # every precision runs the fused MFMA update block (fp16: v_mfma_f32_32x32x16_f16; fp32:
        # split-fp32 operands), not eager ops
        assert m._use_fused_update(i1), prec
        preds = m(i1, i2, iters=3)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        scaler.scale(loss).backward()
        g = torch.cat([p.grad.reshape(-1).float() for p in m.parameters()])
        if prec == 'fp16':
            g = g / scaler.get_scale()
        grads[prec] = g
    ref = grads['fp32']
    rel16 = ((grads['fp16'] - ref).norm() / ref.norm()).item()
    rel_bf = ((grads['bf16'] - ref).norm() / ref.norm()).item()
    print('rel grad err vs fp32: fp16 %.3e  bf16 %.3e' % (rel16, rel_bf))
    assert torch.isfinite(grads['fp16']).all()
    assert rel16 < 2e-2, rel16
    assert rel16 < 1.5 * rel_bf + 1e-3, (rel16, rel_bf)


def test_fp16_train_step_gradscaler(ext_ops):
    """fp16 TrainState steps: loss scaling, unscale before clip, device-side found-inf skip (fused
    AdamW takes found_inf / no host sync) and the scale update.  A 2^40 initial scale overflows
    the fp16 gradients: that step must leave the weights untouched and halve the scale; later
    steps train normally."""
    from pytorch_raft_amd.engine.trainer import TrainState
    args = _fp16_args()
    torch.manual_seed(0)
    m = RAFT(args).to(DEV).train()
    st = TrainState(m, args, torch.device(DEV))
    assert st.scaler.is_enabled()
    st.scaler = torch.amp.GradScaler('cuda', init_scale=2.0 ** 40, growth_interval=1000)
    i1, i2, flow, valid = make_pair_batch(2, 128, 160, device=DEV)
    w0 = torch.cat([p.detach().reshape(-1).clone() for p in m.parameters()])
    st.step(i1, i2, flow, valid)
    w1 = torch.cat([p.detach().reshape(-1).clone() for p in m.parameters()])
    assert torch.equal(w0, w1), 'overflowed step must be skipped'
    assert st.scaler.get_scale() < 2.0 ** 40
    losses = []
    for _ in range(60):
        s0 = st.scaler.get_scale()
        loss, _ = st.step(i1, i2, flow, valid)
        if st.scaler.get_scale() >= s0:   # no overflow: the step was taken
            losses.append(loss.item())
        if len(losses) >= 4:
            break
    w2 = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
    assert not torch.equal(w1, w2), 'no step was taken once the scale came down'
    assert all(l == l for l in losses) and losses[-1] < losses[0] * 1.5, losses


def test_bf16_encoder_streams_first_call_serial(ext_ops):
    """bf16 autocast runs the context encoder on a side stream -- from the SECOND call of an input
    signature on: the first call (MIOpen's solver search for the strided convs) stays on one
    stream.  The two-stream call gives the same features, flows and gradients as the one-stream
    call (the encoders are deterministic)."""
    from pytorch_raft_amd.models import raft as raft_mod
    from pytorch_raft_amd.ops.loss import sequence_loss
    if raft_mod._ENC_STREAMS != 'auto':
        pytest.skip('RAFT_ENC_STREAMS forced')
    raft_mod._ENC_SEEN.clear()
    i1, i2, flow, valid = make_pair_batch(2, 96, 128, device=DEV)
    m = _model('hip', mixed=True).train()
    m.freeze_bn()
    outs = []
    for _ in range(2):
        m.zero_grad(set_to_none=True)
        preds = m(i1, i2, iters=2)
        loss, _ = sequence_loss(preds, flow, valid, 0.8)
        loss.backward()
        outs.append((m.last_enc_streams, preds[-1].detach().float(),
                     torch.cat([p.grad.reshape(-1).float() for p in m.parameters() if p.grad is not None])))
    assert outs[0][0] == 1 and outs[1][0] == 2
    torch.testing.assert_close(outs[1][1], outs[0][1], atol=1e-3, rtol=1e-3)
    rel = ((outs[1][2] - outs[0][2]).norm() / outs[0][2].norm()).item()
    assert rel < 1e-3, rel
