"""CPU checks of the one-gather weight packing (fused update block) and the batched encoder
weight cast: both must equal the per-layer reference formulation exactly."""
import argparse

import torch
import torch.nn as nn

from pytorch_raft_amd import RAFT
from pytorch_raft_amd.ops import conv as C
from pytorch_raft_amd.ops import update_hip as U
from pytorch_raft_amd.ops.encoder import cast_conv_weights


def _ub():
    torch.manual_seed(0)
    return RAFT(argparse.Namespace(small=False, mixed_precision=True)).update_block


def test_pack_plan_matches_direct_packing():
    ub = _ub()
    params = U.flat_params(ub)
    pk = U._Packed(ub, params, torch.device('cpu'), need_grad=True)
    with torch.no_grad():
        w, wd, b, x = U._pack_layers(U.module_params(ub), True, torch.bfloat16)
    for name in w:
        assert torch.equal(pk.w[name], w[name]), name
        assert torch.equal(pk.b[name], b[name].float()), name
        assert pk.kpad[name] == w[name].shape[1]
    assert set(pk.wd) == set(wd)
    for name in wd:
        assert torch.equal(pk.wd[name], wd[name]), name
    fw = ub.flow_head.conv2.weight.detach().to(torch.bfloat16)
    assert torch.equal(pk.fh2_wf.reshape(3, 3, 2, 256), fw.permute(2, 3, 0, 1))
    assert torch.equal(pk.fh2_wd.reshape(3, 3, 256, 2), fw.permute(2, 3, 1, 0))
    assert pk.fh2_wf.data_ptr() % 16 == 0 and pk.fh2_wd.data_ptr() % 16 == 0


def test_unpack_grads_matches_per_layer_unpack():
    ub = _ub()
    params = U.flat_params(ub)
    pk = U._Packed(ub, params, torch.device('cpu'), need_grad=True)
    g = torch.Generator().manual_seed(1)
    pk.dwflat.copy_(torch.randn(pk.dwflat.shape, generator=g))
    # per spec: module-layout gradient of the input channels it owns (in_sel), bias if it has one
    parts = {}
    for s in U.SPECS:
        dw, db = pk.dw[s.name] * s.scale, pk.db[s.name] * s.scale
        if s.small:
            wg = C.unpack_weight_grad_small(dw, s.cout, s.in_real[0], s.k)
        else:
            wg = C.unpack_weight_grad(dw, s.cout, s.in_real, s.in_pad, s.k)
        base = s.name[:-1] if s.name.endswith('i') else s.name
        sel = s.in_sel or [(0, wg.shape[1])]
        full = parts.setdefault(base, [None, None])
        if full[0] is None:  # split GRU convs: module weight over [h | inp | mf] = 384
            full[0] = torch.zeros(s.cout, 3 * U.HD if s.in_sel else wg.shape[1], *s.k)
        off = 0
        for a, n in sel:
            full[0][:, a:a + n] = wg[:, off:off + n]
            off += n
        if not s.no_bias:
            full[1] = db
    ref = []
    for s in U.SPECS:
        if s.name not in parts:
            continue
        wg, db = parts[s.name]
        if s.name in ('zr1', 'zr2', 'head'):
            h = s.cout // 2
            ref += [wg[:h], db[:h], wg[h:], db[h:]]
        else:
            ref += [wg, db]
    got = U._unpack_grads(pk)
    assert len(got) == len(ref) == len(params)
    for a, r, p in zip(got, ref, params):
        assert a.shape == p.shape
        assert torch.equal(a, r)


def test_batched_encoder_weight_cast():
    convs = [nn.Conv2d(3, 8, 7), nn.Conv2d(8, 16, 1), nn.Conv2d(16, 4, 3),
             nn.Conv2d(64, 128, 3, padding=1), nn.Conv2d(96, 96, 3, padding=1)]
    m, adj, fwd = cast_conv_weights(convs)
    for c in convs:
        w = m[c]
        assert w.is_contiguous(memory_format=torch.channels_last)
        assert torch.equal(w.float(), c.weight.to(torch.bfloat16).float())
    # the adjoint (input-gradient) weight of the native 3x3 convs: W'[c][tap'][o] = W[o][c][flip],
    # K slots of 64-multiples (zeros past Cout); a padded forward pack where Cin % 64 != 0
    assert list(adj) == [convs[3], convs[4]] and list(fwd) == [convs[4]]
    w = convs[3].weight.to(torch.bfloat16)
    ref = w.flip(2, 3).permute(1, 2, 3, 0).reshape(64, 9 * 128)
    assert torch.equal(adj[convs[3]], ref) and not adj[convs[3]].requires_grad
    w = convs[4].weight.to(torch.bfloat16)
    ref = torch.nn.functional.pad(w.flip(2, 3).permute(1, 2, 3, 0), (0, 32)).reshape(96, 9 * 128)
    assert torch.equal(adj[convs[4]], ref)
    ref = torch.nn.functional.pad(w.permute(0, 2, 3, 1), (0, 32)).reshape(96, 9 * 128)
    assert torch.equal(fwd[convs[4]], ref)
    loss = sum((m[c].float() ** 2).sum() * (i + 1) for i, c in enumerate(convs))
    loss.backward()
    for i, c in enumerate(convs):
        ref = 2 * (i + 1) * c.weight.to(torch.bfloat16).float()
        torch.testing.assert_close(c.weight.grad, ref, rtol=1e-2, atol=1e-3)


def test_fp32_prepack_matches_per_conv_split_packs():
    """conv_fp32.prepack (one gather over all convs, residual halves from the same sources) lays
    out exactly the [w_hi | w_hi | w_lo] forward and adjoint packs _pack3 builds per conv."""
    from pytorch_raft_amd.ops import conv_fp32
    g = torch.Generator().manual_seed(0)
    ws = [torch.randn(s, generator=g) for s in [(64, 64, 3, 3), (96, 64, 3, 3), (128, 96, 3, 3),
                                                 (96, 96, 1, 1)]]
    with conv_fp32.enabled(True):
        conv_fp32.prepack([(w, w) for w in ws])
        cache = conv_fp32._ACTIVE['packed']
        for w in ws:
            co, ci = w.shape[:2]
            fwd = conv_fp32._pack3(w, C.round_up(ci, 64))
            adj = conv_fp32._pack3(w.flip(2, 3).transpose(0, 1).contiguous(), C.round_up(co, 64))
            assert torch.equal(cache[(w.data_ptr(), w._version, tuple(w.shape), C.round_up(ci, 64), False)], fwd)
            assert torch.equal(cache[(w.data_ptr(), w._version, tuple(w.shape), C.round_up(co, 64), True)], adj)


def test_split_pack_plan_matches_split_weight():
    """fp32 schedule: the one-gather split packs equal the fp32 packs run through
    C.split_weight ([w_hi | w_hi | w_lo] per tap) view by view."""
    ub = _ub()
    params = U.flat_params(ub)
    pk = U._Packed(ub, params, torch.device('cpu'), need_grad=True, dtype=torch.float32)
    with torch.no_grad():
        w, wd, b, x = U._pack_layers(U.module_params(ub), True, torch.float32, spl=True)
    for kind, d, ref in (('w', pk.w, w), ('wd', pk.wd, wd)):
        assert set(d) == set(ref), kind
        for name in ref:
            exp = C.split_weight(ref[name], U._taps_of(U.FULL, kind, name))
            assert torch.equal(d[name], exp), (kind, name)
    for name in ('zrq1', 'zrq2'):
        assert torch.equal(pk.x[name], C.split_weight(x[name], U._taps_of(U.FULL, 'x', name))), name
    assert torch.equal(pk.x['fh2f'], x['fh2f'].to(torch.bfloat16))
