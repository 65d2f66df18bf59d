"""Checkpoint-schema contract (`SURVEY.md` §2.5): key names, shapes, duplicates, param counts."""
import argparse

import torch

from pytorch_raft_amd import RAFT
from pytorch_raft_amd.engine import checkpoint as ckpt


def _model(small):
    return RAFT(argparse.Namespace(small=small, mixed_precision=False))


def test_param_counts():
    assert sum(p.numel() for p in _model(False).parameters()) == 5257536
    assert sum(p.numel() for p in _model(True).parameters()) == 990162


def test_key_counts_and_buffers():
    full = _model(False)
    sd = full.state_dict()
    assert len(sd) == 179
    buffer_keys = [k for k in sd if k.rsplit('.', 1)[-1] in
                   ('running_mean', 'running_var', 'num_batches_tracked')]
    assert len(buffer_keys) == 51
    small = _model(True)
    assert len(small.state_dict()) == 106
    assert len(list(small.buffers())) == 0


def test_duplicate_norm3_downsample_keys():
    sd = _model(False).state_dict()
    for layer in (2, 3):
        for suffix in ('weight', 'bias', 'running_mean', 'running_var', 'num_batches_tracked'):
            a = 'cnet.layer%d.0.norm3.%s' % (layer, suffix)
            b = 'cnet.layer%d.0.downsample.1.%s' % (layer, suffix)
            assert a in sd and b in sd
            assert sd[a].data_ptr() == sd[b].data_ptr()


def test_update_block_shapes_full():
    sd = _model(False).state_dict()
    expect = {
        'update_block.encoder.convc1.weight': (256, 324, 1, 1),
        'update_block.encoder.convc2.weight': (192, 256, 3, 3),
        'update_block.encoder.convf1.weight': (128, 2, 7, 7),
        'update_block.encoder.convf2.weight': (64, 128, 3, 3),
        'update_block.encoder.conv.weight': (126, 256, 3, 3),
        'update_block.gru.convz1.weight': (128, 384, 1, 5),
        'update_block.gru.convq2.weight': (128, 384, 5, 1),
        'update_block.flow_head.conv1.weight': (256, 128, 3, 3),
        'update_block.flow_head.conv2.weight': (2, 256, 3, 3),
        'update_block.mask.0.weight': (256, 128, 3, 3),
        'update_block.mask.2.weight': (576, 256, 1, 1),
    }
    for k, shape in expect.items():
        assert tuple(sd[k].shape) == shape, k


def test_update_block_shapes_small():
    sd = _model(True).state_dict()
    expect = {
        'update_block.encoder.convc1.weight': (96, 196, 1, 1),
        'update_block.encoder.convf1.weight': (64, 2, 7, 7),
        'update_block.encoder.convf2.weight': (32, 64, 3, 3),
        'update_block.encoder.conv.weight': (80, 128, 3, 3),
        'update_block.gru.convz.weight': (96, 242, 3, 3),
        'update_block.flow_head.conv1.weight': (128, 96, 3, 3),
        'update_block.flow_head.conv2.weight': (2, 128, 3, 3),
    }
    for k, shape in expect.items():
        assert tuple(sd[k].shape) == shape, k
    assert not any(k.startswith('update_block.mask') for k in sd)
    assert not any(k.startswith('cnet.norm1') for k in sd)


def test_args_mutation_quirk():
    a = argparse.Namespace(small=False, mixed_precision=False)
    RAFT(a)
    assert a.corr_levels == 4 and a.corr_radius == 4 and a.dropout == 0 and a.alternate_corr is False
    b = argparse.Namespace(small=True, mixed_precision=False)
    RAFT(b)
    assert b.corr_radius == 3


def test_checkpoint_roundtrip_module_prefix(tmp_path):
    m = _model(False)
    path = str(tmp_path / 'raft-test.pth')
    ckpt.save_weights(m, path)
    raw = torch.load(path, weights_only=True)
    assert all(k.startswith('module.') for k in raw)
    assert len(raw) == 179
    m2 = _model(False)
    ckpt.load_weights(m2, path, strict=True)
    for (k, a), b in zip(m.state_dict().items(), m2.state_dict().values()):
        assert torch.equal(a, b), k
    # unprefixed files load too
    torch.save(m.state_dict(), str(tmp_path / 'plain.pth'))
    ckpt.load_weights(m2, str(tmp_path / 'plain.pth'), strict=True)
    # and a DataParallel-wrapped model loads our file strictly, like the reference demos
    dp = torch.nn.DataParallel(_model(False))
    dp.load_state_dict(torch.load(path, weights_only=True), strict=True)
