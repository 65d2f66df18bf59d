"""Checkpoint IO, compatible with the reference ``raft-*.pth`` files (`SURVEY.md` §2.5).

* Weights file: ``torch.save(state_dict)`` with every key prefixed ``module.`` (the reference saves the
  ``nn.DataParallel`` wrapper, `train.py:187,212`); the duplicate ``norm3`` / ``downsample.1`` keys are
  produced naturally by the model.  Written by rank 0 only.
* Loading accepts prefixed or unprefixed keys, strict or not, and only ever uses
  ``torch.load(weights_only=True)``.
* Optional resume sidecar ``<name>.state.pth`` (optimizer, scheduler, scaler, step, RNG) -- the reference
  has no true resume.  Written atomically (tmp + rename).
"""
import os

import torch

PREFIX = 'module.'


def to_reference_keys(state_dict):
    return {(k if k.startswith(PREFIX) else PREFIX + k): v for k, v in state_dict.items()}


def strip_prefix(state_dict):
    return {(k[len(PREFIX):] if k.startswith(PREFIX) else k): v for k, v in state_dict.items()}


def unwrap(model):
    return model.module if hasattr(model, 'module') else model


def _atomic_save(obj, path):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    tmp = path + '.tmp'
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_weights(model, path):
    sd = {k: v.detach().cpu() for k, v in unwrap(model).state_dict().items()}
    _atomic_save(to_reference_keys(sd), path)
    return path


def load_weights(model, path, strict=True, map_location='cpu'):
    sd = torch.load(path, map_location=map_location, weights_only=True)
    if isinstance(sd, dict) and 'state_dict' in sd and isinstance(sd['state_dict'], dict):
        sd = sd['state_dict']
    return unwrap(model).load_state_dict(strip_prefix(sd), strict=strict)


def sidecar_path(path):
    return path[:-4] + '.state.pth' if path.endswith('.pth') else path + '.state.pth'


def save_training_state(path, optimizer, scheduler, step, scaler=None, extra=None):
    state = {
        'optimizer': optimizer.state_dict(),
        'scheduler': scheduler.state_dict() if scheduler is not None else None,
        'scaler': scaler.state_dict() if scaler is not None else None,
        'step': int(step),
        'rng_cpu': torch.get_rng_state(),
        'rng_cuda': torch.cuda.get_rng_state_all() if torch.cuda.is_available() else None,
        'extra': extra or {},
    }
    _atomic_save(state, sidecar_path(path))


def load_training_state(path, optimizer, scheduler=None, scaler=None):
    sp = sidecar_path(path)
    if not os.path.exists(sp):
        return None
    st = torch.load(sp, map_location='cpu', weights_only=True)
    optimizer.load_state_dict(st['optimizer'])
    if scheduler is not None and st.get('scheduler') is not None:
        scheduler.load_state_dict(st['scheduler'])
    if scaler is not None and st.get('scaler') is not None:
        scaler.load_state_dict(st['scaler'])
    if st.get('rng_cpu') is not None:
        torch.set_rng_state(st['rng_cpu'])
    if st.get('rng_cuda') is not None and torch.cuda.is_available():
        try:
            torch.cuda.set_rng_state_all(st['rng_cuda'])
        except Exception:
            pass
    return st
