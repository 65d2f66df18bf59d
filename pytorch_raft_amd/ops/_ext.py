"""Loader for the in-tree native extension ``pytorch_raft_amd/_C.so``.

The extension registers its operators with ``TORCH_LIBRARY(raft_amd, ...)`` so they are reachable
as ``torch.ops.raft_amd.<name>``.  It is built by ``python -m pytorch_raft_amd.build`` (also run by
``__graft_entry__.build()``) with ``hipcc --offload-arch=gfx950``.

Policy: on a machine that has a GPU the HIP path is *the* path -- if the extension is missing or
fails to load we raise instead of silently falling back to PyTorch (set ``RAFT_AMD_ALLOW_FALLBACK=1``
to opt out, e.g. for debugging).  On CPU-only machines the pure-PyTorch path is used.
"""
import os
import threading

import torch

_LOCK = threading.Lock()
_STATE = {'loaded': None, 'error': None}
_PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(_PKG_DIR, '_C.so')


def _try_load():
    with _LOCK:
        if _STATE['loaded'] is not None:
            return _STATE['loaded']
        if not os.path.exists(LIB_PATH):
            _STATE['loaded'] = False
            _STATE['error'] = 'native extension not built: %s (run python -m pytorch_raft_amd.build)' % LIB_PATH
            return False
        try:
            torch.ops.load_library(LIB_PATH)
            _STATE['loaded'] = True
        except Exception as e:  # pragma: no cover - depends on the build
            _STATE['loaded'] = False
            _STATE['error'] = 'failed to load %s: %r' % (LIB_PATH, e)
        return _STATE['loaded']


def loaded():
    return _try_load()


def load_error():
    _try_load()
    return _STATE['error']


def fallback_allowed():
    return os.environ.get('RAFT_AMD_ALLOW_FALLBACK', '0') == '1'


def require():
    """Return ``torch.ops.raft_amd`` or raise loudly."""
    if not _try_load():
        raise RuntimeError('pytorch_raft_amd HIP extension unavailable: %s' % _STATE['error'])
    return torch.ops.raft_amd


def gpu_path_enabled(required=False):
    """True if GPU tensors should run through the HIP kernels.

    ``required`` forces an error when the extension is missing.  Without it a missing extension on
    a GPU machine still raises unless RAFT_AMD_ALLOW_FALLBACK=1.
    """
    if _try_load():
        return True
    if required or not fallback_allowed():
        raise RuntimeError('pytorch_raft_amd HIP extension unavailable on a GPU tensor: %s'
                           % _STATE['error'])
    return False


def ops():
    return require()
