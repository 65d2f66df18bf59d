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
SUM_MAX = 32  # summands per sum_bf16_ launch (RAFT_SUM_MAX in csrc/kernels/launchers.h)


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
        if _STATE['loaded']:
            _STATE['tune_rows'] = load_conv_tune_db()
        return _STATE['loaded']


# ---------------------------------------------------------------------------------------------
# Persisted conv tile table.  The implicit-GEMM convs pick a tile config per geometry by timing
# every candidate once per process (conv_igemm.hip: autotune).  Isolated timings of near-tied
# candidates flip from box to box, so the step time did too.  A checked-in table of picks
# (tune_db/conv_gfx950.txt: one row of 13 ints per key -- P H W KH KW cin cout small eclass cfg
# bm bn creal, as conv_tune_table() returns them) is imported when the library loads; the
# autotuner then runs only for keys the table lacks.  RAFT_CONV_TUNE_DB=<path> picks another
# table, RAFT_CONV_TUNE_DB=0 disables it.
TUNE_DB = os.path.join(_PKG_DIR, 'tune_db', 'conv_gfx950.txt')


def tune_db_path():
    p = os.environ.get('RAFT_CONV_TUNE_DB', TUNE_DB)
    return None if p in ('', '0') else p


def read_tune_rows(path):
    rows = []
    with open(path) as f:
        for line in f:
            line = line.split('#', 1)[0].strip()
            if not line:
                continue
            r = [int(x) for x in line.split()]
            if len(r) != 13:
                raise ValueError('%s: tune row of %d ints (13 expected): %r' % (path, len(r), line))
            rows.append(r)
    return rows


def load_conv_tune_db(path=None):
    """Import the persisted conv tile picks into the native cache; returns the rows imported."""
    path = path or tune_db_path()
    if not path or not os.path.exists(path):
        return 0
    rows = read_tune_rows(path)
    if not rows:
        return 0
    flat = [v for r in rows for v in r]
    return int(torch.ops.raft_amd.conv_tune_import(flat))


def dump_conv_tune_db(path, merge=True):
    """Write this process's conv tile table (imported rows + fresh autotune picks) to ``path``;
    with ``merge`` the rows already in ``path`` whose keys this process did not touch are kept."""
    rows = list(torch.ops.raft_amd.conv_tune_table())
    new = [rows[i:i + 13] for i in range(0, len(rows), 13)]
    key = lambda r: tuple(r[:9]) + (r[12],)  # noqa: E731
    table = {}
    if merge and os.path.exists(path):
        for r in read_tune_rows(path):
            table[key(r)] = r
    for r in new:
        table[key(r)] = r
    d = os.path.dirname(path)
    if d:
        os.makedirs(d, exist_ok=True)
    with open(path, 'w') as f:
        f.write('# conv tile picks for gfx950 (pytorch_raft_amd/ops/_ext.py: load_conv_tune_db)\n')
        f.write('# P H W KH KW cin cout small eclass cfg bm bn creal\n')
        for k in sorted(table):
            f.write(' '.join(str(v) for v in table[k]) + '\n')
    return len(table)


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
    if _DRY['on']:
        return True
    if _try_load():
        return True
    if required or not fallback_allowed():
        raise RuntimeError('pytorch_raft_amd HIP extension unavailable on a GPU tensor: %s'
                           % _STATE['error'])
    return False


def ops():
    if _DRY['on']:
        return _DRY['ops']
    return require()


def device_ok(t):
    """True if ``t`` should take the HIP path (a GPU tensor, or any tensor during a dry run)."""
    return bool(t.is_cuda) or _DRY['on']


# ---------------------------------------------------------------------------------------------
# Dry run: execute the full HIP-path orchestration on CPU with every native op replaced by a
# schema-checking stub (arguments are validated against the registered TORCH_LIBRARY schema; ops
# that return tensors return zeros of the right shape).  Used by the CPU test-suite to catch
# Python-side bugs of GPU-only code paths without a GPU.
_DRY = {'on': False, 'ops': None}


class _DryOps:
    def __init__(self, returns):
        torch.ops.load_library(LIB_PATH)
        self._returns = returns
        self.calls = []

    def __getattr__(self, name):
        op = getattr(torch.ops.raft_amd, name)
        schema = op.default._schema

        def call(*args):
            params = list(schema.arguments)
            required = [p for p in params if not p.has_default_value()]
            if not (len(required) <= len(args) <= len(params)):
                raise TypeError('%s: %d args for schema %s' % (name, len(args), schema))
            for p, v in zip(params, args):
                t = str(p.type)
                ok = True
                if t == 'Tensor':
                    ok = isinstance(v, torch.Tensor)
                elif t == 'Optional[Tensor]' or t == 'Tensor?':
                    ok = v is None or isinstance(v, torch.Tensor)
                elif t in ('List[Tensor]', 'Tensor[]'):
                    ok = isinstance(v, (list, tuple)) and all(isinstance(x, torch.Tensor) for x in v)
                elif t == 'int':
                    ok = isinstance(v, int) and not isinstance(v, bool)
                elif t == 'float':
                    ok = isinstance(v, (int, float)) and not isinstance(v, bool)
                elif t in ('List[int]', 'int[]'):
                    ok = isinstance(v, (list, tuple)) and all(isinstance(x, int) for x in v)
                elif t == 'bool':
                    ok = isinstance(v, bool)
                if not ok:
                    raise TypeError('%s: argument %s expects %s, got %r' % (name, p.name, t, type(v)))
            self.calls.append(name)
            fn = self._returns.get(name)
            return fn(*args) if fn is not None else None
        return call


class dry_run:
    """Context manager enabling the dry run (see above)."""

    def __init__(self, returns):
        self.returns = returns

    def __enter__(self):
        _DRY['ops'] = _DryOps(self.returns)
        _DRY['on'] = True
        return _DRY['ops']

    def __exit__(self, *a):
        _DRY['on'] = False
        _DRY['ops'] = None
        return False
