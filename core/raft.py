"""Compat shim: `sys.path.append('core'); from raft import RAFT` (reference `core/raft.py`)."""
import _bootstrap  # noqa: F401
from pytorch_raft_amd.models.raft import RAFT  # noqa: F401
from pytorch_raft_amd.utils.utils import bilinear_sampler, coords_grid, upflow8  # noqa: F401
