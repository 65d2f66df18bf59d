"""Compat shim for reference `core/utils/utils.py`."""
import os
import sys
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
from pytorch_raft_amd.utils.utils import (  # noqa: F401,E402
    InputPadder, forward_interpolate, bilinear_sampler, coords_grid, upflow8)
