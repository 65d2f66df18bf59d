"""Compat shim for reference `core/utils/augmentor.py`."""
import os
import sys
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
from pytorch_raft_amd.data.augmentor import FlowAugmentor, SparseFlowAugmentor, ColorJitter  # noqa: F401,E402
