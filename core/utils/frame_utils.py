"""Compat shim for reference `core/utils/frame_utils.py`."""
import os
import sys
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
from pytorch_raft_amd.utils.frame_utils import (  # noqa: F401,E402
    TAG_CHAR, readFlow, writeFlow, readPFM, writePFM, readFlowKITTI, readDispKITTI, writeFlowKITTI,
    read_gen)
