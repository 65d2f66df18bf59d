"""Compat shim for reference `core/update.py`."""
import _bootstrap  # noqa: F401
from pytorch_raft_amd.models.update import (  # noqa: F401
    FlowHead, ConvGRU, SepConvGRU, SmallMotionEncoder, BasicMotionEncoder, SmallUpdateBlock,
    BasicUpdateBlock)
