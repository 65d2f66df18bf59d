"""Compat shim for reference `core/extractor.py`."""
import _bootstrap  # noqa: F401
from pytorch_raft_amd.models.extractor import (  # noqa: F401
    ResidualBlock, BottleneckBlock, BasicEncoder, SmallEncoder)
