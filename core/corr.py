"""Compat shim for reference `core/corr.py`."""
import _bootstrap  # noqa: F401
from pytorch_raft_amd.models.corr import CorrBlock, AlternateCorrBlock  # noqa: F401
