"""Compat shim for reference `core/datasets.py`."""
import _bootstrap  # noqa: F401
from pytorch_raft_amd.data.datasets import (  # noqa: F401
    FlowDataset, MpiSintel, FlyingChairs, FlyingThings3D, KITTI, HD1K, fetch_dataloader)
