"""Compat shim for reference `core/utils/flow_viz.py`."""
import os
import sys
_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
from pytorch_raft_amd.utils.flow_viz import make_colorwheel, flow_uv_to_colors, flow_to_image  # noqa: F401,E402
