"""HIP operator wrappers (autograd Functions) + pure-torch oracles."""
from . import _ext
