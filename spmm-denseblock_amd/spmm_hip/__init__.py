"""spmm_hip — Python mirror of the MI355X-native SpMM engine's C ABI.

Importing this package does not touch the GPU. ``prep`` (host preprocessing
and data feeders) works without a GPU; ``ops`` needs a HIP device; ``dist``
adds the row-partitioned multi-GPU path over torch.distributed (RCCL).
"""
from . import _lib, prep  # noqa: F401
from ._lib import SpmmError, lib  # noqa: F401

__version__ = "1.0.0"
