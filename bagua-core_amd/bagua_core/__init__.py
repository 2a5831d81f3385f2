"""bagua_core — MI355X-native drop-in for bagua-core's Python module.

Exports the four classes of the reference module (bagua-core-py/src/lib.rs:506-509)
plus `show_version`.  All compute runs in gfx950 HIP kernels
(libbagua_kernels.so) and all collectives in RCCL via the C++ host runtime
(libbagua_core.so); importing fails if those in-tree libraries are missing.
"""
from . import _native
from .backend import BaguaCommBackendPy
from .bucket import BaguaBucketPy
from .communicator import BaguaSingleCommunicatorPy
from .tensor import METHODS, BaguaTensorPy

__version__ = "0.1.0+mi355x"

__all__ = ["BaguaCommBackendPy", "BaguaBucketPy", "BaguaSingleCommunicatorPy", "BaguaTensorPy", "METHODS",
           "show_version"]


def show_version() -> None:
    """bagua-core-internal/src/lib.rs:103-123"""
    import sys
    import torch
    print(f"project_name: bagua-core (MI355X)\nversion: {__version__}\n"
          f"kernels: {_native.KERNELS_PATH}\ncore: {_native.CORE_PATH}\n"
          f"torch: {torch.__version__} hip {torch.version.hip}", file=sys.stderr)
