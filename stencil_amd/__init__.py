"""stencil_amd -- MI355X-native iterative Jacobi stencil engine.

The compute path is libstencil_hip.so (hand-written gfx950 HIP kernels behind
the C-ABI in include/stencil_hip.h).  Python provides the device-memory,
stream and torch.distributed plumbing around it: `engine` (one GPU) and
`slab` (Z-slab decomposition with halo exchange, one process per GPU).
"""
from . import _lib  # noqa: F401

__all__ = ["_lib"]
