"""hkcsa — MI355X-native H_k-CSA construction and query engine (host side).

The compute lives in libhkcsa.so (hand-written HIP kernels for gfx950, built from
../csrc); this package is the thin ctypes host layer.  The reference-compatible
class surface is the sibling package `csa` (and `utils`).
"""
from ._native import HkcsaError, device_count, load, LIB_PATH, EXPORTED  # noqa: F401
from .codec import TextCodec  # noqa: F401
from .index import DeviceIndex, QuerySet, pack_patterns, bwt_gather, comm_unique_id  # noqa: F401

__all__ = ["HkcsaError", "DeviceIndex", "QuerySet", "TextCodec", "pack_patterns", "bwt_gather",
           "comm_unique_id", "device_count", "load", "LIB_PATH", "EXPORTED"]
