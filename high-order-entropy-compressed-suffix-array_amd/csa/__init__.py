"""Reference-compatible surface of the H_k-CSA (drop-in for the reference's `csa`).

Modules mirror the reference's paths: csa.suffix_array, csa.bwt,
csa.wavelet_tree, csa.enhanced_fm_index, csa.csa.  Everything computes on the
GPU through libhkcsa.so; there is no CPU fallback.
"""
from .csa import CSA, CompressedSuffixArray  # noqa: F401
from .enhanced_fm_index import EnhancedFMIndex  # noqa: F401

__all__ = ["CSA", "CompressedSuffixArray", "EnhancedFMIndex"]
