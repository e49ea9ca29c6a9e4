"""Drop-in for the reference's utils/utils.py.

build_count (:16-24) is a GPU byte histogram + scan (hkcsa_get_C); build_occ
(:26-32) returns a lazy {symbol: occ column} mapping backed by a GPU wavelet tree
over `bwt` instead of materialising O(n * sigma) Python ints.
"""
from __future__ import annotations

import time

from hkcsa import DeviceIndex, TextCodec


def time_function(func):
    """utils/utils.py:4-14: wrap `func` to return (result, seconds)."""
    def wrapper(*args, **kwargs):
        t0 = time.time()
        result = func(*args, **kwargs)
        return result, time.time() - t0
    return wrapper


def _as_str(text) -> str:
    return text if isinstance(text, str) else "".join(text)


def build_count(text) -> dict:
    text = _as_str(text)
    if not text:
        return {}
    codec = TextCodec(text)
    dev = DeviceIndex.from_parts(codec.parts(text))
    try:
        C = dev.C()
        return {codec.decode(bytes([b])): int(C[b]) for b in dev.alphabet()}
    finally:
        dev.close()


def build_occ(bwt):
    from csa.enhanced_fm_index import OccView
    bwt = _as_str(bwt)
    if not bwt:
        return {}
    codec = TextCodec(bwt)
    dev = DeviceIndex.from_parts(codec.parts(bwt))
    dev.use_text_as_bwt()
    dev.build_wt()
    return OccView(dev, codec, len(bwt))
