"""Drop-in for the reference's csa/suffix_array.py.

build_suffix_array(text) (:131-134) returns the suffix array of `text` in
Python str order (no sentinel added), computed on the GPU by hkcsa_build_sa (the
keyed bucket build: cursor partition passes and LDS bucket sorts, tied suffixes
refined in LDS items, prefix doubling for repetitive text).  ksa(T) (:46-129) is the reference's DC3 attempt; it is only correct when
its recursion is not needed (and raises TypeError otherwise),
and whenever it returns it equals build_suffix_array(T) — so the drop-in returns
the suffix array for every input.  Unlike the reference, importing this module
prints nothing (the reference runs a demo at import time, :136-138).
"""
from __future__ import annotations

from hkcsa import DeviceIndex, TextCodec


def _as_str(text) -> str:
    return text if isinstance(text, str) else "".join(text)


def build_suffix_array(text) -> list:
    text = _as_str(text)
    if not text:
        return []
    codec = TextCodec(text)
    dev = DeviceIndex.from_parts(codec.parts(text))
    try:
        dev.build_sa()
        return [int(x) for x in dev.sa()]
    finally:
        dev.close()


def ksa(T) -> list:
    return build_suffix_array(T)
