"""Drop-in for the reference's csa/bwt.py:3-13 (bwt_transform).

bwt[i] = text[sa[i] - 1], with sa[i] == 0 wrapping to the last symbol — one
gather kernel over the suffix array on the GPU (hkcsa_bwt_gather).
"""
from __future__ import annotations

from hkcsa import TextCodec, bwt_gather


def bwt_transform(text, suffix_array) -> str:
    text = text if isinstance(text, str) else "".join(text)
    if not text:
        return ""
    sa = list(suffix_array)
    if len(sa) < len(text):
        raise IndexError("list index out of range")
    codec = TextCodec(text)
    return codec.decode(bwt_gather(codec.encode_text(text), sa[:len(text)]))
