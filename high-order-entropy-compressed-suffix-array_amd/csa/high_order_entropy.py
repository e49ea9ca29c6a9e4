"""Drop-in for the reference's csa/high_order_entropy.py:4-32 (calculate_high_order_entropy).

The k-th order empirical entropy is computed on the GPU (hkcsa_entropy): H_0 from the byte
histogram; for k > 0, contexts are runs of the suffix array, so
    n·H_k = sum_w n_w log2 n_w - sum_(w,c) n_wc log2 n_wc
needs only two run-length reductions over the SA of the text.  Same edge cases as the
reference: empty text or k < 0 -> 0, n <= k -> 0, the sum is divided by n (not n - k).
Results agree with the reference to floating-point rounding (different summation order).
"""
from __future__ import annotations

from hkcsa import DeviceIndex, TextCodec


def calculate_high_order_entropy(text, k):
    """Calculate k-th order empirical entropy."""
    if not text or k < 0:
        return 0
    if not isinstance(text, str):
        text = "".join(text)
    codec = TextCodec(text)
    dev = DeviceIndex.from_parts(codec.parts(text))
    try:
        return dev.entropy(int(k))
    finally:
        dev.close()
