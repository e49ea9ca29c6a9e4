"""Python front of the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
module, and only as the checker.  The product (the `csa` package over
libhkcsa.so) never imports it.

Two restatements of the reference live here:
  * liboracle.so (hkcsa_oracle.c): C versions of build_suffix_array, bwt_transform,
    build_count, occ/rank and find_range, an O(n) SA checker, the full levelwise
    wavelet tree, the synthetic-text generator and the shard partition;
  * ref_port.py: pure-Python loops that follow the reference line by line, for
    small inputs and for the timed CPU baseline.
Both are pinned to the golden vectors generated from the reference itself
(tests/golden/make_golden.py) by tests/test_oracle.py.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        L = C.CDLL(LIB)
        vp, u64 = C.c_void_p, C.c_uint64
        L.oracle_suffix_array.argtypes = [vp, u64, vp]
        L.oracle_bwt.argtypes = [vp, u64, vp, vp]
        L.oracle_count.argtypes = [vp, u64, vp]
        L.oracle_occ_new.argtypes = [vp, u64]
        L.oracle_occ_new.restype = vp
        L.oracle_occ_free.argtypes = [vp]
        L.oracle_occ.argtypes = [vp, C.c_uint8, u64]
        L.oracle_occ.restype = u64
        L.oracle_find_range.argtypes = [vp, vp, vp, vp, vp, u64, vp]
        L.oracle_check_sa.argtypes = [vp, u64, vp]
        L.oracle_check_sa.restype = u64
        L.oracle_synth_text.argtypes = [u64, vp, C.c_int, u64, C.c_uint8, vp]
        L.oracle_wt_levels.argtypes = [vp, u64, vp]
        L.oracle_wt_levels.restype = C.c_int
        L.oracle_shard_hist.argtypes = [vp, u64, u64, u64, vp]
        L.oracle_shard_below.argtypes = [vp, u64, u64, u64, vp, C.c_int, vp]
        L.oracle_shard_scheme.argtypes = [vp, u64, vp, vp, vp]
        L.oracle_shard_scheme.restype = C.c_int
        L.oracle_key_geometry.argtypes = [vp, u64, vp, vp, vp, vp, vp]
        L.oracle_golomb.argtypes = [vp, u64, C.c_uint32, vp]
        L.oracle_golomb.restype = u64
        _lib = L
    return _lib


def _u8(a) -> np.ndarray:
    if isinstance(a, (bytes, bytearray)):
        return np.frombuffer(bytes(a), dtype=np.uint8)
    return np.ascontiguousarray(a, dtype=np.uint8)


def _p(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def suffix_array(t) -> np.ndarray:
    t = _u8(t)
    sa = np.empty(len(t), dtype=np.uint64)
    lib().oracle_suffix_array(_p(t), len(t), _p(sa))
    return sa


def bwt(t, sa) -> np.ndarray:
    t = _u8(t)
    sa = np.ascontiguousarray(sa, dtype=np.uint64)
    out = np.empty(len(t), dtype=np.uint8)
    lib().oracle_bwt(_p(t), len(t), _p(sa), _p(out))
    return out


def count_array(t) -> np.ndarray:
    t = _u8(t)
    Cv = np.empty(257, dtype=np.uint64)
    lib().oracle_count(_p(t), len(t), _p(Cv))
    return Cv


def check_sa(t, sa) -> int:
    """0 if `sa` is the suffix array of `t`, else 1 + first offending index."""
    t = _u8(t)
    sa = np.ascontiguousarray(sa, dtype=np.uint64)
    if len(sa) != len(t):
        return 1
    return int(lib().oracle_check_sa(_p(t), len(t), _p(sa)))


def synth_text(n: int, alphabet: bytes, seed: int, terminator: int = ord("$")) -> np.ndarray:
    a = _u8(alphabet)
    out = np.empty(n, dtype=np.uint8)
    lib().oracle_synth_text(n, _p(a), len(a), seed, terminator, _p(out))
    return out


def wt_levels(seq) -> np.ndarray:
    """(L, n) uint8 bit matrix of the full levelwise wavelet tree."""
    s = _u8(seq)
    bits = np.zeros((8, max(1, len(s))), dtype=np.uint8)
    L = lib().oracle_wt_levels(_p(s), len(s), _p(bits))
    return bits[:L, :len(s)].copy()


def shard_scheme(t) -> int:
    """lb of the keyed coarse partition (exact 16-bit sym-prefix histogram), 0: the sampled key."""
    t = _u8(t)
    dig = np.zeros(256, dtype=np.uint16)
    ut, mt = C.c_int(0), C.c_int(0)
    return int(lib().oracle_shard_scheme(_p(t) if len(t) else None, len(t), _p(dig), C.byref(ut), C.byref(mt)))


def shard_hist(t, lo: int, hi: int) -> np.ndarray:
    """The sharded build's partition histogram of [lo, hi) (65536 bins; see oracle_shard_hist)."""
    t = _u8(t)
    h = np.zeros(65536, dtype=np.uint64)
    lib().oracle_shard_hist(_p(t), len(t), lo, hi, _p(h))
    return h


def shard_below(t, lo: int, hi: int, splitters) -> np.ndarray:
    """#positions p in [lo, hi) whose partition bucket is below each splitter."""
    t = _u8(t)
    B = np.ascontiguousarray(splitters, dtype=np.uint32)
    out = np.zeros(len(B), dtype=np.uint64)
    lib().oracle_shard_below(_p(t), len(t), lo, hi, _p(B), len(B), _p(out))
    return out


def key_geometry(t) -> tuple[int, int, int, int]:
    """(q, pb, radix, key_bits) the build chooses for text t."""
    t = _u8(t)
    q, pb, kb = C.c_int(0), C.c_int(0), C.c_int(0)
    R = C.c_uint64(0)
    code = np.zeros(256, dtype=np.uint16)
    lib().oracle_key_geometry(_p(t), len(t), C.byref(q), C.byref(pb), C.byref(R), C.byref(kb), _p(code))
    return q.value, pb.value, R.value, kb.value


def golomb_m(ones: int, total: int) -> int:
    """csa/wavelet_tree.py:32-38 (Python float arithmetic, as the reference)."""
    import math
    if ones == 0:
        return 1
    return max(1, int(math.log2(1 / (ones / total))))


def golomb(bits, m: int | None = None) -> tuple[int, np.ndarray]:
    """(m, code bits) of GolombRiceEncoder(bits).encode(bits) (csa/wavelet_tree.py:27-63)."""
    b = np.ascontiguousarray(bits, dtype=np.uint8)
    if m is None:
        m = golomb_m(int(b.sum()), int(b.size))
    nb = lib().oracle_golomb(_p(b) if b.size else None, b.size, m, None)
    out = np.zeros(max(1, nb), dtype=np.uint8)
    lib().oracle_golomb(_p(b) if b.size else None, b.size, m, _p(out))
    return m, out[:nb]


def entropy(t, k: int) -> float:
    """Empirical H_k (csa/high_order_entropy.py:4-32) by numpy k-mer counting: (k+1)-grams packed
    base sigma into int64 (needs (k+1)·log2(sigma) < 63), counted with np.unique."""
    import math
    t = _u8(t)
    n = len(t)
    if n == 0 or k < 0:
        return 0.0
    syms, codes = np.unique(t, return_inverse=True)
    if k == 0:
        c = np.bincount(codes).astype(np.float64)
        p = c / n
        return float(-(p * np.log2(p)).sum())
    if n <= k:
        return 0.0
    sig = max(2, len(syms))
    if (k + 1) * math.log2(sig) >= 62:
        raise ValueError("context too long for the packed oracle")
    m = n - k
    ctx = np.zeros(m, dtype=np.int64)
    for j in range(k):
        ctx = ctx * sig + codes[j:j + m]
    pair = ctx * sig + codes[k:k + m]
    _, cw = np.unique(ctx, return_counts=True)
    _, cp = np.unique(pair, return_counts=True)
    cw = cw.astype(np.float64)
    cp = cp.astype(np.float64)
    return float(((cw * np.log2(cw)).sum() - (cp * np.log2(cp)).sum()) / n)


class FM:
    """Backward search over T' with the oracle's occ table (csa/enhanced_fm_index.py)."""

    def __init__(self, tp, sa=None):
        self.t = _u8(tp).copy()
        self.n = len(self.t)
        self.sa = suffix_array(self.t) if sa is None else np.ascontiguousarray(sa, dtype=np.uint64)
        self.bwt = bwt(self.t, self.sa)
        self.C = count_array(self.t)
        self.present = np.zeros(256, dtype=np.uint8)
        self.present[np.unique(self.t)] = 1
        self._occ = lib().oracle_occ_new(_p(self.bwt), self.n)

    def __del__(self):
        if getattr(self, "_occ", None):
            lib().oracle_occ_free(self._occ)
            self._occ = None

    def rank(self, c: int, i: int) -> int:
        if not self.present[c]:
            return 0
        return int(lib().oracle_occ(self._occ, c, i))

    def find_range(self, pats: list[bytes]) -> np.ndarray:
        data = np.frombuffer(b"".join(pats), dtype=np.uint8) if pats else np.zeros(0, np.uint8)
        data = np.ascontiguousarray(data)
        offs = np.zeros(len(pats) + 1, dtype=np.uint64)
        offs[1:] = np.cumsum([len(p) for p in pats]) if pats else []
        lr = np.empty(2 * len(pats), dtype=np.int64)
        if len(data) == 0:
            data = np.zeros(1, np.uint8)
        lib().oracle_find_range(self._occ, _p(self.C), _p(self.present), _p(data), _p(offs), len(pats), _p(lr))
        return lr.reshape(-1, 2)

    def find(self, pats: list[bytes]) -> list[list[int]]:
        lr = self.find_range(pats)
        return [[] if l < 0 else [int(x) for x in self.sa[l:r + 1]] for l, r in lr]
