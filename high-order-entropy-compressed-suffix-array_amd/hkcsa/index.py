"""DeviceIndex — Python handle over one hkcsa_index (libhkcsa.so).

All arrays returned are numpy; all compute happens in the HIP kernels behind
the C-ABI (include/hkcsa.h).  Used by the `csa` drop-in classes, by bench.py
and by the GPU parity tests.
"""
from __future__ import annotations

import ctypes as C
from typing import Iterable, Sequence

import numpy as np

from . import _native as N


def _ptr(a: np.ndarray):
    return a.ctypes.data_as(C.c_void_p)


def pack_patterns(patterns: Sequence[bytes]) -> tuple[np.ndarray, np.ndarray]:
    """Concatenate byte patterns into (data u8, offsets u64[P+1])."""
    offs = np.zeros(len(patterns) + 1, dtype=np.uint64)
    if patterns:
        offs[1:] = np.cumsum(np.fromiter((len(p) for p in patterns), dtype=np.uint64, count=len(patterns)))
    data = np.frombuffer(b"".join(patterns), dtype=np.uint8) if offs[-1] else np.zeros(0, dtype=np.uint8)
    return np.ascontiguousarray(data), offs


class QuerySet:
    """Device-resident batch of patterns (hkcsa_queries)."""

    def __init__(self, index: "DeviceIndex", data: np.ndarray, offs: np.ndarray):
        self.index = index
        self.P = len(offs) - 1
        self._h = C.c_void_p()
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        N.check(index.lib.hkcsa_queries_upload(index.h, _ptr(data) if len(data) else None, _ptr(offs),
                                               self.P, C.byref(self._h)))
        self.total = None

    def count(self):
        N.check(self.index.lib.hkcsa_queries_count(self.index.h, self._h))

    def locate(self) -> int:
        t = C.c_uint64(0)
        N.check(self.index.lib.hkcsa_queries_locate(self.index.h, self._h, C.byref(t)))
        self.total = t.value
        return self.total

    def ranges(self) -> np.ndarray:
        lr = np.empty((self.P, 2), dtype=np.int64)
        N.check(self.index.lib.hkcsa_queries_download(self.index.h, self._h, _ptr(lr), None, None, 0))
        return lr

    def positions(self) -> tuple[np.ndarray, np.ndarray]:
        if self.total is None:
            self.locate()
        offs = np.empty(self.P + 1, dtype=np.uint64)
        pos = np.empty(max(1, self.total), dtype=np.uint64)
        N.check(self.index.lib.hkcsa_queries_download(self.index.h, self._h, None, _ptr(offs), _ptr(pos),
                                                      len(pos)))
        return offs, pos[:self.total]

    def close(self):
        if self._h:
            self.index.lib.hkcsa_queries_free(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


FLAG_POS64 = 1   # HKCSA_FLAG_POS64: 64-bit positions in sharded builds at any n
FLAG_GLOBAL_SORT = 4   # HKCSA_FLAG_GLOBAL_SORT: build by full-width LSD sort (no bucket sorts)
FLAG_MUL_BINS = 8      # HKCSA_FLAG_MUL_BINS: sharded slices use multiplicative bucket bins (diagnostic)
FLAG_MAX_BUCKETS = 16  # HKCSA_FLAG_MAX_BUCKETS: single GPU, the most bucket bits at any n (diagnostic)
FLAG_SLICES = 32       # HKCSA_FLAG_SLICES: single GPU, the multi-slice build (n >= 2^32 - 1) at any n
FLAG_LINKS = 64        # HKCSA_FLAG_LINKS: single GPU, doubling links at any tie count (parity tests)
FLAG_NO_LINKS = 128    # HKCSA_FLAG_NO_LINKS: single GPU, no doubling links (diagnostic)


class DeviceIndex:
    """One text T' resident in HBM plus its SA / BWT / wavelet tree."""

    def __init__(self, handle: C.c_void_p, n: int):
        self.lib = N.load()
        self.h = handle
        self.n = n

    # ------------------------------------------------------------ creation
    @classmethod
    def from_bytes(cls, data, device: int = -1, flags: int = 0) -> "DeviceIndex":
        lib = N.load()
        arr = np.frombuffer(bytes(data), dtype=np.uint8) if isinstance(data, (bytes, bytearray)) else \
            np.ascontiguousarray(data, dtype=np.uint8)
        if len(arr) == 0:
            raise ValueError("DeviceIndex needs a non-empty text (append the sentinel first)")
        o = N.Opts(device=device, flags=flags)
        h = C.c_void_p()
        N.check(lib.hkcsa_create(_ptr(arr), len(arr), C.byref(o), C.byref(h)))
        return cls(h, len(arr))

    @classmethod
    def from_parts(cls, parts: Sequence[np.ndarray], device: int = -1, flags: int = 0) -> "DeviceIndex":
        """T' = the concatenation of `parts` (uint8 arrays, e.g. TextCodec.parts(text, "$")), uploaded
        piece by piece (hkcsa_create_parts): no host-side concatenation."""
        lib = N.load()
        arrs = [np.ascontiguousarray(p).view(np.uint8) for p in parts]
        n = sum(len(a) for a in arrs)
        if n == 0:
            raise ValueError("DeviceIndex needs a non-empty text (append the sentinel first)")
        ptrs = (C.c_void_p * len(arrs))(*[a.ctypes.data if len(a) else None for a in arrs])
        lens = (C.c_uint64 * len(arrs))(*[len(a) for a in arrs])
        o = N.Opts(device=device, flags=flags)
        h = C.c_void_p()
        N.check(lib.hkcsa_create_parts(ptrs, lens, len(arrs), C.byref(o), C.byref(h)))
        return cls(h, n)

    @classmethod
    def synthetic(cls, n: int, alphabet: bytes, seed: int, terminator: int = ord("$"),
                  device: int = -1, flags: int = 0) -> "DeviceIndex":
        lib = N.load()
        a = np.frombuffer(bytes(alphabet), dtype=np.uint8)
        o = N.Opts(device=device, flags=flags)
        h = C.c_void_p()
        N.check(lib.hkcsa_create_synthetic(n, _ptr(a), len(a), seed, terminator, C.byref(o), C.byref(h)))
        return cls(h, n)

    def close(self):
        if self.h:
            self.lib.hkcsa_free(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ------------------------------------------------------------ builds
    def build_sa(self):
        N.check(self.lib.hkcsa_build_sa(self.h))

    def build_bwt(self):
        N.check(self.lib.hkcsa_build_bwt(self.h))

    def build_wt(self):
        N.check(self.lib.hkcsa_build_wt(self.h))

    def build_all(self):
        N.check(self.lib.hkcsa_build_all(self.h))

    def use_text_as_bwt(self):
        N.check(self.lib.hkcsa_use_text_as_bwt(self.h))

    def release_workspace(self):
        N.check(self.lib.hkcsa_release_workspace(self.h))

    def synchronize(self):
        N.check(self.lib.hkcsa_synchronize(self.h))

    def build_samples(self, rate: int):
        """SA/ISA samples every `rate` positions (hkcsa_build_samples)."""
        N.check(self.lib.hkcsa_build_samples(self.h, int(rate)))

    def compact(self):
        """Drop SA, BWT array, text and workspace; queries continue from the WT + samples."""
        N.check(self.lib.hkcsa_compact(self.h))

    def entropy(self, k: int) -> float:
        """Empirical H_k of the stored buffer (hkcsa_entropy)."""
        out = C.c_double(0)
        N.check(self.lib.hkcsa_entropy(self.h, int(k), C.byref(out)))
        return out.value

    def space(self) -> dict:
        out = np.zeros(8, dtype=np.uint64)
        N.check(self.lib.hkcsa_space(self.h, _ptr(out)))
        keys = ["text", "sa", "bwt", "wt", "sample_marks", "samples", "sample_rate", "sampled"]
        return {k: int(v) for k, v in zip(keys, out)}

    # ------------------------------------------------------------ exports
    def sa(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.n if hi is None else hi
        out = np.empty(max(0, hi - lo), dtype=np.uint64)
        N.check(self.lib.hkcsa_get_sa(self.h, lo, hi, _ptr(out) if len(out) else None))
        return out

    def bwt(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.n if hi is None else hi
        out = np.empty(max(0, hi - lo), dtype=np.uint8)
        N.check(self.lib.hkcsa_get_bwt(self.h, lo, hi, _ptr(out) if len(out) else None))
        return out

    def text(self, lo: int = 0, hi: int | None = None) -> np.ndarray:
        hi = self.n if hi is None else hi
        out = np.empty(max(0, hi - lo), dtype=np.uint8)
        N.check(self.lib.hkcsa_get_text(self.h, lo, hi, _ptr(out) if len(out) else None))
        return out

    def extract(self, i: int, j: int) -> bytes:
        if j <= i:
            return b""
        out = np.empty(j - i, dtype=np.uint8)
        N.check(self.lib.hkcsa_extract(self.h, i, j, _ptr(out)))
        return out.tobytes()

    def C(self) -> np.ndarray:
        out = np.empty(257, dtype=np.uint64)
        N.check(self.lib.hkcsa_get_C(self.h, _ptr(out)))
        return out

    def alphabet(self) -> bytes:
        syms = np.zeros(256, dtype=np.uint8)
        s = C.c_int(0)
        N.check(self.lib.hkcsa_get_alphabet(self.h, _ptr(syms), C.byref(s)))
        return syms[:s.value].tobytes()

    def wt_levels(self) -> int:
        L = C.c_int(0)
        N.check(self.lib.hkcsa_wt_levels(self.h, C.byref(L)))
        return L.value

    def wt_level_bits(self, depth: int) -> np.ndarray:
        """Level `depth` as a uint8 0/1 array of length n."""
        nb = C.c_uint64(0)
        N.check(self.lib.hkcsa_wt_level(self.h, depth, C.byref(nb), None))
        words = np.empty((nb.value + 63) // 64 or 1, dtype=np.uint64)
        N.check(self.lib.hkcsa_wt_level(self.h, depth, C.byref(nb), _ptr(words)))
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")
        return bits[:nb.value]

    def wt_golomb(self, depth: int, nbits: int | None = None, m: int = 0, sizes_only: bool = False):
        """Golomb-Rice code of level `depth`'s first nbits bits: (m, ones, code bits as u8 0/1 array)
        — or (m, ones, code length) with sizes_only."""
        nbits = self.n if nbits is None else nbits
        mo, ones, nb = C.c_uint32(0), C.c_uint64(0), C.c_uint64(0)
        if sizes_only:
            N.check(self.lib.hkcsa_wt_golomb(self.h, depth, nbits, m, C.byref(mo), C.byref(ones), C.byref(nb),
                                             None, 0))
            return mo.value, ones.value, nb.value
        N.check(self.lib.hkcsa_wt_golomb(self.h, depth, nbits, m, C.byref(mo), C.byref(ones), C.byref(nb), None, 0))
        words = np.zeros(max(1, (nb.value + 63) // 64), dtype=np.uint64)
        N.check(self.lib.hkcsa_wt_golomb(self.h, depth, nbits, m, C.byref(mo), C.byref(ones), C.byref(nb),
                                         _ptr(words), len(words)))
        bits = np.unpackbits(words.view(np.uint8), bitorder="little")[:nb.value]
        return mo.value, ones.value, bits

    def rank(self, cs, idx) -> np.ndarray:
        cs = np.ascontiguousarray(cs, dtype=np.uint8)
        idx = np.ascontiguousarray(idx, dtype=np.uint64)
        out = np.empty(len(cs), dtype=np.uint64)
        if len(cs):
            N.check(self.lib.hkcsa_rank(self.h, _ptr(cs), _ptr(idx), len(cs), _ptr(out)))
        return out

    # ------------------------------------------------------------ queries
    def queries(self, patterns: Sequence[bytes] | None = None, data=None, offs=None) -> QuerySet:
        if patterns is not None:
            data, offs = pack_patterns(patterns)
        return QuerySet(self, data, offs)

    def count_ranges(self, patterns: Sequence[bytes]) -> np.ndarray:
        q = self.queries(patterns)
        try:
            q.count()
            return q.ranges()
        finally:
            q.close()

    def locate(self, patterns: Sequence[bytes]) -> tuple[np.ndarray, np.ndarray]:
        q = self.queries(patterns)
        try:
            q.locate()
            return q.positions()
        finally:
            q.close()

    def locate_batch(self, data: np.ndarray, offs: np.ndarray, cap: int | None = None) -> tuple[np.ndarray, np.ndarray]:
        """hkcsa_locate_batch from host buffers: (CSR offsets u64[P+1], positions u64) in caller-owned
        arrays.  One call when `cap` (default 2 positions per pattern + 1024) holds every position,
        else a second call with the exact size the first one reported."""
        data = np.ascontiguousarray(data, dtype=np.uint8)
        offs = np.ascontiguousarray(offs, dtype=np.uint64)
        P = len(offs) - 1
        occ = np.empty(P + 1, dtype=np.uint64)
        cap = 2 * P + 1024 if cap is None else int(cap)
        pos = np.empty(max(1, cap), dtype=np.uint64)
        rc = self.lib.hkcsa_locate_batch(self.h, _ptr(data) if len(data) else None, _ptr(offs), P, _ptr(occ),
                                         _ptr(pos), cap)
        if rc == N.E_RANGE:
            pos = np.empty(max(1, int(occ[P])), dtype=np.uint64)
            rc = self.lib.hkcsa_locate_batch(self.h, _ptr(data) if len(data) else None, _ptr(offs), P,
                                             _ptr(occ), _ptr(pos), len(pos))
        N.check(rc)
        return occ, pos[:int(occ[P])]

    # ------------------------------------------------------------ sharding
    def build_sa_sharded(self, uid: bytes, nranks: int, rank: int):
        b = np.frombuffer(uid, dtype=np.uint8)
        N.check(self.lib.hkcsa_build_sa_sharded(self.h, _ptr(b), nranks, rank))

    def shard_scheme(self) -> int:
        """1: keyed coarse partition (exact 65536-bin histogram), 0: sampled partition key."""
        s = C.c_int(0)
        N.check(self.lib.hkcsa_shard_scheme(self.h, C.byref(s)))
        return s.value

    def shard_histogram(self, nranks: int, rank: int) -> np.ndarray:
        out = np.empty(self.lib.hkcsa_shard_buckets(), dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_histogram(self.h, nranks, rank, _ptr(out)))
        return out

    def shard_counts(self, global_hist: np.ndarray, nranks: int, rank: int) -> np.ndarray:
        g = np.ascontiguousarray(global_hist, dtype=np.uint64)
        out = np.zeros(nranks + 1, dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_counts(self.h, _ptr(g), nranks, rank, _ptr(out)))
        return out

    def shard_build(self, global_hist: np.ndarray, global_below: np.ndarray, nranks: int, rank: int):
        g = np.ascontiguousarray(global_hist, dtype=np.uint64)
        b = np.ascontiguousarray(global_below, dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_build(self.h, _ptr(g), _ptr(b), nranks, rank))

    def shard_range(self) -> tuple[int, int]:
        lo, hi = C.c_uint64(0), C.c_uint64(0)
        N.check(self.lib.hkcsa_shard_range(self.h, C.byref(lo), C.byref(hi)))
        return lo.value, hi.value

    def shard_status(self) -> tuple[int, int, int, int]:
        """(lo, hi, tied suffixes left in the slice, their common-prefix length)."""
        st = np.zeros(4, dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_status(self.h, _ptr(st)))
        return tuple(int(x) for x in st)

    def shard_isa_segment(self, sa_segment: np.ndarray, lo: int):
        """Load ISA[sa_segment[j]] = lo + j into this rank's ISA replica (one call per rank slice)."""
        a = np.ascontiguousarray(sa_segment, dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_isa_segment(self.h, _ptr(a) if len(a) else None, len(a), int(lo)))

    def shard_updates(self) -> np.ndarray:
        """(position, ISA) pairs of the last build / doubling step of this rank, shape (k, 2)."""
        c = C.c_uint64(0)
        N.check(self.lib.hkcsa_shard_updates(self.h, None, 0, C.byref(c)))
        out = np.empty((max(1, c.value), 2), dtype=np.uint64)
        N.check(self.lib.hkcsa_shard_updates(self.h, _ptr(out), c.value, C.byref(c)))
        return out[:c.value]

    def shard_apply(self, pairs: np.ndarray):
        p = np.ascontiguousarray(pairs, dtype=np.uint64).reshape(-1, 2)
        N.check(self.lib.hkcsa_shard_apply(self.h, _ptr(p) if len(p) else None, len(p)))

    def shard_round(self, K: int):
        N.check(self.lib.hkcsa_shard_round(self.h, int(K)))

    def shard_replicate(self):
        """RCCL all-gather of every rank's SA slice and BWT rows: this handle becomes a full index."""
        N.check(self.lib.hkcsa_shard_replicate(self.h))

    def shard_adopt(self, sa: np.ndarray, bwt: np.ndarray):
        """Host-assembled replica: the full SA and BWT (hosts running their own collectives)."""
        s = np.ascontiguousarray(sa, dtype=np.uint64)
        b = np.ascontiguousarray(bwt, dtype=np.uint8)
        if len(s) != self.n or len(b) != self.n:
            raise ValueError("shard_adopt needs n SA entries and n BWT bytes")
        N.check(self.lib.hkcsa_shard_adopt(self.h, _ptr(s), _ptr(b)))

    def shard_sa(self, out: np.ndarray | None = None) -> np.ndarray:
        """SA[lo:hi) of this rank (u64); `out` (a contiguous u64 array of hi - lo entries) is filled in
        place when given."""
        lo, hi = self.shard_range()
        if out is None:
            out = np.empty(max(1, hi - lo), dtype=np.uint64)
        elif out.dtype != np.uint64 or not out.flags.c_contiguous or len(out) != hi - lo:
            raise ValueError("shard_sa: out must be a contiguous u64 array of the slice's length")
        if hi > lo:
            N.check(self.lib.hkcsa_get_shard_sa(self.h, 0, hi - lo, _ptr(out)))
        return out[:hi - lo]

    def shard_bwt(self, out: np.ndarray | None = None) -> np.ndarray:
        lo, hi = self.shard_range()
        if out is None:
            out = np.empty(max(1, hi - lo), dtype=np.uint8)
        elif out.dtype != np.uint8 or not out.flags.c_contiguous or len(out) != hi - lo:
            raise ValueError("shard_bwt: out must be a contiguous u8 array of the slice's length")
        if hi > lo:
            N.check(self.lib.hkcsa_get_shard_bwt(self.h, 0, hi - lo, _ptr(out)))
        return out[:hi - lo]

    # ------------------------------------------------------------ timing
    def timing(self, on: bool):
        N.check(self.lib.hkcsa_timing_enable(self.h, 1 if on else 0))

    def timing_reset(self):
        N.check(self.lib.hkcsa_timing_reset(self.h))

    def kernel_stats(self, name: str) -> tuple[int, float, float]:
        l, ms, b = C.c_uint64(0), C.c_double(0), C.c_double(0)
        N.check(self.lib.hkcsa_kernel_stats(self.h, name.encode(), C.byref(l), C.byref(ms), C.byref(b)))
        return l.value, ms.value, b.value

    def build_info(self) -> list[int]:
        out = np.zeros(64, dtype=np.uint64)
        N.check(self.lib.hkcsa_build_info(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), 64))
        return [int(x) for x in out]


def comm_unique_id() -> bytes:
    lib = N.load()
    b = np.zeros(128, dtype=np.uint8)
    N.check(lib.hkcsa_comm_unique_id(_ptr(b)))
    return b.tobytes()


def bwt_gather(text: bytes, sa: Iterable[int]) -> bytes:
    lib = N.load()
    t = np.frombuffer(bytes(text), dtype=np.uint8)
    s = np.ascontiguousarray(np.fromiter(sa, dtype=np.uint64) if not isinstance(sa, np.ndarray) else sa,
                             dtype=np.uint64)
    if len(s) != len(t):
        raise ValueError("suffix array length differs from text length")
    if len(t) == 0:
        return b""
    out = np.empty(len(t), dtype=np.uint8)
    N.check(lib.hkcsa_bwt_gather(_ptr(t), len(t), _ptr(s), _ptr(out)))
    return out.tobytes()
