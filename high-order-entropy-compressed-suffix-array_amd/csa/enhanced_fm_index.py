"""Drop-in for the reference's csa/enhanced_fm_index.py:7-40 (EnhancedFMIndex).

Same constructor, attributes and methods; construction and every query run on
the GPU through libhkcsa.so:
  * __init__      -> hkcsa_build_all: SA + BWT by the keyed bucket build (q-symbol suffix
                     keys grouped into buckets by two lookback-free scatter passes, LDS
                     bucket sorts that write SA and BWT together, refinement of tied
                     suffixes, prefix doubling for long repeats; texts of >= 2^32 - 1
                     symbols as slices of the final SA), C array and the levelwise
                     wavelet tree (replaces the O(n*sigma) occ table)
  * find_range    -> batched backward search kernel (one lane per pattern)
  * find          -> find_range + SA gather, positions in SA order (:15-19)
  * rank          -> wavelet-tree rank kernel; occ[c][i] semantics incl. the
                     clamp of :37-38
Large attributes (.suffix_array, .bwt, .occ) are materialised lazily from HBM.
Batched variants (find_range_many, find_many) expose the throughput path.
"""
from __future__ import annotations

from collections.abc import Mapping, Sequence

import numpy as np

from hkcsa import DeviceIndex, TextCodec, pack_patterns


class OccColumn(Sequence):
    """occ[c] of utils/utils.py:26-32: length n+1, item i = #c in bwt[0:i)."""

    def __init__(self, dev: DeviceIndex, byte: int, n: int):
        self._dev, self._b, self._n = dev, byte, n

    def __len__(self):
        return self._n + 1

    def __getitem__(self, i):
        if isinstance(i, slice):
            idx = np.arange(*i.indices(self._n + 1), dtype=np.uint64)
            return [int(x) for x in self._dev.rank(np.full(len(idx), self._b, np.uint8), idx)]
        i = int(i)
        if i < 0:
            i += self._n + 1
        if not 0 <= i <= self._n:
            raise IndexError("occ index out of range")
        return int(self._dev.rank(np.array([self._b], np.uint8), np.array([i], np.uint64))[0])

    def __eq__(self, other):
        if isinstance(other, (list, tuple, OccColumn)):
            return len(other) == len(self) and list(self[:]) == list(other)
        return NotImplemented


class OccView(Mapping):
    """Lazy dict {symbol: OccColumn} over the device wavelet tree."""

    def __init__(self, dev: DeviceIndex, codec: TextCodec, n: int):
        self._dev, self._codec, self._n = dev, codec, n
        self._keys = [codec.decode(bytes([b])) for b in dev.alphabet()]

    def __getitem__(self, ch):
        if ch not in self._keys:
            raise KeyError(ch)
        return OccColumn(self._dev, self._codec.encode_symbol(ch), self._n)

    def __iter__(self):
        return iter(self._keys)

    def __len__(self):
        return len(self._keys)

    def __contains__(self, ch):
        return ch in self._keys


class EnhancedFMIndex:
    def __init__(self, text):
        # T' = text + "$" (:9) is uploaded as two pieces — the str's own code-point buffer and the
        # sentinel — so no concatenated copy of a GiB-sized text is built on the host; .text
        # materialises it on first access
        self._raw = text
        self._text = None
        self._codec = TextCodec(text, "$")
        self._dev = DeviceIndex.from_parts(self._codec.parts(text, "$"))
        self._dev.build_all()
        self._dev.release_workspace()
        self._n = len(text) + 1
        C = self._dev.C()
        self.count = {self._codec.decode(bytes([b])): int(C[b]) for b in self._dev.alphabet()}
        self._sa = None
        self._bwt = None
        self._occ = None

    # ---------------------------------------------------------- attributes
    @property
    def text(self) -> str:
        if self._text is None:
            self._text = self._raw + "$"
        return self._text

    @property
    def suffix_array(self) -> list:
        if self._sa is None:
            self._sa = [int(x) for x in self._dev.sa()]
        return self._sa

    @property
    def bwt(self) -> str:
        if self._bwt is None:
            self._bwt = self._codec.decode(self._dev.bwt().tobytes())
        return self._bwt

    @property
    def occ(self) -> OccView:
        if self._occ is None:
            self._occ = OccView(self._dev, self._codec, self._n)
        return self._occ

    @property
    def device_index(self) -> DeviceIndex:
        return self._dev

    # ---------------------------------------------------------- queries
    def _encode(self, queries):
        enc = [self._codec.encode_pattern(q) for q in queries]
        # a symbol the text cannot hold never matches; send a byte absent from T' instead
        absent = self._absent_byte()
        return [e if e is not None else (bytes([absent]) if absent is not None else None) for e in enc]

    def _absent_byte(self):
        present = set(self._dev.alphabet())
        for b in range(256):
            if b not in present:
                return b
        return None

    def find_range_many(self, queries) -> np.ndarray:
        enc = self._encode(queries)
        ok = [e is not None for e in enc]
        lr = np.full((len(enc), 2), -1, dtype=np.int64)
        send = [e for e in enc if e is not None]
        if send:
            lr[np.array(ok)] = self._dev.count_ranges(send)
        return lr

    def find_many(self, queries) -> list:
        enc = self._encode(queries)
        send_idx = [i for i, e in enumerate(enc) if e is not None]
        out = [[] for _ in enc]
        if send_idx:
            data, poffs = pack_patterns([enc[i] for i in send_idx])
            offs, pos = self._dev.locate_batch(data, poffs)   # hkcsa_locate_batch: host in, host out
            for k, i in enumerate(send_idx):
                out[i] = [int(x) for x in pos[offs[k]:offs[k + 1]]]
        return out

    def find_range(self, query):
        l, r = self.find_range_many([query])[0]
        return int(l), int(r)

    def find(self, query):
        return self.find_many([query])[0]

    def rank(self, character, index):
        if character not in self.count:
            return 0
        i = int(index)
        if i >= self._n + 1:
            i = self._n
        if i < 0:
            i += self._n + 1
            if i < 0:
                raise IndexError("list index out of range")
        b = self._codec.encode_symbol(character)
        return int(self._dev.rank(np.array([b], np.uint8), np.array([i], np.uint64))[0])
