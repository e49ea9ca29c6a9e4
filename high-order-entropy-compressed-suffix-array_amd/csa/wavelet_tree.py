"""Drop-in for the reference's csa/wavelet_tree.py.

WaveletTree(seq) builds the FULL balanced wavelet tree of `seq` on the GPU
(levelwise bitvectors with interleaved 64-B rank lines, hkcsa_build_wt) and
exposes the reference's view of it:
  * .tree[l] = (golomb_bits, left_alphabet, right_alphabet, next_text) and
    .rank_structures[l] for the reference's left-spine levels (:72-100).  Level l
    of the reference is the prefix of device level l of length |leftmost node|
    (SURVEY.md §8 "WT levels"), so it is read straight from HBM.
  * .m, .compress() (:151-156) — Golomb-Rice parameters/codes of those levels,
    coded on the GPU (hkcsa_wt_golomb); GolombRiceEncoder stays as the host class.
  * .rank(c, i) / .select(c, k) keep the reference's behaviour of ignoring `c`
    and answering on the last level (:133-149).
  * .alphabet ends as the reference leaves it (the last left alphabet, :99).
Additions: .occ(c, i) — a correct rank of symbol c in seq[0:i) on the GPU — and
.decompress() returning the sequence (the reference's decoder returns '').
"""
from __future__ import annotations

import math

import numpy as np

from hkcsa import DeviceIndex, TextCodec


class SuccinctRankSelect:
    """csa/wavelet_tree.py:5-25: plain bitvector + uint32 prefix ranks, binary-search select."""

    def __init__(self, bitmap):
        self.bit_vector = np.asarray(bitmap, dtype=np.uint8)
        self.n = int(self.bit_vector.size)
        self.rank_support = np.zeros(self.n + 1, dtype=np.uint32)
        np.cumsum(self.bit_vector, dtype=np.uint32, out=self.rank_support[1:])

    def rank(self, i):
        return self.rank_support[i]

    def select(self, k):
        p = int(np.searchsorted(self.rank_support, k, side="left"))
        return min(p, self.n)


class GolombRiceEncoder:
    """csa/wavelet_tree.py:27-63: Golomb-code the lengths of the runs of ones."""

    def __init__(self, bitmap):
        bits = np.asarray(bitmap, dtype=np.uint8)
        self.m = self.compute_dynamic_m(int(bits.sum()), int(bits.size))

    def compute_dynamic_m(self, ones_count, total_len):
        if ones_count == 0:
            return 1
        return max(1, int(math.log2(1 / (ones_count / total_len))))

    def encode(self, bitmap):
        bits = np.asarray(bitmap, dtype=np.int8)
        if bits.size == 0:
            return []
        edges = np.diff(np.concatenate(([0], bits, [0])))
        runs = np.flatnonzero(edges == -1) - np.flatnonzero(edges == 1)
        m = self.m
        out: list = []
        for v in runs.tolist():
            q, r = divmod(v, m)
            out.extend([0] * q)
            out.append(1)
            out.extend((r >> (m - 1 - k)) & 1 for k in range(m))
        return out


def _as_str(seq) -> str:
    return seq if isinstance(seq, str) else "".join(seq)


class WaveletTree:
    def __init__(self, text):
        self.text = text
        self.alphabet = sorted(set(text))
        self.m = None
        self.build_tree()

    def build_tree(self):
        s = _as_str(self.text)
        self.tree = []
        self.rank_structures = []
        self._dev = None
        if not s:
            return
        self._codec = TextCodec(s)
        enc = self._codec.parts(s)[0]          # (a read-only view of s when no remap is needed)
        self._dev = DeviceIndex.from_parts([enc])
        self._dev.use_text_as_bwt()
        self._dev.build_wt()
        C = self._dev.C()
        syms = list(self._dev.alphabet())                      # sorted present bytes
        ccode = [int(C[b]) for b in syms] + [len(enc)]         # ones... #codes < k
        alpha = [self._codec.decode(bytes([b])) for b in syms]
        cur = enc
        level = 0
        width = len(alpha)
        while width > 1:
            half = width // 2
            left, right = alpha[:half], alpha[half:width]
            nbits = ccode[width]
            bits = self._dev.wt_level_bits(level)[:nbits]
            m, _, code = self._dev.wt_golomb(level, nbits)      # GPU Golomb-Rice pass (:84-86)
            gbits = code.tolist()
            if self.m is None:
                self.m = m
            nxt = cur[bits == 0]
            next_text = list(self._codec.decode(nxt.tobytes()))
            self.tree.append((gbits, left, right, next_text))
            self.rank_structures.append(SuccinctRankSelect(bits))
            self.alphabet = left
            cur = nxt
            width = half
            level += 1

    def run_length_encode(self, bitmap):
        # csa/wavelet_tree.py:102-117 expands the runs it finds back into the same bitmap
        return list(bitmap)

    def level_ordered_encode(self, bitmap):
        # csa/wavelet_tree.py:119-131: (bit, run length) pairs
        bits = np.asarray(bitmap, dtype=np.int8)
        if bits.size == 0:
            raise IndexError("list index out of range")
        cut = np.flatnonzero(np.diff(bits)) + 1
        starts = np.concatenate(([0], cut))
        ends = np.concatenate((cut, [bits.size]))
        return [(int(bits[a]), int(b - a)) for a, b in zip(starts, ends)]

    def rank(self, c, i):
        result = 0
        for level in range(len(self.tree)):
            result = self.rank_structures[level].rank(i + 1)
        return result

    def select(self, c, k):
        result = 0
        for level in range(len(self.tree)):
            result = self.rank_structures[level].select(k)
        return result

    def compress(self):
        return [lvl[0] for lvl in self.tree]

    def decompress(self, compressed=None):
        if self._dev is None:
            return ""
        return self._codec.decode(self._dev.text().tobytes())

    def occ(self, c, i) -> int:
        """Number of `c` in seq[0:i) (GPU wavelet-tree rank)."""
        if self._dev is None:
            return 0
        b = self._codec.encode_symbol(c)
        if b is None:
            return 0
        return int(self._dev.rank(np.array([b], np.uint8), np.array([max(0, int(i))], np.uint64))[0])
