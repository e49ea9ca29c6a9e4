"""Pure-Python restatement of the reference algorithms — TEST INFRASTRUCTURE ONLY.

Used by tests/ (small parity cases) and by bench.py's cpu_baseline leg (the
single-core "port" baseline).  Never imported by the product.
Every routine names the reference lines it restates; the loops keep the
reference's algorithmic cost (O(n^2)-memory suffix sort, O(n*sigma) occ table)
so the timed baseline is representative of the reference itself.
"""
from __future__ import annotations

import math
from collections import Counter


# csa/suffix_array.py:131-134 — sort every suffix slice, keep the start indices
def naive_suffix_array(text: str) -> list[int]:
    return sorted(range(len(text)), key=lambda i: text[i:])


# csa/bwt.py:3-13 — symbol before each sorted suffix, wrapping at the start
def bwt_of(text: str, sa: list[int]) -> str:
    return "".join(text[p - 1] if p > 0 else text[-1] for p in sa) if text else ""


# utils/utils.py:16-24 — symbols smaller than c, for each present c
def count_table(text: str) -> dict:
    freq = Counter(text)
    out, acc = {}, 0
    for ch in sorted(freq):
        out[ch] = acc
        acc += freq[ch]
    return out


# utils/utils.py:26-32 — dense occurrence table, one running count list per symbol
def occ_table(bwt: str) -> dict:
    tab = {ch: [0] for ch in set(bwt)}
    for sym in bwt:
        for ch, col in tab.items():
            col.append(col[-1] + (1 if sym == ch else 0))
    return tab


class FMIndexPort:
    """csa/enhanced_fm_index.py:7-40 restated: T' = text + '$', SA, BWT, occ, C."""

    def __init__(self, text: str, sa: list[int] | None = None):
        self.text = text + "$"
        self.suffix_array = naive_suffix_array(self.text) if sa is None else list(sa)
        self.bwt = bwt_of(self.text, self.suffix_array)
        self.occ = occ_table(self.bwt)
        self.count = count_table(self.text)

    def rank(self, ch: str, i: int) -> int:
        col = self.occ.get(ch)
        if col is None:
            return 0
        return col[min(i, len(col) - 1)]

    def find_range(self, pattern: str):
        lo, hi = 0, len(self.bwt) - 1
        for ch in pattern[::-1]:
            base = self.count.get(ch, 0)
            nlo = base + self.rank(ch, lo)
            nhi = base + self.rank(ch, hi + 1) - 1
            if nlo > nhi:
                return -1, -1
            lo, hi = nlo, nhi
        return lo, hi

    def find(self, pattern: str) -> list[int]:
        lo, hi = self.find_range(pattern)
        if lo == -1 or hi == -1:
            return []
        return self.suffix_array[lo:hi + 1]


# csa/wavelet_tree.py:33-38 — Golomb parameter from the density of ones (float log2)
def golomb_m(bits: list[int]) -> int:
    ones = sum(bits)
    if ones == 0:
        return 1
    return max(1, int(math.log2(1 / (ones / len(bits)))))


# csa/wavelet_tree.py:40-63 — Golomb-code the length of every run of ones
def golomb_encode(bits: list[int], m: int) -> list[int]:
    out: list[int] = []

    def emit(v: int):
        q, r = divmod(v, m)
        out.extend([0] * q)
        out.append(1)
        out.extend(int(b) for b in format(r, "b").zfill(m))

    run = 0
    for b in bits:
        if b == 1:
            run += 1
        elif run:
            emit(run)
            run = 0
    if run:
        emit(run)
    return out


def left_spine_levels(seq) -> list[dict]:
    """csa/wavelet_tree.py:72-100: follow the left child while it has more than one symbol."""
    alpha = sorted(set(seq))
    cur = list(seq)
    levels = []
    while len(alpha) > 1:
        half = len(alpha) // 2
        left, right = alpha[:half], alpha[half:]
        rset = set(right)
        bits = [1 if s in rset else 0 for s in cur]
        m = golomb_m(bits)
        levels.append({"left": left, "right": right, "bits": bits, "m": m,
                       "golomb": golomb_encode(bits, m)})
        lset = set(left)
        cur = [s for s in cur if s in lset]
        alpha = left
    return levels


# csa/high_order_entropy.py:4-32 — empirical H_0 / H_k
def high_order_entropy(text: str, k: int) -> float:
    if not text or k < 0:
        return 0
    n = len(text)
    if k == 0:
        return -sum((c / n) * math.log2(c / n) for c in Counter(text).values())
    if n <= k:
        return 0
    ctx: dict = {}
    for i in range(n - k):
        ctx.setdefault(text[i:i + k], Counter())[text[i + k]] += 1
    h = 0.0
    for counts in ctx.values():
        tot = sum(counts.values())
        h += (tot / n) * -sum((c / tot) * math.log2(c / tot) for c in counts.values())
    return h
