"""Pattern sampling of the reference's benchmark (tests/test_patterns.py:3-9).

generate_random_patterns(text, pattern_lengths) returns one substring of `text` per requested
length, min(length, len(text)) symbols long, starting at a uniformly random offset in
[0, len(text) - length] — the reference's behaviour, here with an optional `seed` (the
reference draws from the unseeded global `random`).  sample_substrings() is the batched form
the GPU bench uses: P substrings of one length as a flat uint8 array plus offsets, ready for
hkcsa_count_batch / hkcsa_locate_batch.
"""
from __future__ import annotations

import random

import numpy as np


def generate_random_patterns(text, pattern_lengths, seed=None):
    rng = random.Random(seed) if seed is not None else random
    patterns = []
    for length in pattern_lengths:
        actual = min(length, len(text))
        start = rng.randint(0, len(text) - actual)
        patterns.append(text[start:start + actual])
    return patterns


def sample_substrings(text, count: int, length: int, seed: int = 1):
    """`count` substrings of `length` bytes at uniform offsets: (flat u8 data, u64 offsets[count+1])."""
    t = np.frombuffer(text, np.uint8) if isinstance(text, (bytes, bytearray)) else np.asarray(text, np.uint8)
    length = min(length, len(t))
    rng = np.random.default_rng(seed)
    starts = rng.integers(0, len(t) - length + 1, size=count)
    data = t[starts[:, None] + np.arange(length)[None, :]].reshape(-1)
    offs = np.arange(count + 1, dtype=np.uint64) * np.uint64(length)
    return np.ascontiguousarray(data), offs
