"""Seeded natural-language-like text: the shape of configs[2]'s corpus without the corpus.

BASELINE.json configs[2] is Pizza&Chili english.200MB (the corpora of the reference's
tests/dataset_benchmark.py:10-16), read as latin-1 (utils/data_loader.py:3-7).  It is not available
offline, and iid printable bytes miss what matters for suffix sorting English: a skewed alphabet,
Zipf-distributed words (so short contexts repeat constantly) and long repeated passages (so many
suffixes share prefixes far longer than any fixed key).  english_like() builds such a text:

* a vocabulary of `vocab` words over English letter frequencies (a few percent of them numbers or
  words with latin-1 accented bytes), the most frequent ranks seeded with English function words;
* a word stream drawn by a Zipf law (p(rank) ~ 1 / (rank + 2.7)^1.05), words joined by spaces,
  commas, sentence ends (". " / ".\\n") and paragraph breaks, each sentence capitalised;
* the final text alternates fresh stretches of that stream (exponential lengths) with verbatim
  copies of earlier stretches (`copy_frac` of all bytes, log-uniform lengths in [min_copy,
  max_copy]), plus `long_copies` copies of 64 KiB - 1 MiB passages: LCPs of 50 symbols to a megabyte.

protein_like() is the shape of the corpus' proteins file (tests/dataset_benchmark.py:13): sequences
over the 20 amino-acid letters (plus the rare B, Z, X, U, O: sigma = 25) at their natural frequencies,
one per line, lengths ~ Gamma(mean 350), where a share of the sequences are family members — copies of
an earlier sequence with point substitutions — and a few are exact duplicates:
repeats with mismatches every few dozen symbols, so ties break slowly but no prefix runs for megabytes.

Everything is a pure function of (n, seed, parameters): tests and bench.py regenerate the same
bytes on any host (numpy Generator PCG64, chunked so memory stays O(n)).
"""
from __future__ import annotations

import numpy as np

_LETTERS = np.frombuffer(b"etaoinshrdlcumwfgypbvkjxqz", dtype=np.uint8)
_LETTER_P = np.array([12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8, 2.4, 2.4, 2.2, 2.0,
                      2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07])
_FUNCTION_WORDS = [b"the", b"of", b"and", b"to", b"a", b"in", b"that", b"is", b"was", b"he", b"for", b"it",
                   b"with", b"as", b"his", b"on", b"be", b"at", b"by", b"i", b"this", b"had", b"not", b"are",
                   b"but", b"from", b"or", b"have", b"an", b"they", b"which", b"one", b"you", b"were", b"her",
                   b"all", b"she", b"there", b"would", b"their", b"we", b"him", b"been", b"has", b"when"]
_ACCENTED = np.frombuffer(bytes([0xE9, 0xE8, 0xEA, 0xE0, 0xE2, 0xE7, 0xF4, 0xFC, 0xF6, 0xE4, 0xF1, 0xDF]),
                          dtype=np.uint8)
# token separators: (bytes, probability)
_SEPS = [(b" ", 0.845), (b", ", 0.07), (b". ", 0.06), (b".\n", 0.015), (b".\n\n", 0.005), (b"; ", 0.005)]


def _vocabulary(rng: np.random.Generator, vocab: int) -> tuple[np.ndarray, np.ndarray]:
    """Flat bytes + offsets[vocab + 1] of the word list, in Zipf rank order."""
    words = list(_FUNCTION_WORDS)
    lp = _LETTER_P / _LETTER_P.sum()
    lens = np.clip(np.round(rng.gamma(4.0, 1.35, size=vocab)).astype(np.int64), 2, 18)
    kind = rng.random(vocab)
    for i in range(len(words), vocab):
        L = int(lens[i])
        if kind[i] < 0.02:      # a number
            w = bytes(rng.integers(0x30, 0x3A, size=min(L, 6)).astype(np.uint8))
        else:
            w = _LETTERS[rng.choice(26, size=L, p=lp)].copy()
            if kind[i] > 0.985:  # a latin-1 accented letter somewhere
                w[int(rng.integers(0, L))] = _ACCENTED[int(rng.integers(0, len(_ACCENTED)))]
            w = w.tobytes()
        words.append(w)
    offs = np.zeros(vocab + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(w) for w in words[:vocab]])
    return np.frombuffer(b"".join(words[:vocab]), dtype=np.uint8), offs


def _stream(rng: np.random.Generator, nbytes: int, flat: np.ndarray, woffs: np.ndarray) -> np.ndarray:
    """`nbytes` of Zipf word stream with separators and capitalised sentence starts."""
    vocab = len(woffs) - 1
    cdf = np.cumsum(1.0 / (np.arange(vocab) + 2.7) ** 1.05)
    cdf /= cdf[-1]
    sep_bytes = [s for s, _ in _SEPS]
    sep_p = np.array([p for _, p in _SEPS])
    sep_p /= sep_p.sum()
    sep_len = np.array([len(s) for s in sep_bytes], dtype=np.int64)
    sep_flat = np.frombuffer(b"".join(sep_bytes), dtype=np.uint8)
    sep_off = np.concatenate(([0], np.cumsum(sep_len)))
    ends_sentence = np.array([s.startswith(b".") for s in sep_bytes])
    wlen = np.diff(woffs)
    out = np.empty(nbytes, dtype=np.uint8)
    pos = 0
    cap_next = True
    while pos < nbytes:
        W = 1 << 20
        ids = np.searchsorted(cdf, rng.random(W))
        sep = rng.choice(len(sep_bytes), size=W, p=sep_p)
        tl = wlen[ids] + sep_len[sep]
        starts = np.concatenate(([0], np.cumsum(tl)[:-1]))
        total = int(tl.sum())
        tok = np.repeat(np.arange(W), tl)
        k = np.arange(total) - starts[tok]
        wl = wlen[ids][tok]
        in_word = k < wl
        buf = np.where(in_word, flat[np.minimum(woffs[ids][tok] + k, len(flat) - 1)],
                       sep_flat[np.clip(sep_off[sep][tok] + (k - wl), 0, len(sep_flat) - 1)])
        # capitalise the first letter of every sentence
        cap = np.concatenate(([cap_next], ends_sentence[sep][:-1]))
        first = starts[cap]
        b = buf[first]
        buf[first] = np.where((b >= 0x61) & (b <= 0x7A), b - 32, b)
        cap_next = bool(ends_sentence[sep][-1])
        take = min(total, nbytes - pos)
        out[pos:pos + take] = buf[:take]
        pos += take
    return out


def english_like(n: int, seed: int = 0, copy_frac: float = 0.25, min_copy: int = 50, max_copy: int = 5000,
                 long_copies: int = 8, vocab: int = 30000) -> np.ndarray:
    """n bytes (uint8) of seeded natural-language-like latin-1 text (no '$' appended)."""
    if n <= 0:
        return np.zeros(0, dtype=np.uint8)
    rng = np.random.default_rng(seed)
    flat, woffs = _vocabulary(rng, vocab)
    # block plan: fresh stretches and copies of earlier stretches of the base stream
    mean_copy = (max_copy - min_copy) / np.log(max_copy / min_copy) if max_copy > min_copy else float(min_copy)
    mean_fresh = mean_copy * (1 - copy_frac) / max(copy_frac, 1e-9) if copy_frac > 0 else float(n)
    nblk = int(n / (mean_fresh + mean_copy) * 1.3) + 16
    fresh = np.maximum(1, rng.exponential(mean_fresh, size=nblk)).astype(np.int64)
    copy = np.exp(rng.uniform(np.log(min_copy), np.log(max_copy), size=nblk)).astype(np.int64) if copy_frac > 0 \
        else np.zeros(nblk, dtype=np.int64)
    if long_copies and copy_frac > 0:
        pick = rng.choice(np.arange(nblk // 4, nblk // 2), size=min(long_copies, max(1, nblk // 8)), replace=False)
        copy[pick] = rng.integers(1 << 16, 1 << 20, size=len(pick))
    lens = np.stack([fresh, copy], axis=1).reshape(-1)
    out_start = np.concatenate(([0], np.cumsum(lens)[:-1]))
    keep = out_start < n
    lens, out_start = lens[keep], out_start[keep]
    lens[-1] = n - out_start[-1]
    is_copy = (np.arange(len(lens)) % 2) == 1
    fresh_len = np.where(is_copy, 0, lens)
    base_start = np.concatenate(([0], np.cumsum(fresh_len)[:-1]))   # base cursor before each block
    base_n = int(fresh_len.sum())
    base = _stream(rng, max(base_n, 1), flat, woffs)
    # copies read an earlier stretch of the base stream (start uniform over what precedes the block)
    room = np.maximum(base_start - lens, 0)
    src = np.where(is_copy & (base_start >= lens), (rng.random(len(lens)) * room).astype(np.int64), -1)
    src = np.where(is_copy & (src < 0), 0, src)
    blk_src = np.where(is_copy, src, base_start)
    # a copy longer than the base stretch before it wraps inside [0, base_start) (still a repeat)
    out = np.empty(n, dtype=np.uint8)
    for b0 in range(0, len(lens), 1 << 16):
        sl = slice(b0, b0 + (1 << 16))
        L, S, O = lens[sl], blk_src[sl], out_start[sl]
        tot = int(L.sum())
        blk = np.repeat(np.arange(len(L)), L)
        k = np.arange(tot) - (O - O[0])[blk]
        idx = S[blk] + k
        lim = np.where(is_copy[sl], np.maximum(base_start[sl], 1), base_n)[blk]
        idx = np.where(idx < lim, idx, idx % lim)
        out[O[0]:O[0] + tot] = base[np.minimum(idx, base_n - 1)]
    return out


_AMINO = np.frombuffer(b"LAGVESIKRDTPNQFYMHCWXBZUO", dtype=np.uint8)
_AMINO_P = np.array([9.9, 8.3, 7.1, 6.9, 6.8, 6.6, 5.9, 5.8, 5.5, 5.5, 5.3, 4.7, 4.1, 3.9, 3.9, 2.9, 2.4, 2.3, 1.4,
                     1.1, 0.08, 0.01, 0.01, 0.005, 0.001])


def protein_like(n: int, seed: int = 0, family_frac: float = 0.35, dup_frac: float = 0.05,
                 mut_rate: float = 0.08) -> np.ndarray:
    """n bytes (uint8) of seeded protein-database-like text: newline-separated sequences (no '$').
    Built in batches of sequences: fresh ones drawn at once, family members / duplicates gathered from
    sequences of earlier batches (a family member then takes point substitutions at `mut_rate`)."""
    if n <= 0:
        return np.zeros(0, dtype=np.uint8)
    rng = np.random.default_rng(seed)
    # letters by a 2^16-entry table of the cumulative frequencies (every letter keeps at least one entry)
    cnt = np.maximum(1, np.round(_AMINO_P / _AMINO_P.sum() * 65536)).astype(np.int64)
    cnt[0] -= int(cnt.sum()) - 65536
    table = np.repeat(_AMINO, cnt)
    draw = lambda size: table[rng.integers(0, 65536, size=size, dtype=np.uint32)]
    out = np.empty(n, dtype=np.uint8)
    starts = np.zeros(0, dtype=np.int64)   # earlier batches' sequences
    slens = np.zeros(0, dtype=np.int64)
    pos = 0
    while pos < n:
        K = 1 << 15
        kind = rng.random(K)
        lens = np.maximum(20, rng.gamma(2.0, 175.0, size=K)).astype(np.int64)
        copy = (kind < dup_frac + family_frac) & (len(starts) > 0)
        src = np.full(K, -1, dtype=np.int64)
        if len(starts):
            pick = rng.integers(0, len(starts), size=K)
            src = np.where(copy, starts[pick], -1)
            lens = np.where(copy, slens[pick], lens)
        tl = lens + 1                                        # + the newline
        st = pos + np.concatenate(([0], np.cumsum(tl)[:-1]))
        keep = st < n
        lens, tl, st, src, kind = lens[keep], tl[keep], st[keep], src[keep], kind[keep]
        tot = int(min(int(tl.sum()), n - pos))
        seq = np.repeat(np.arange(len(lens)), tl)[:tot]
        k = np.arange(pos, pos + tot) - st[seq]
        buf = draw(tot)
        is_copy = (src[seq] >= 0) & (k < lens[seq])
        buf[is_copy] = out[src[seq][is_copy] + k[is_copy]]
        fam = is_copy & (kind[seq] >= dup_frac)
        mut = fam & (rng.random(tot) < mut_rate)
        buf[mut] = draw(int(mut.sum()))
        buf[k == lens[seq]] = 0x0A
        out[pos:pos + tot] = buf
        full = st + lens <= pos + tot
        starts = np.concatenate([starts, st[full]])
        slens = np.concatenate([slens, lens[full]])
        pos += tot
    return out


def protein_like_text(n: int, seed: int = 0, **kw) -> np.ndarray:
    """T' = protein_like(n - 1) + '$'."""
    t = np.empty(n, dtype=np.uint8)
    t[:-1] = protein_like(n - 1, seed, **kw)
    t[-1] = ord("$")
    return t


def english_like_text(n: int, seed: int = 0, **kw) -> np.ndarray:
    """T' = english_like(n - 1) + '$' (the reference's sentinel, csa/enhanced_fm_index.py:9)."""
    t = np.empty(n, dtype=np.uint8)
    t[:-1] = english_like(n - 1, seed, **kw)
    t[-1] = ord("$")
    return t
