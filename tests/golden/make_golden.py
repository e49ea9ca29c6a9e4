"""Generate the golden parity vectors for hkcsa from the reference Python itself.

Runs ONLY in the build container, where the read-only reference lives at
/root/reference (override with HKCSA_REFERENCE).  It imports the reference's
own modules (stdout of their import-time demos suppressed, no bytecode
written), runs them on seeded inputs and writes plain data fixtures:

  tests/golden/kat.json           known-answer vectors
  tests/golden/random_cases.npz   seeded small cases (8c-2)
  tests/golden/large_cases.npz    2^16 / 2^17 cases, hashed (8c-3)

The fixtures are data (inputs + the reference's outputs); nothing of the
reference's source is copied.  Reference entry points exercised:
  csa/enhanced_fm_index.py:7-40   EnhancedFMIndex(text) .suffix_array .bwt
                                  .count .rank() .find_range() .find()
  csa/wavelet_tree.py:65-156      WaveletTree(seq) .tree .rank_structures .m
                                  .compress() .rank() .select()
  csa/suffix_array.py:46-134      ksa(), build_suffix_array()
  csa/high_order_entropy.py:4-32  calculate_high_order_entropy()

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import contextlib
import hashlib
import io
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REF = os.environ.get("HKCSA_REFERENCE", "/root/reference")

# symbol sets for the randomised cases (sigma -> byte alphabet)
ALPHABETS = {
    2: b"ab",
    4: b"ACGT",
    16: bytes(range(0x21, 0x31)),     # contains '$' (0x24)
    95: bytes(range(0x20, 0x7F)),     # printable, contains '$' and ' '
    256: bytes(range(256)),
}
SIZES = [1, 2, 3, 7, 64, 1000, 4096]
SEEDS = [0, 1, 2, 3]


def _import_reference():
    sys.dont_write_bytecode = True
    sys.path.insert(0, REF)
    with contextlib.redirect_stdout(io.StringIO()):
        from csa import enhanced_fm_index, wavelet_tree, suffix_array, high_order_entropy  # noqa
    return enhanced_fm_index, wavelet_tree, suffix_array, high_order_entropy


def gen_text(seed: int, sigma: int, n: int) -> bytes:
    """Seeded synthetic text; reproducible without the reference."""
    alpha = np.frombuffer(ALPHABETS[sigma], dtype=np.uint8)
    rng = np.random.default_rng(1000 * seed + sigma)
    return alpha[rng.integers(0, len(alpha), size=n)].tobytes()


def gen_patterns(seed: int, tp: bytes, alpha: bytes, count: int, maxlen: int = 20):
    """70% substrings of T' (text+'$'), 30% random strings (absent symbols,
    '$' and the empty pattern included)."""
    rng = np.random.default_rng(7919 * seed + len(tp))
    extra = bytes([0x7F, 0x00, ord("$"), ord("z")])
    pool = np.frombuffer(alpha + extra, dtype=np.uint8)
    pats = [b"", b"$"]
    while len(pats) < count:
        if rng.random() < 0.7:
            m = int(rng.integers(1, min(maxlen, len(tp)) + 1))
            s = int(rng.integers(0, len(tp) - m + 1))
            pats.append(tp[s:s + m])
        else:
            m = int(rng.integers(0, maxlen + 1))
            pats.append(pool[rng.integers(0, len(pool), size=m)].tobytes())
    return pats


def pack_bits(bits) -> tuple[np.ndarray, int]:
    a = np.asarray(bits, dtype=np.uint8)
    return np.packbits(a), int(a.size)


def flat(seqs, dtype):
    offs = np.zeros(len(seqs) + 1, dtype=np.int64)
    for i, s in enumerate(seqs):
        offs[i + 1] = offs[i] + len(s)
    data = np.concatenate([np.asarray(list(s), dtype=dtype) for s in seqs]) if offs[-1] else np.zeros(0, dtype)
    return data, offs


def s2b(s: str) -> bytes:
    return s.encode("latin-1")


def run_case(mods, text: bytes, seed: int, npat: int, sample_occ: bool = True, full_wt: bool = True):
    efm, wtm, _, hoe = mods
    t = text.decode("latin-1")
    idx = efm.EnhancedFMIndex(t)
    tp = s2b(idx.text)
    out = {}
    out["text"] = np.frombuffer(text, dtype=np.uint8)
    out["sa"] = np.asarray(idx.suffix_array, dtype=np.uint32)
    out["bwt"] = np.frombuffer(s2b(idx.bwt), dtype=np.uint8)
    syms = sorted(idx.count)
    out["C_sym"] = np.asarray([ord(c) for c in syms], dtype=np.uint8)
    out["C_val"] = np.asarray([idx.count[c] for c in syms], dtype=np.int64)
    rng = np.random.default_rng(seed + 17 * len(text))
    if sample_occ:
        occ_c, occ_i, occ_v = [], [], []
        for c in syms + ["\x7f", "z"]:
            for i in rng.integers(0, len(tp) + 6, size=64):
                occ_c.append(ord(c)); occ_i.append(int(i)); occ_v.append(idx.rank(c, int(i)))
        out["occ_c"] = np.asarray(occ_c, dtype=np.uint8)
        out["occ_i"] = np.asarray(occ_i, dtype=np.int64)
        out["occ_v"] = np.asarray(occ_v, dtype=np.int64)
    alpha = bytes(sorted(set(text))) or b"a"
    pats = gen_patterns(seed, tp, alpha, npat)
    pdata, poffs = flat(pats, np.uint8)
    out["pat_data"], out["pat_offs"] = pdata, poffs
    lr = [idx.find_range(p.decode("latin-1")) for p in pats]
    out["pat_lr"] = np.asarray(lr, dtype=np.int64).reshape(-1, 2)
    locs = [idx.find(p.decode("latin-1")) for p in pats]
    ldata, loffs = flat(locs, np.int64)
    out["loc_data"], out["loc_offs"] = ldata, loffs
    if full_wt:
        wt = wtm.WaveletTree(idx.bwt)
        out["wt_m"] = np.asarray([-1 if wt.m is None else wt.m], dtype=np.int64)
        out["wt_levels"] = np.asarray([len(wt.tree)], dtype=np.int64)
        for lv, (gbits, left, right, nxt) in enumerate(wt.tree):
            bv = wt.rank_structures[lv].bit_vector
            out[f"wt{lv}_left"] = np.frombuffer(s2b("".join(left)), dtype=np.uint8)
            out[f"wt{lv}_right"] = np.frombuffer(s2b("".join(right)), dtype=np.uint8)
            out[f"wt{lv}_bits"], nb = pack_bits(bv)
            out[f"wt{lv}_nbits"] = np.asarray([nb], dtype=np.int64)
            out[f"wt{lv}_golomb"], ng = pack_bits(gbits)
            out[f"wt{lv}_ngolomb"] = np.asarray([ng], dtype=np.int64)
            out[f"wt{lv}_next"] = np.frombuffer(s2b("".join(nxt)), dtype=np.uint8)
            rs = wt.rank_structures[lv].rank_support
            out[f"wt{lv}_rank_last"] = np.asarray([int(rs[-1])], dtype=np.int64)
        # the reference's c-ignoring rank/select on the last level (csa/wavelet_tree.py:133-149)
        if wt.tree:
            last = wt.rank_structures[-1]
            qi = rng.integers(0, max(1, last.n), size=16)   # rank(i+1) must stay in range
            out["wtq_i"] = qi.astype(np.int64)
            out["wtq_rank"] = np.asarray([int(wt.rank("A", int(i))) for i in qi], dtype=np.int64)
            out["wtq_select"] = np.asarray([int(wt.select("A", int(i))) for i in qi], dtype=np.int64)
    ent = [hoe.calculate_high_order_entropy(t, k) for k in range(4)]
    out["entropy"] = np.asarray(ent, dtype=np.float64)
    return out


def kats(mods):
    efm, wtm, sam, hoe = mods
    k = {}
    with contextlib.redirect_stdout(io.StringIO()):
        k["ksa_banana"] = sam.ksa("banana")
    for word in ["banana", "mississippi", "ACGTTGCAAC", "", "a", "$", "this is an example text"]:
        idx = efm.EnhancedFMIndex(word)
        ent = {"sa": list(idx.suffix_array), "bwt": idx.bwt, "C": dict(idx.count), "find": {}, "find_range": {}}
        for p in ["ana", "", "z", "issi", "ss", "i$", "p$", "$", "AC", "CAA", "example", "a", "$$"]:
            ent["find"][p] = idx.find(p)
            ent["find_range"][p] = list(idx.find_range(p))
        wt = wtm.WaveletTree(idx.bwt)
        ent["wt_bwt"] = [{"left": "".join(L), "right": "".join(R),
                          "bits": "".join(str(int(b)) for b in wt.rank_structures[i].bit_vector),
                          "golomb": "".join(map(str, G))} for i, (G, L, R, _) in enumerate(wt.tree)]
        ent["wt_bwt_m"] = wt.m
        k[word] = ent
    demo = "this is an example text"
    wt = wtm.WaveletTree(demo)
    k["demo_wt_compress"] = wt.compress()
    k["demo_wt_bits"] = ["".join(str(int(b)) for b in rs.bit_vector) for rs in wt.rank_structures]
    k["demo_wt_m"] = wt.m
    k["entropy_demo"] = [hoe.calculate_high_order_entropy(demo, kk) for kk in range(5)]
    return k


def main():
    mods = _import_reference()
    with open(os.path.join(HERE, "kat.json"), "w") as f:
        json.dump(kats(mods), f, indent=1, sort_keys=True)

    arrays = {}
    cases = []
    for seed in SEEDS:
        for sigma in ALPHABETS:
            for n in SIZES:
                name = f"s{seed}_a{sigma}_n{n}"
                text = gen_text(seed, sigma, n)
                out = run_case(mods, text, seed, npat=200)
                for kk, v in out.items():
                    arrays[f"{name}/{kk}"] = v
                cases.append(name)
    arrays["cases"] = np.asarray(cases)
    np.savez_compressed(os.path.join(HERE, "random_cases.npz"), **arrays)

    large = {}
    lnames = []
    for sigma in (4, 256):
        for n in (1 << 16, 1 << 17):
            name = f"large_a{sigma}_n{n}"
            text = gen_text(9, sigma, n)
            efm = mods[0]
            idx = efm.EnhancedFMIndex(text.decode("latin-1"))
            sa = np.asarray(idx.suffix_array, dtype=np.uint32)
            bwt = s2b(idx.bwt)
            large[f"{name}/text"] = np.frombuffer(text, dtype=np.uint8)
            large[f"{name}/sa_sha256"] = np.asarray([hashlib.sha256(sa.astype("<u4").tobytes()).hexdigest()])
            large[f"{name}/bwt_sha256"] = np.asarray([hashlib.sha256(bwt).hexdigest()])
            rng = np.random.default_rng(n + sigma)
            si = np.sort(rng.integers(0, len(sa), size=4096))
            large[f"{name}/sa_i"] = si.astype(np.int64)
            large[f"{name}/sa_v"] = sa[si].astype(np.int64)
            tp = s2b(idx.text)
            pats = []
            for _ in range(1000):
                m = 16 if sigma == 4 else 6
                s = int(rng.integers(0, len(tp) - m + 1))
                pats.append(tp[s:s + m])
            pdata, poffs = flat(pats, np.uint8)
            large[f"{name}/pat_data"], large[f"{name}/pat_offs"] = pdata, poffs
            lr = [idx.find_range(p.decode("latin-1")) for p in pats]
            large[f"{name}/pat_lr"] = np.asarray(lr, dtype=np.int64).reshape(-1, 2)
            locs = [idx.find(p.decode("latin-1")) for p in pats]
            ld, lo = flat(locs, np.int64)
            large[f"{name}/loc_data"], large[f"{name}/loc_offs"] = ld, lo
            lnames.append(name)
            del idx
    large["cases"] = np.asarray(lnames)
    np.savez_compressed(os.path.join(HERE, "large_cases.npz"), **large)
    print("wrote", len(cases), "random cases and", len(lnames), "large cases")


if __name__ == "__main__":
    main()
