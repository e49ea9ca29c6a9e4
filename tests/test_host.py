"""Host-side logic of the package (no GPU): codec, pattern packing, the reference's
rank/select and Golomb-Rice classes, shard slice bounds."""
import numpy as np
import pytest

from conftest import wt_golden_levels
from csa.wavelet_tree import GolombRiceEncoder, SuccinctRankSelect
from hkcsa import TextCodec, pack_patterns
from hkcsa.shard import slice_bounds
from oracle import oracle


def test_codec_identity_latin1():
    c = TextCodec("banana$")
    assert c.identity
    assert c.encode_text("banana$") == b"banana$"
    assert c.encode_pattern("an") == b"an"
    assert c.encode_pattern("€") is None
    assert c.decode(b"nab") == "nab"


def test_codec_remap_preserves_order():
    t = "αβγα$"
    c = TextCodec(t)
    assert not c.identity
    enc = c.encode_text(t)
    assert sorted(enc) == [c.encode_symbol(ch) for ch in sorted(t)]
    assert c.decode(enc) == t
    assert c.encode_pattern("x") is None


def test_codec_parts_zero_copy_and_remap():
    """TextCodec.parts: T' = text + sentinel as pieces without the concatenation; the identity case is
    a view of the str's own storage (no copy), a >= 256 code-point remap is vectorised and equals the
    dense sorted-order remap (csa/wavelet_tree.py:68 order) of text + '$'."""
    from hkcsa import codec
    rng = np.random.default_rng(4)
    for t in ["banana", "caf\xe9 cr\xe8me", "", "x" * 1000]:
        c = TextCodec(t, "$")
        assert c.identity
        p = c.parts(t, "$")
        assert b"".join(x.tobytes() for x in p) == (t + "$").encode("latin-1")
        if len(t) > 16 and codec._LAYOUT is not None:
            assert not p[0].flags.owndata          # a view of the str itself
    cps = np.array([0x3B1, 0x3B2, 0x3B3, 0x20AC, 0x1F600, 0x41, 0xE9], dtype=np.uint32)
    for kind_t in [cps[:4], cps]:                  # UCS2 and UCS4 storage
        t = "".join(chr(int(x)) for x in kind_t[rng.integers(0, len(kind_t), size=5000)])
        c = TextCodec(t, "$")
        assert not c.identity
        enc = b"".join(x.tobytes() for x in c.parts(t, "$"))
        syms = sorted(set(t + "$"))
        assert enc == bytes(syms.index(ch) for ch in t + "$")
        assert c.decode(enc) == t + "$"
        assert c.encode_text(t) == enc[:-1]
    # lone surrogates survive the round trip
    t = "a\ud800b\udfffa$"
    c = TextCodec(t)
    assert c.decode(c.encode_text(t)) == t


def test_codec_too_many_symbols():
    with pytest.raises(ValueError):
        TextCodec("".join(chr(0x400 + i) for i in range(300)))


def test_pack_patterns():
    d, o = pack_patterns([b"ab", b"", b"xyz"])
    assert d.tobytes() == b"abxyz"
    assert list(o) == [0, 2, 2, 5]
    d, o = pack_patterns([])
    assert len(d) == 0 and list(o) == [0]


def test_rank_select_and_golomb_vs_golden(random_cases):
    checked = 0
    for name in random_cases.names:
        c = random_cases.get(name)
        for g in wt_golden_levels(c):
            enc = GolombRiceEncoder(g["bits"])
            assert np.array_equal(np.asarray(enc.encode(g["bits"]), np.uint8), g["golomb"]), name
            rs = SuccinctRankSelect(g["bits"])
            assert int(rs.rank(len(g["bits"]))) == int(g["bits"].sum())
            checked += 1
        if "wtq_i" in c:
            gl = wt_golden_levels(c)[-1]
            rs = SuccinctRankSelect(gl["bits"])
            for i, r, s in zip(c["wtq_i"], c["wtq_rank"], c["wtq_select"]):
                assert int(rs.rank(int(i) + 1)) == int(r), name
                assert int(rs.select(int(i))) == int(s), name
    assert checked > 100


def test_golomb_m_matches_kat(kat):
    for word in ["banana", "mississippi", "ACGTTGCAAC"]:
        lv = kat[word]["wt_bwt"]
        if lv:
            bits = [int(x) for x in lv[0]["bits"]]
            assert GolombRiceEncoder(bits).m == kat[word]["wt_bwt_m"]


@pytest.mark.parametrize("nranks,alpha", [(1, b"ACGT"), (2, b"ACGT"), (3, b"ACGT"), (8, b"ACGT"),
                                          (2, b"AC$GT"), (3, bytes(range(0x20, 0x7F))), (8, b"AC$GT")])
def test_slice_bounds_tile_the_sa(nranks, alpha):
    """Partition histogram -> splitters -> exact below-counts -> slices tile [0, n) near n/N each.
    ACGT (+ the unique '$'): keyed radix 4, the exact coarse histogram; '$' inside the text / printable
    bytes: the sampled partition key."""
    from hkcsa.shard import split_buckets
    t = oracle.synth_text(20000, alpha, seed=4)
    keyed = oracle.shard_scheme(t) > 0
    assert keyed == (alpha == b"ACGT")
    h = oracle.shard_hist(t, 0, len(t))
    assert int(h.sum()) == (len(t) if keyed else (len(t) + 63) // 64)
    B = split_buckets(h, nranks, aligned=keyed)
    below = sum(oracle.shard_below(t, len(t) * r // nranks, len(t) * (r + 1) // nranks, B) for r in range(nranks))
    assert np.array_equal(below, oracle.shard_below(t, 0, len(t), B))
    b = slice_bounds(below, nranks)
    if keyed:   # exact histogram: the bounds are its prefix sums at the splitters
        cum = np.concatenate(([0], np.cumsum(h)))
        assert [int(cum[x]) for x in B] == [int(x) for x in below]
    assert b[0][0] == 0 and b[-1][1] == len(t)
    for (lo, hi), (lo2, _) in zip(b, b[1:]):
        assert hi == lo2 and lo <= hi
    # slices stay near n/N for a high-entropy text
    for lo, hi in b:
        assert abs((hi - lo) - len(t) / nranks) < 0.08 * len(t) + 64


def test_csa_sample_rate():
    from csa.csa import sample_rate
    assert sample_rate(2**30 + 1, 0.5) == 6       # ceil(sqrt(30.000...))
    assert sample_rate(2**20 + 1, 1.0) == 21
    assert sample_rate(1000, 0) == 1
    assert sample_rate(1, 0.5) == 1


def test_generate_random_patterns_reference_semantics():
    """tests/test_patterns.py:3-9: one substring per length, clipped to the text, at a random
    offset — here seedable; the seeded draw equals the reference's draw from random.Random(seed)."""
    import random
    from utils.patterns import generate_random_patterns, sample_substrings
    text = "mississippi$" * 7
    lens = [1, 5, 10, 50, 100, 1000]
    pats = generate_random_patterns(text, lens, seed=7)
    assert [len(p) for p in pats] == [min(n, len(text)) for n in lens]
    assert all(p in text for p in pats)
    rng = random.Random(7)
    want = []
    for n in lens:
        a = min(n, len(text))
        s = rng.randint(0, len(text) - a)
        want.append(text[s:s + a])
    assert pats == want
    assert generate_random_patterns("", [3]) == [""]
    data, offs = sample_substrings(text.encode(), 50, 4, seed=3)
    assert len(offs) == 51 and int(offs[-1]) == len(data) == 200
    blob = text.encode()
    for i in range(50):
        assert data[offs[i]:offs[i + 1]].tobytes() in blob


def test_english_like_text_shape():
    """utils.textgen (the configs[2] stand-in): deterministic, latin-1 words with long repeats, and
    small texts whose SA the oracle's naive sort (csa/suffix_array.py:131-134) and O(n) checker agree on."""
    from oracle import oracle
    from utils.textgen import english_like, english_like_text
    a = english_like(1 << 20, seed=4)
    assert len(a) == 1 << 20 and np.array_equal(a, english_like(1 << 20, seed=4))
    assert not np.array_equal(a[:4096], english_like(1 << 20, seed=5)[:4096])
    assert ord("$") not in set(a.tolist()) and 60 <= len(np.unique(a)) <= 120
    assert b" the " in a.tobytes()
    # long repeats: some 256-byte window occurs at least twice
    w = np.lib.stride_tricks.sliding_window_view(a[: 1 << 18], 64)[::64]
    keys = {bytes(x) for x in w}
    assert len(keys) < len(w)
    t = english_like_text(20001, seed=9, copy_frac=0.5, min_copy=20, max_copy=400, vocab=200)
    assert t[-1] == ord("$") and len(t) == 20001
    sa = oracle.suffix_array(t)
    assert oracle.check_sa(t, sa) == 0
    assert english_like(0).size == 0
