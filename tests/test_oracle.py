"""Pin the CPU oracle (oracle/) to the reference's own outputs (tests/golden/).

Runs without a GPU.  Every check compares a restatement with vectors produced by
importing the reference itself (tests/golden/make_golden.py).
"""
import hashlib

import numpy as np
import pytest

from conftest import locs_of, patterns_of, wt_golden_levels
from oracle import oracle, ref_port

KAT_WORDS = ["banana", "mississippi", "ACGTTGCAAC", "", "a", "$", "this is an example text"]


@pytest.mark.parametrize("word", KAT_WORDS)
def test_kat_c_oracle(kat, word):
    k = kat[word]
    tp = (word + "$").encode("latin-1")
    sa = oracle.suffix_array(tp)
    assert [int(x) for x in sa] == k["sa"]
    assert oracle.bwt(tp, sa).tobytes().decode("latin-1") == k["bwt"]
    C = oracle.count_array(tp)
    assert {chr(b): int(C[b]) for b in set(tp)} == k["C"]
    fm = oracle.FM(tp, sa)
    pats = list(k["find"].keys())
    enc = [p.encode("latin-1") for p in pats]
    assert [list(map(int, x)) for x in fm.find_range(enc)] == [k["find_range"][p] for p in pats]
    assert fm.find(enc) == [k["find"][p] for p in pats]


@pytest.mark.parametrize("word", KAT_WORDS)
def test_kat_python_port(kat, word):
    k = kat[word]
    idx = ref_port.FMIndexPort(word)
    assert idx.suffix_array == k["sa"]
    assert idx.bwt == k["bwt"]
    assert idx.count == k["C"]
    for p in k["find"]:
        assert idx.find(p) == k["find"][p]
        assert list(idx.find_range(p)) == k["find_range"][p]
    levels = ref_port.left_spine_levels(idx.bwt)
    assert len(levels) == len(k["wt_bwt"])
    for got, want in zip(levels, k["wt_bwt"]):
        assert "".join(got["left"]) == want["left"]
        assert "".join(got["right"]) == want["right"]
        assert "".join(map(str, got["bits"])) == want["bits"]
        assert "".join(map(str, got["golomb"])) == want["golomb"]
    if levels:
        assert levels[0]["m"] == k["wt_bwt_m"]


def test_kat_misc(kat):
    assert kat["ksa_banana"] == [5, 3, 1, 0, 4, 2]
    assert [int(x) for x in oracle.suffix_array(b"banana")] == kat["ksa_banana"]
    demo = "this is an example text"
    lv = ref_port.left_spine_levels(demo)
    assert [l["golomb"] for l in lv] == kat["demo_wt_compress"]
    assert ["".join(map(str, l["bits"])) for l in lv] == kat["demo_wt_bits"]
    assert lv[0]["m"] == kat["demo_wt_m"]
    for kk, v in enumerate(kat["entropy_demo"]):
        assert ref_port.high_order_entropy(demo, kk) == pytest.approx(v, rel=1e-12, abs=1e-12)


def test_random_cases_c_oracle(random_cases):
    for name in random_cases.names:
        c = random_cases.get(name)
        tp = c["text"].tobytes() + b"$"
        sa = oracle.suffix_array(tp)
        assert np.array_equal(sa, c["sa"].astype(np.uint64)), name
        assert oracle.check_sa(tp, sa) == 0
        bwt = oracle.bwt(tp, sa)
        assert np.array_equal(bwt, c["bwt"]), name
        C = oracle.count_array(tp)
        assert np.array_equal(C[c["C_sym"]], c["C_val"].astype(np.uint64)), name
        fm = oracle.FM(tp, sa)
        got = [fm.rank(int(ch), int(i)) for ch, i in zip(c["occ_c"], c["occ_i"])]
        assert got == [int(v) for v in c["occ_v"]], name
        pats = patterns_of(c)
        assert np.array_equal(fm.find_range(pats), c["pat_lr"]), name
        assert fm.find(pats) == locs_of(c), name
        # full levelwise WT: the reference's left-spine level l is the prefix of level l
        full = oracle.wt_levels(bwt)
        for lv, g in enumerate(wt_golden_levels(c)):
            assert np.array_equal(full[lv][:len(g["bits"])], g["bits"]), (name, lv)


def test_random_cases_python_wt(random_cases):
    for name in random_cases.names:
        if not name.endswith(("_n7", "_n64", "_n1000")):
            continue
        c = random_cases.get(name)
        levels = ref_port.left_spine_levels(c["bwt"].tobytes().decode("latin-1"))
        gold = wt_golden_levels(c)
        assert len(levels) == len(gold), name
        for got, want in zip(levels, gold):
            assert np.array_equal(np.asarray(got["bits"], np.uint8), want["bits"]), name
            assert np.array_equal(np.asarray(got["golomb"], np.uint8), want["golomb"]), name
        if gold:
            assert levels[0]["m"] == int(c["wt_m"][0])


def test_golomb_c_oracle_vs_golden(random_cases):
    """oracle_golomb (C) with the reference's m on every golden left-spine level."""
    seen = 0
    for name in random_cases.names:
        c = random_cases.get(name)
        for lv, g in enumerate(wt_golden_levels(c)):
            m, code = oracle.golomb(g["bits"])
            assert np.array_equal(code, g["golomb"]), (name, lv)
            if lv == 0:
                assert m == int(c["wt_m"][0]), name
            seen += 1
    assert seen > 100


def test_golomb_c_oracle_vs_port():
    rng = np.random.default_rng(5)
    cases = [np.zeros(0, np.uint8), np.ones(200, np.uint8), np.zeros(77, np.uint8),
             np.tile([1, 0], 100).astype(np.uint8)]
    for p in (0.02, 0.3, 0.5, 0.9, 0.995):
        cases.append((rng.random(3000) < p).astype(np.uint8))
    for bits in cases:
        m_ref = ref_port.golomb_m(bits.tolist()) if bits.size else 1
        for m in (None, 1, 3, 17):
            mm, code = oracle.golomb(bits, m)
            want = ref_port.golomb_encode(bits.tolist(), m_ref if m is None else m)
            assert np.array_equal(code, np.asarray(want, np.uint8))
            assert mm == (m_ref if m is None else m)


def test_entropy_numpy_oracle(random_cases, kat):
    for name in random_cases.names:
        c = random_cases.get(name)
        t = c["text"]
        for k in range(4):
            assert oracle.entropy(t, k) == pytest.approx(float(c["entropy"][k]), rel=1e-9, abs=1e-12), (name, k)
    demo = b"this is an example text"
    for kk, v in enumerate(kat["entropy_demo"]):
        assert oracle.entropy(demo, kk) == pytest.approx(v, rel=1e-9, abs=1e-12)


def test_random_cases_entropy(random_cases):
    for name in random_cases.names[:40]:
        c = random_cases.get(name)
        t = c["text"].tobytes().decode("latin-1")
        for k in range(4):
            assert ref_port.high_order_entropy(t, k) == pytest.approx(float(c["entropy"][k]), rel=1e-12, abs=1e-12)


def test_large_cases_c_oracle(large_cases):
    for name in large_cases.names:
        c = large_cases.get(name)
        tp = c["text"].tobytes() + b"$"
        sa = oracle.suffix_array(tp)
        assert hashlib.sha256(sa.astype("<u4").tobytes()).hexdigest() == str(c["sa_sha256"][0]), name
        bwt = oracle.bwt(tp, sa)
        assert hashlib.sha256(bwt.tobytes()).hexdigest() == str(c["bwt_sha256"][0]), name
        assert np.array_equal(sa[c["sa_i"]], c["sa_v"].astype(np.uint64)), name
        fm = oracle.FM(tp, sa)
        pats = patterns_of(c)
        assert np.array_equal(fm.find_range(pats), c["pat_lr"]), name
        assert fm.find(pats) == locs_of(c), name


def test_sa_checker_rejects():
    t = oracle.synth_text(5000, b"ACGT", seed=1)
    sa = oracle.suffix_array(t)
    assert oracle.check_sa(t, sa) == 0
    bad = sa.copy()
    bad[10], bad[11] = bad[11], bad[10]
    assert oracle.check_sa(t, bad) != 0
    dup = sa.copy()
    dup[3] = dup[4]
    assert oracle.check_sa(t, dup) != 0


def test_synth_text_deterministic():
    a = oracle.synth_text(1000, b"ACGT", seed=5)
    b = oracle.synth_text(1000, b"ACGT", seed=5)
    c = oracle.synth_text(1000, b"ACGT", seed=6)
    assert np.array_equal(a, b) and not np.array_equal(a, c)
    assert a[-1] == ord("$") and set(a[:-1].tobytes()) <= set(b"ACGT")


def test_oracle_occ_superblocks():
    """oracle_occ's u64 superblocks + u16 relative samples against a cumulative count, across several
    2^16 superblock seams and 64-symbol sample seams (the table that lets oracle.FM check texts past 2^32)."""
    from oracle import oracle
    rng = np.random.default_rng(12)
    t = np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=300_000)].copy()
    t[-1] = ord("$")
    fm = oracle.FM(t, sa=np.arange(len(t), dtype=np.uint64))   # any permutation gives a BWT-like sequence
    b = fm.bwt
    for c in (ord("A"), ord("T"), ord("$"), ord("Z")):
        cum = np.concatenate([[0], np.cumsum(b == c)])
        idx = np.concatenate([rng.integers(0, len(b) + 1, size=400), [0, 63, 64, 65535, 65536, 131072, len(b)]])
        for i in idx:
            assert fm.rank(c, int(i)) == int(cum[i]), (chr(c), i)
