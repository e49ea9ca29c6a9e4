"""The reference's class/module surface (csa.*, utils.*) running on the GPU, checked against
the known-answer vectors generated from the reference (tests/golden/kat.json)."""
import numpy as np
import pytest

from oracle import ref_port

pytestmark = pytest.mark.gpu

WORDS = ["banana", "mississippi", "ACGTTGCAAC", "", "a", "$", "this is an example text"]


@pytest.mark.parametrize("word", WORDS)
def test_enhanced_fm_index_kat(kat, word):
    from csa.enhanced_fm_index import EnhancedFMIndex
    k = kat[word]
    idx = EnhancedFMIndex(word)
    assert idx.text == word + "$"
    assert idx.suffix_array == k["sa"]
    assert idx.bwt == k["bwt"]
    assert idx.count == k["C"]
    for p, want in k["find"].items():
        assert idx.find(p) == want, p
        assert list(idx.find_range(p)) == k["find_range"][p], p
    port = ref_port.FMIndexPort(word)
    for ch in sorted(set(word + "$")) + ["\x7f", "zz"]:
        for i in [0, 1, 2, len(word), len(word) + 1, len(word) + 5, -1]:
            assert idx.rank(ch, i) == (port.occ[ch][min(i, len(word) + 1)] if ch in port.occ else 0), (ch, i)
    assert set(idx.occ.keys()) == set(port.occ.keys())
    for ch in port.occ:
        assert list(idx.occ[ch]) == port.occ[ch]


def test_wavelet_tree_kat(kat):
    from csa.wavelet_tree import WaveletTree
    demo = "this is an example text"
    wt = WaveletTree(demo)
    assert wt.compress() == kat["demo_wt_compress"]
    assert ["".join(str(int(b)) for b in rs.bit_vector) for rs in wt.rank_structures] == kat["demo_wt_bits"]
    assert wt.m == kat["demo_wt_m"]
    assert wt.decompress(wt.compress()) == demo
    for word in ["banana", "mississippi", "ACGTTGCAAC"]:
        k = kat[word]
        wt = WaveletTree(k["bwt"])
        assert len(wt.tree) == len(k["wt_bwt"])
        for (g, L, R, _), want in zip(wt.tree, k["wt_bwt"]):
            assert "".join(L) == want["left"] and "".join(R) == want["right"]
            assert "".join(map(str, g)) == want["golomb"]
        assert wt.occ("a" if word == "banana" else k["bwt"][0], len(k["bwt"])) == k["bwt"].count(
            "a" if word == "banana" else k["bwt"][0])


def test_wavelet_tree_random_cases(random_cases):
    from conftest import wt_golden_levels
    from csa.wavelet_tree import WaveletTree
    for name in random_cases.names:
        if not name.endswith(("_n64", "_n1000")):
            continue
        c = random_cases.get(name)
        wt = WaveletTree(c["bwt"].tobytes().decode("latin-1"))
        gold = wt_golden_levels(c)
        assert len(wt.tree) == len(gold), name
        for (g, L, R, nxt), rs, want in zip(wt.tree, wt.rank_structures, gold):
            assert np.array_equal(rs.bit_vector, want["bits"]), name
            assert np.array_equal(np.asarray(g, np.uint8), want["golomb"]), name
            assert "".join(L).encode("latin-1") == want["left"]
            assert "".join(R).encode("latin-1") == want["right"]
            assert "".join(nxt).encode("latin-1") == want["next"]
        if gold:
            assert wt.m == int(c["wt_m"][0])
        if "wtq_i" in c:
            for i, r, s in zip(c["wtq_i"], c["wtq_rank"], c["wtq_select"]):
                assert int(wt.rank("A", int(i))) == int(r)
                assert int(wt.select("A", int(i))) == int(s)


def test_module_functions(kat):
    from csa.bwt import bwt_transform
    from csa.suffix_array import build_suffix_array, ksa
    from utils.utils import build_count, build_occ
    assert ksa("banana") == kat["ksa_banana"]
    for word in ["banana", "mississippi", "ACGTTGCAAC"]:
        k = kat[word]
        tp = word + "$"
        sa = build_suffix_array(tp)
        assert sa == k["sa"]
        assert bwt_transform(tp, sa) == k["bwt"]
        assert build_count(tp) == k["C"]
        occ = build_occ(k["bwt"])
        assert dict((c, list(v)) for c, v in occ.items()) == ref_port.occ_table(k["bwt"])
    assert build_suffix_array("") == [] and bwt_transform("", []) == ""


def test_csa_surface():
    from csa import CSA, CompressedSuffixArray
    from csa.csa import CompressedSuffixArray as C2
    assert CompressedSuffixArray is CSA and C2 is CSA
    text = "mississippi$" * 50
    csa = CompressedSuffixArray(text, epsilon=0.5)
    port = ref_port.FMIndexPort(text)
    for p in ["ssi", "mississippi", "i$m", "x", "", "pp", "$"]:
        assert csa.locate(p) == port.find(p)
        l, r = port.find_range(p)
        assert csa.count(p) == (0 if l == -1 else r - l + 1)
    assert csa.count_many(["ssi", "x"]) == [csa.count("ssi"), 0]
    assert csa.locate_many(["ssi"]) == [csa.locate("ssi")]
    for i, j in [(0, 5), (3, 3), (-4, None), (10, 2), (0, 10 ** 9), (-10 ** 9, 4)]:
        assert csa.extract(i, j) == text[i:j]
    # epsilon=0.5 compacts: SA, BWT array and text left HBM; answers come from LF walks
    sp = csa.space()
    assert sp["sa"] == 0 and sp["text"] == 0 and sp["sampled"] == 1 and sp["sample_rate"] == csa.sample_rate
    assert csa.suffix_array == port.suffix_array and csa.bwt == port.bwt
    full = CompressedSuffixArray(text, epsilon=0.5, compact=False)
    assert full.space()["sa"] > 0 and full.locate("ssi") == csa.locate("ssi")
    for eps in (0, 1.0):
        c = CompressedSuffixArray(text, epsilon=eps)
        assert c.locate("issi") == port.find("issi")


def test_high_order_entropy_dropin(kat, random_cases):
    from csa.high_order_entropy import calculate_high_order_entropy as hk
    demo = "this is an example text"
    for k, v in enumerate(kat["entropy_demo"]):
        assert hk(demo, k) == pytest.approx(v, rel=1e-9, abs=1e-12)
    assert hk("", 2) == 0 and hk("abc", -1) == 0 and hk("ab", 2) == 0 and hk("ab", 5) == 0
    for name in random_cases.names[::7]:
        c = random_cases.get(name)
        t = c["text"].tobytes().decode("latin-1")
        for k in range(4):
            assert hk(t, k) == pytest.approx(float(c["entropy"][k]), rel=1e-9, abs=1e-12), (name, k)


def test_unicode_text_remap():
    from csa.enhanced_fm_index import EnhancedFMIndex
    text = "αβγαβ€αβ"
    idx = EnhancedFMIndex(text)
    port = ref_port.FMIndexPort(text)
    assert idx.suffix_array == port.suffix_array
    assert idx.bwt == port.bwt
    assert idx.count == port.count
    for p in ["αβ", "β€", "€α", "z", "ααα"]:
        assert idx.find(p) == port.find(p)


def test_run_full_benchmark_harness(capsys):
    """tests/benchmark.py:54-106 over the GPU CSA: the reference's fields, one locate per length and
    iteration, occurrence counts equal to the restatement's find()."""
    from utils.benchmark import print_benchmark_summary, run_full_benchmark
    text = "mississippi$" * 1000
    res = run_full_benchmark(text, pattern_lengths=[5, 10, 50, 100, 500, 1000], iterations=2, seed=11)
    assert res.construction_time > 0 and res.total_time >= res.construction_time
    assert sorted(res.pattern_times) == [5, 10, 50, 100, 500, 1000]
    assert res.peak_memory >= res.construction_memory and res.device_bytes > 0
    from utils.patterns import generate_random_patterns
    port = ref_port.FMIndexPort(text)
    for p in generate_random_patterns(text, [5, 10, 50, 100, 500, 1000], seed=11):
        assert res.occurrences[len(p)] == len(port.find(p))
    print_benchmark_summary(res)
    out = capsys.readouterr().out
    assert "=== Benchmark Summary ===" in out and "Peak Memory" in out


def test_locate_batch_host_boundary():
    """hkcsa_locate_batch from host buffers (EnhancedFMIndex.find, csa/enhanced_fm_index.py:15-19):
    one call when the caller's buffer is large enough, HKCSA_E_RANGE with the CSR sizes (nothing
    gathered) when it is not, sizes only with a NULL position buffer."""
    import ctypes as C

    import hkcsa
    from hkcsa import _native as N
    from hkcsa.index import _ptr, pack_patterns
    from oracle import oracle
    text = oracle.synth_text(1 << 16, b"ACGT", seed=12)
    dev = hkcsa.DeviceIndex.from_bytes(text, device=0)
    dev.build_all()
    fm = oracle.FM(text)
    pats = [b"A", b"ACG", b"", b"TTTTTTTTTTTTTTTTTTTT", b"$", b"GATTACA"] + \
        [text[s:s + 9].tobytes() for s in range(0, 60000, 997)]
    data, offs = pack_patterns(pats)
    want = fm.find(pats)
    for cap in (None, 0, 5, sum(map(len, want))):
        occ, pos = dev.locate_batch(data, offs, cap=cap)
        assert [list(map(int, pos[occ[i]:occ[i + 1]])) for i in range(len(pats))] == want, cap
    occ = np.zeros(len(pats) + 1, dtype=np.uint64)
    small = np.zeros(3, dtype=np.uint64)
    rc = dev.lib.hkcsa_locate_batch(dev.h, _ptr(data), _ptr(offs), len(pats), _ptr(occ), _ptr(small), 3)
    assert rc == N.E_RANGE and int(occ[-1]) == sum(map(len, want)) and not small.any()
    occ[:] = 0
    assert dev.lib.hkcsa_locate_batch(dev.h, _ptr(data), _ptr(offs), len(pats), _ptr(occ), None, 0) == 0
    assert [int(occ[i + 1] - occ[i]) for i in range(len(pats))] == [len(w) for w in want]
    dev.close()


def test_batch_calls_chunked_upload_and_bad_offsets():
    """hkcsa_count_batch / hkcsa_locate_batch over 600,000 patterns (three upload chunks of 2^18, each counted
    while the next one uploads) equal the device-resident query set on the same patterns, and the oracle on
    the patterns at the chunk seams; offsets out of order or past offs[P] fail with HKCSA_E_INVALID (the
    count kernel flags them, no pattern byte outside the batch is read) and leave the handle usable."""
    import hkcsa
    from hkcsa import _native as N
    from hkcsa.index import _ptr
    from oracle import oracle
    text = oracle.synth_text(1 << 18, b"ACGT", seed=31)
    dev = hkcsa.DeviceIndex.from_bytes(text, device=0)
    dev.build_all()
    rng = np.random.default_rng(5)
    P = 600_000
    lens = rng.integers(8, 17, P).astype(np.uint64)   # (short patterns would each locate a large share of all n suffixes)
    starts = rng.integers(0, len(text) - 16, P)
    offs = np.zeros(P + 1, np.uint64)
    offs[1:] = np.cumsum(lens)
    tot = int(offs[-1])
    src = np.repeat(starts, lens.astype(np.int64)) + (np.arange(tot) - np.repeat(offs[:-1].astype(np.int64),
                                                                                lens.astype(np.int64)))
    data = np.ascontiguousarray(np.asarray(text)[src], dtype=np.uint8)
    lr = np.empty(2 * P, np.int64)
    assert dev.lib.hkcsa_count_batch(dev.h, _ptr(data), _ptr(offs), P, _ptr(lr)) == 0
    q = dev.queries(data=data, offs=offs)
    q.count()
    want_lr = q.ranges().reshape(-1)
    q_offs, q_pos = q.positions()
    q.close()
    assert np.array_equal(lr, want_lr)
    occ, pos = dev.locate_batch(data, offs)
    assert np.array_equal(occ, q_offs) and np.array_equal(pos, q_pos)
    fm = oracle.FM(text)
    seam = [i for c in (1 << 18, 2 << 18) for i in range(c - 3, c + 3)] + [0, P - 1]
    pats = [data[int(offs[i]):int(offs[i + 1])].tobytes() for i in seam]
    got = [list(map(int, pos[occ[i]:occ[i + 1]])) for i in seam]
    assert got == fm.find(pats)
    bad = offs.copy()
    bad[400_000] = bad[400_002]                 # pattern 400,001 ends before it starts
    assert dev.lib.hkcsa_count_batch(dev.h, _ptr(data), _ptr(bad), P, _ptr(lr)) == N.E_INVALID
    occ2 = np.empty(P + 1, np.uint64)
    assert dev.lib.hkcsa_locate_batch(dev.h, _ptr(data), _ptr(bad), P, _ptr(occ2), None, 0) == N.E_INVALID
    bad = offs.copy()
    bad[P - 1] = bad[P] + 64                    # past the last byte (and out of order with offs[P])
    assert dev.lib.hkcsa_count_batch(dev.h, _ptr(data), _ptr(bad), P, _ptr(lr)) == N.E_INVALID
    assert dev.lib.hkcsa_count_batch(dev.h, _ptr(data), _ptr(offs), P, _ptr(lr)) == 0
    assert np.array_equal(lr, want_lr)
    dev.close()


def test_unicode_64MiB_text_remap():
    """A 64 MiB str with code points >= 256 (Cyrillic letters in English-like text, as a UTF-8 corpus read
    by tests/dataset_benchmark.py:22 would give) through EnhancedFMIndex (csa/enhanced_fm_index.py:8-13):
    the vectorised dense remap, the SA (O(n) checker) and BWT against the oracle on the remapped bytes,
    and 2,000 20-symbol find_range / 200 find calls against the oracle FM index."""
    from csa.enhanced_fm_index import EnhancedFMIndex
    from oracle import oracle
    from utils.textgen import english_like
    base = english_like(64 << 20, seed=5)
    lut = np.arange(256, dtype=np.uint32)
    lut[ord("a"):ord("z") + 1] = 0x430 + np.arange(26, dtype=np.uint32)
    cps = lut[base]
    text = cps.astype("<u4").tobytes().decode("utf-32-le")
    del base
    idx = EnhancedFMIndex(text)
    syms, enc = np.unique(np.concatenate([cps, np.array([ord("$")], np.uint32)]), return_inverse=True)
    enc = enc.astype(np.uint8)
    dev = idx.device_index
    sa = dev.sa()
    assert oracle.check_sa(enc, sa) == 0
    fm = oracle.FM(enc, sa)
    assert np.array_equal(dev.bwt(), fm.bwt)
    assert idx.count == {chr(int(c)): int(fm.C[i]) for i, c in enumerate(syms)}
    rng = np.random.default_rng(6)
    starts = rng.integers(0, len(text) - 20, size=2000)
    pats = [text[s:s + 20] for s in starts]
    want = fm.find_range([enc[s:s + 20].tobytes() for s in starts])
    assert np.array_equal(idx.find_range_many(pats), want)
    for p, s in zip(pats[:200], starts[:200]):
        assert idx.find(p) == fm.find([enc[s:s + 20].tobytes()])[0]
    assert idx.find_range("абz一") == (-1, -1)   # a symbol the text cannot hold
