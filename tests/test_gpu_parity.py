"""GPU parity: the HIP path (through the C-ABI) against the golden vectors generated from the
reference, and against the CPU oracle on seeded inputs; full-size configs through the O(n)
SA checker.  Every comparison is bit-exact (integer / byte / index work)."""
import hashlib

import numpy as np
import pytest

from conftest import locs_of, patterns_of, wt_golden_levels
from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hk():
    import hkcsa
    if hkcsa.device_count() < 1:
        pytest.fail("no GPU visible: the HIP path is required (there is no CPU fallback)")
    return hkcsa


def _build(hk, tp: bytes):
    dev = hk.DeviceIndex.from_bytes(tp, device=0)
    dev.build_all()
    return dev


def _check_against_golden_case(dev, c, name):
    n = len(c["sa"])
    assert np.array_equal(dev.sa(), c["sa"].astype(np.uint64)), name
    assert np.array_equal(dev.bwt(), c["bwt"]), name
    C = dev.C()
    assert np.array_equal(C[c["C_sym"]], c["C_val"].astype(np.uint64)), name
    present = set(c["C_sym"].tolist())
    ranks = dev.rank(c["occ_c"], np.minimum(c["occ_i"], np.iinfo(np.int64).max).astype(np.uint64))
    want = c["occ_v"].astype(np.uint64)
    got = np.where(np.isin(c["occ_c"], list(present)), ranks, 0)
    assert np.array_equal(got, want), name
    pats = patterns_of(c)
    assert np.array_equal(dev.count_ranges(pats), c["pat_lr"]), name
    offs, pos = dev.locate(pats)
    got_l = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(pats))]
    assert got_l == locs_of(c), name
    gold = wt_golden_levels(c)
    if gold:
        assert dev.wt_levels() >= len(gold)
    for lv, g in enumerate(gold):
        bits = dev.wt_level_bits(lv)
        assert len(bits) == n
        assert np.array_equal(bits[:len(g["bits"])], g["bits"]), (name, lv)
        m, ones, code = dev.wt_golomb(lv, len(g["bits"]))
        assert np.array_equal(code, g["golomb"]), (name, lv)
        assert ones == int(g["bits"].sum())
        if lv == 0:
            assert m == int(c["wt_m"][0]), name


def test_random_golden_cases(hk, random_cases):
    for name in random_cases.names:
        c = random_cases.get(name)
        dev = _build(hk, c["text"].tobytes() + b"$")
        _check_against_golden_case(dev, c, name)
        dev.close()


def test_large_golden_cases(hk, large_cases):
    for name in large_cases.names:
        c = large_cases.get(name)
        dev = _build(hk, c["text"].tobytes() + b"$")
        sa = dev.sa()
        assert hashlib.sha256(sa.astype("<u4").tobytes()).hexdigest() == str(c["sa_sha256"][0]), name
        assert hashlib.sha256(dev.bwt().tobytes()).hexdigest() == str(c["bwt_sha256"][0]), name
        assert np.array_equal(sa[c["sa_i"]], c["sa_v"].astype(np.uint64)), name
        pats = patterns_of(c)
        assert np.array_equal(dev.count_ranges(pats), c["pat_lr"]), name
        offs, pos = dev.locate(pats)
        got = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(pats))]
        assert got == locs_of(c), name
        dev.close()


def _texts():
    rng = np.random.default_rng(99)
    yield "dna_1M", oracle.synth_text((1 << 20) + 1, b"ACGT", seed=7)
    yield "bytes_1M", oracle.synth_text((1 << 20) + 1, bytes(range(256)), seed=8)
    yield "binary_256K", oracle.synth_text((1 << 18) + 1, b"ab", seed=9)
    yield "printable_1M", oracle.synth_text((1 << 20) + 1, bytes(range(0x20, 0x7F)), seed=10)
    # the count directory's one-level (9 <= sigma <= 16) and two-level (sigma = 17: one node a side at
    # depth 1) shapes
    yield "sigma12_300K", oracle.synth_text(300001, b"ABCDEFGHIJK", seed=11)
    yield "sigma17_300K", oracle.synth_text(300001, b"ABCDEFGHIJKLMNOP", seed=12)
    base = rng.integers(0, 4, size=5000).astype(np.uint8) + ord("A")
    rep = np.tile(base, 40)                                   # long repeats: many doubling rounds
    rep[rng.integers(0, len(rep), size=50)] = ord("T")
    yield "repeats_200K", np.concatenate([rep, [ord("$")]]).astype(np.uint8)
    yield "periodic_64K", np.frombuffer(b"abc" * 21845 + b"$", dtype=np.uint8)
    yield "run_a_20K", np.frombuffer(b"a" * 20000 + b"$", dtype=np.uint8)
    yield "single", np.frombuffer(b"$", dtype=np.uint8)
    yield "two", np.frombuffer(b"z$", dtype=np.uint8)
    yield "nul_bytes", np.frombuffer(bytes([0, 0, 1, 0, 0, 0, 1, 1, 0]) + b"$", dtype=np.uint8)


@pytest.mark.parametrize("name,text", list(_texts()))
def test_sa_bwt_wt_vs_oracle(hk, name, text):
    dev = _build(hk, text.tobytes())
    sa = dev.sa()
    assert oracle.check_sa(text, sa) == 0, name
    if len(text) <= (1 << 20) + 1 and not name.startswith(("run_", "periodic", "repeats")):
        assert np.array_equal(sa, oracle.suffix_array(text)), name
    bwt = dev.bwt()
    assert np.array_equal(bwt, oracle.bwt(text, sa)), name
    assert np.array_equal(dev.C(), oracle.count_array(text)), name
    full = oracle.wt_levels(bwt)
    assert dev.wt_levels() == len(full), name
    for lv in range(len(full)):
        assert np.array_equal(dev.wt_level_bits(lv), full[lv]), (name, lv)
    # random rank queries (incl. i > n clamp and absent symbols)
    rng = np.random.default_rng(len(text))
    cs = rng.integers(0, 256, size=2000).astype(np.uint8)
    cs[:500] = text[rng.integers(0, len(text), size=500)]
    idx = rng.integers(0, len(text) + 10, size=2000).astype(np.uint64)
    fm = oracle.FM(text, sa)
    want = np.array([fm.rank(int(c), int(i)) for c, i in zip(cs, idx)], dtype=np.uint64)
    assert np.array_equal(dev.rank(cs, idx), want), name
    # count / locate of substrings, random strings, '$' quirk patterns and the empty pattern
    n = len(text)
    pats = [b"", b"$", bytes(text[-3:])]
    for _ in range(400):
        m = int(rng.integers(1, 24))
        s = int(rng.integers(0, max(1, n - m)))
        pats.append(text[s:s + m].tobytes())
    for _ in range(100):
        m = int(rng.integers(1, 8))
        pats.append(bytes(rng.choice(np.unique(text), size=m)))
    assert np.array_equal(dev.count_ranges(pats), fm.find_range(pats)), name
    offs, pos = dev.locate(pats)
    want_l = fm.find(pats)
    got_l = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(pats))]
    assert got_l == want_l, name
    dev.close()


def _binary_level_cases():
    rng = np.random.default_rng(21)
    yield "alternating", np.tile([0, 1], 3000)
    yield "all_ones", np.ones(5000, np.int64)
    yield "no_ones", np.zeros(999, np.int64)
    yield "one_long_run", np.concatenate([np.zeros(37), np.ones(1500), np.zeros(3)])
    runs = []
    for _ in range(400):                      # runs around the 64-bit word / 448-bit line seams
        runs += [0] * int(rng.integers(1, 70)) + [1] * int(rng.choice([1, 2, 63, 64, 65, 447, 448, 449, 900]))
    yield "seams", np.array(runs)
    for p in (0.01, 0.25, 0.5, 0.75, 0.97):
        yield f"iid_{p}", (rng.random(200_003) < p).astype(np.int64)


@pytest.mark.parametrize("name,bits", list(_binary_level_cases()))
def test_golomb_level_vs_oracle(hk, name, bits):
    """Level 0 of sequence over {a} | {b, c} is the bit pattern itself: Golomb-code prefixes of it."""
    seq = np.where(np.asarray(bits) == 1, ord("b"), ord("a")).astype(np.uint8)
    dev = hk.DeviceIndex.from_bytes(np.concatenate([seq, np.array([ord("c")], np.uint8)]), device=0)
    dev.use_text_as_bwt()
    dev.build_wt()
    lvl = dev.wt_level_bits(0)
    n = len(seq)
    rng = np.random.default_rng(n)
    for nb in sorted({0, 1, 63, 64, 65, 447, 448, 449, n, n + 1, int(rng.integers(1, n + 1))}):
        ref_bits = lvl[:nb]
        for m in (0, 1, 5):
            got_m, ones, code = dev.wt_golomb(0, nb, m)
            want_m, want = oracle.golomb(ref_bits, m if m else None)
            assert got_m == want_m, (name, nb, m)
            assert ones == int(ref_bits.sum())
            assert np.array_equal(code, want), (name, nb, m)
    dev.close()


def test_repeated_builds_are_identical(hk):
    text = oracle.synth_text(300001, b"ACGT", seed=33)
    dev = hk.DeviceIndex.from_bytes(text, device=0)
    dev.build_sa()
    a = dev.sa()
    dev.build_sa()
    b = dev.sa()
    assert np.array_equal(a, b)
    assert oracle.check_sa(text, a) == 0
    dev.close()


def test_synthetic_matches_host_generator(hk):
    dev = hk.DeviceIndex.synthetic(100001, b"ACGT", seed=4)
    assert np.array_equal(dev.text(), oracle.synth_text(100001, b"ACGT", seed=4))
    dev.close()


def test_full_size_config1_256MiB(hk):
    """configs[1]: 256 MiB sigma=4 text — SA checked in O(n), BWT recomputed, counts sampled."""
    n = (1 << 28) + 1
    dev = hk.DeviceIndex.synthetic(n, b"ACGT", seed=2)
    dev.build_sa()
    dev.build_bwt()
    sa = dev.sa()
    text = oracle.synth_text(n, b"ACGT", seed=2)
    assert np.array_equal(dev.text(0, 4096), text[:4096])
    assert oracle.check_sa(text, sa) == 0
    bwt = oracle.bwt(text, sa)
    assert np.array_equal(dev.bwt(), bwt)
    # WT + Golomb-Rice code of every level at full size (§8f-1)
    dev.build_wt()
    full = oracle.wt_levels(bwt)
    for lv in range(len(full)):
        m, ones, code = dev.wt_golomb(lv)
        wm, want = oracle.golomb(full[lv])
        assert m == wm and ones == int(full[lv].sum()) and np.array_equal(code, want), lv
    dev.close()


def _sampled_queries(text, sa, rng, P=2000):
    n = len(text)
    pats = [b"", b"$", bytes(text[-3:])]
    for _ in range(P):
        m = int(rng.integers(1, 24))
        s = int(rng.integers(0, n - m))
        pats.append(text[s:s + m].tobytes())
    for _ in range(200):
        pats.append(bytes(rng.integers(0, 256, size=int(rng.integers(1, 5))).astype(np.uint8)))
    return pats


def test_full_size_bench_1GiB_sigma4(hk):
    """The bench step's own geometry (1 GiB sigma=4, D=16 bucket bits, ~1M ties): SA by the O(n)
    checker (a checked SA is build_suffix_array's output), BWT recomputed, sampled count / locate /
    rank against the oracle FM index over the checked SA."""
    n = (1 << 30) + 1
    dev = hk.DeviceIndex.synthetic(n, b"ACGT", seed=2)
    dev.build_sa()
    dev.build_bwt()
    info = dev.build_info()
    assert info[7] == 2 and info[4] > 0, info[:10]   # bucket path with packed records, LDS work items
    sa = dev.sa()
    text = oracle.synth_text(n, b"ACGT", seed=2)
    assert oracle.check_sa(text, sa) == 0
    bwt = oracle.bwt(text, sa)
    assert np.array_equal(dev.bwt(), bwt)
    dev.build_wt()
    fm = oracle.FM(text, sa)
    rng = np.random.default_rng(5)
    pats = _sampled_queries(text, sa, rng)
    assert np.array_equal(dev.count_ranges(pats), fm.find_range(pats))
    lp = [p for p in pats[3:] if len(p) >= 12][:500]   # located in full: few occurrences each
    offs, pos = dev.locate(lp)
    got = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(lp))]
    assert got == fm.find(lp)
    cs = text[rng.integers(0, n, size=3000)]
    idx = rng.integers(0, n + 5, size=3000).astype(np.uint64)
    want = np.array([fm.rank(int(c), int(i)) for c, i in zip(cs, idx)], dtype=np.uint64)
    assert np.array_equal(dev.rank(cs, idx), want)
    dev.close()


def test_full_size_config3_sigma256_1GiB(hk):
    """configs[3]: 1 GiB iid bytes (sigma=256): SA by the O(n) checker, BWT, all 8 wavelet-tree levels
    against the oracle's levelwise WT, and sampled rank / count / locate against the oracle FM index."""
    n = (1 << 30) + 1
    dev = hk.DeviceIndex.synthetic(n, bytes(range(256)), seed=4)
    dev.build_all()
    assert dev.wt_levels() == 8
    sa = dev.sa()
    text = oracle.synth_text(n, bytes(range(256)), seed=4)
    assert oracle.check_sa(text, sa) == 0
    bwt = oracle.bwt(text, sa)
    assert np.array_equal(dev.bwt(), bwt)
    del sa
    full = oracle.wt_levels(bwt)
    assert len(full) == 8
    for lv in range(8):
        assert np.array_equal(dev.wt_level_bits(lv), full[lv]), lv
    del full
    sa = dev.sa()
    fm = oracle.FM(text, sa)
    rng = np.random.default_rng(6)
    pats = _sampled_queries(text, sa, rng)
    assert np.array_equal(dev.count_ranges(pats), fm.find_range(pats))
    lp = [p for p in pats[3:] if len(p) >= 4][:500]   # located in full: few occurrences each
    offs, pos = dev.locate(lp)
    got = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(lp))]
    assert got == fm.find(lp)
    cs = rng.integers(0, 256, size=3000).astype(np.uint8)
    idx = rng.integers(0, n + 5, size=3000).astype(np.uint64)
    want = np.array([fm.rank(int(c), int(i)) for c, i in zip(cs, idx)], dtype=np.uint64)
    assert np.array_equal(dev.rank(cs, idx), want)
    dev.close()


def test_wt_and_count_beyond_4gib(hk):
    """n > 2^32, as in the replicated index every rank builds after an N >= 4 sharded build: the WT
    rank against host prefix counts (streamed), and the batched count (k-mer table + flat occ
    directory) against a host backward search driven by the WT rank (csa/enhanced_fm_index.py:21-40).
    The sequence itself stands in for the BWT (hkcsa_use_text_as_bwt)."""
    n = (1 << 32) + (1 << 28) + 1
    dev = hk.DeviceIndex.synthetic(n, b"ACGT", seed=77)
    dev.use_text_as_bwt()
    dev.build_wt()
    rng = np.random.default_rng(7)
    idx = np.concatenate([rng.integers(0, n + 1, size=40), [0, (1 << 32) - 1, 1 << 32, (1 << 32) + 1, n - 1, n]])
    idx = np.sort(idx.astype(np.uint64))
    syms = np.frombuffer(b"$ACGTx", dtype=np.uint8)
    want = np.zeros((len(idx), len(syms)), dtype=np.uint64)
    run = np.zeros(256, dtype=np.uint64)
    chunk, lo, j = 1 << 28, 0, 0
    while lo < n and j < len(idx):
        hi = min(n, lo + chunk)
        part = dev.text(lo, hi)
        while j < len(idx) and int(idx[j]) <= hi:
            k = int(idx[j]) - lo
            want[j] = (run + np.bincount(part[:k], minlength=256).astype(np.uint64))[syms]
            j += 1
        run += np.bincount(part, minlength=256).astype(np.uint64)
        lo = hi
    cs = np.repeat(syms[None, :], len(idx), axis=0).reshape(-1)
    got = dev.rank(cs, np.repeat(idx, len(syms))).reshape(len(idx), len(syms))
    assert np.array_equal(got, want)
    # batched count vs the step-by-step search over the WT rank
    tail = dev.text(n - (1 << 20), n)
    pats = [tail[s:s + m].tobytes() for s, m in zip(rng.integers(0, len(tail) - 24, size=300),
                                                  rng.integers(1, 22, size=300))]
    pats += [bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), size=m)) for m in (8, 9, 12, 16, 20)]
    pats += [b"", b"$", b"ACGTx", b"T" * 12]
    C = dev.C()
    P = len(pats)
    lo_ = np.zeros(P, dtype=np.int64)
    hi_ = np.full(P, n - 1, dtype=np.int64)
    alive = np.ones(P, dtype=bool)
    for k in range(max(len(p) for p in pats)):
        sel = np.array([alive[i] and len(pats[i]) > k for i in range(P)])
        if not sel.any():
            break
        ii = np.nonzero(sel)[0]
        c = np.array([pats[i][len(pats[i]) - 1 - k] for i in ii], dtype=np.uint8)
        rl = dev.rank(c, lo_[ii].astype(np.uint64)).astype(np.int64)
        rr = dev.rank(c, (hi_[ii] + 1).astype(np.uint64)).astype(np.int64)
        cb = C[c].astype(np.int64)
        present = np.isin(c, np.frombuffer(b"$ACGT", np.uint8))
        nl = np.where(present, cb + rl, 0)
        nr = np.where(present, cb + rr - 1, -1)
        dead = nl > nr
        lo_[ii], hi_[ii] = nl, nr
        alive[ii[dead]] = False
    exp = np.stack([np.where(alive, lo_, -1), np.where(alive, hi_, -1)], axis=1)
    assert np.array_equal(dev.count_ranges(pats), exp)
    dev.close()


@pytest.mark.parametrize("nranks,flags,alpha", [(2, 0, b"ACGT"), (3, 0, b"ACGT"), (2, 1, b"ACGT"), (4, 1, b"ACGT"),
                                               (4, 3, b"ACGT"), (5, 0, bytes(range(256))), (3, 0, b"ab"),
                                               (7, 0, b"AC$GT"), (6, 1, bytes(range(0x20, 0x7F))),
                                               (3, 3, bytes(range(256))), (3, 4, b"ACGT"), (2, 5, b"ACGT"),
                                               (3, 0, b"aaaaaaaaaaaaaaab"), (2, 1, b"aaaaaaaab"),
                                               (3, 8, b"ACGT"), (2, 9, bytes(range(0x20, 0x7F))),
                                               (4, 8, b"aaaaaaaab"), (4, 0, bytes([1, 2, 0x41, 0x42])),
                                               (3, 1, bytes([1, 2, 0x41, 0x42]))])
def test_shard_two_phase_emulated(hk, nranks, flags, alpha):
    """Ranks emulated on one GPU; flags=1 forces the 64-bit position kernels (n >= 2^32 path: split
    u32 sort values), flags=3 the whole-u64 value sort, flags=4 the global sort of each slice instead
    of its LDS bucket sorts, flags=8 multiplicative bucket bins; the skewed alphabets give slices
    whose big buckets take the global path.  Keyed coarse scheme (radix 2^lb: ACGT, ab, bytes) and
    the partition-key scheme (AC$GT, printable, aaa..ab) against the oracle's restatement of each;
    the partition-key alphabets cover the byte-image pre-test thresholds for radix 3 .. 257."""
    text = oracle.synth_text(400001, alpha, seed=12 + nranks)
    ref = oracle.suffix_array(text)
    ref_bwt = oracle.bwt(text, ref)
    devs = [hk.DeviceIndex.from_bytes(text, device=0, flags=flags) for _ in range(nranks)]
    scheme = devs[0].shard_scheme()
    assert scheme == (1 if oracle.shard_scheme(text) else 0)
    g = sum(d.shard_histogram(nranks, r) for r, d in enumerate(devs))
    if scheme:   # keyed coarse buckets: every suffix counted
        assert int(g.sum()) == len(text)
    else:        # partition key: every 64th position (hkcsa_shard_sample)
        assert int(g.sum()) == (len(text) + 63) // 64
    assert np.array_equal(g, oracle.shard_hist(text, 0, len(text)))
    from hkcsa.shard import slice_bounds, split_buckets
    B = split_buckets(g, nranks, aligned=bool(scheme))
    below = sum(d.shard_counts(g, nranks, r) for r, d in enumerate(devs))
    assert np.array_equal(below, oracle.shard_below(text, 0, len(text), B))
    assert int(below[-1]) == len(text)
    parts = []
    bounds = slice_bounds(below, nranks)
    for r, d in enumerate(devs):
        d.shard_build(g, below, nranks, r)
        assert d.shard_range() == bounds[r]
    from hkcsa.shard import emulated_doubling
    emulated_doubling(devs)     # skewed texts: slices whose ties outlast the chunk rounds
    for r, d in enumerate(devs):
        parts.append(d.shard_sa())
        lo, hi = bounds[r]
        assert np.array_equal(d.shard_bwt(), ref_bwt[lo:hi]), r
        d.close()
    assert np.array_equal(np.concatenate(parts), ref)


@pytest.mark.parametrize("n,nranks,flags,alpha", [((24 << 20) + 1, 3, 0, b"ACGT"), ((24 << 20) + 1, 2, 1, b"ACGT"),
                                                  ((24 << 20) + 1, 4, 8, b"ACGT"), ((12 << 20) + 1, 2, 0, bytes(range(256)))],
                         ids=["dna24M-3", "dna24M-2-pos64", "dna24M-4-mul", "bytes12M-2"])
def test_shard_large_slices(hk, n, nranks, flags, alpha):
    """Slices of millions of suffixes, so the slice's cursor partition runs both passes (more than 2^8
    bins) as at the bench sizes: the concatenated slices checked by the O(n) SA checker and against the
    oracle BWT; flags=1 64-bit positions, flags=8 multiplicative bins."""
    text = oracle.synth_text(n, alpha, seed=31 + nranks)
    devs, _ = _emulated_shard_build(hk, text, nranks, flags)
    sa = np.concatenate([d.shard_sa() for d in devs])
    assert oracle.check_sa(text, sa) == 0
    assert np.array_equal(np.concatenate([d.shard_bwt() for d in devs]), oracle.bwt(text, sa))
    assert max(d.build_info()[4] for d in devs) > 256   # bucket items: more than pass A's 256 digits
    for d in devs:
        d.close()


@pytest.mark.parametrize("nranks,flags", [(4, 0), (8, 1), (3, 4)])
def test_shard_keyed_dense_units(hk, nranks, flags):
    """DNA with a long run and a periodic stretch: the run's suffixes all fall in one slice, so that
    slice's pass A units hold more kept suffixes than one tile (each sub-tile then ranked and written
    on its own), its buckets exceed one LDS sort (the slice's global path) and its ties outlast the
    chunk rounds (prefix doubling with the rank exchange).  flags 4: the global sort everywhere."""
    rng = np.random.default_rng(nranks)
    dna = np.frombuffer(b"ACGT", dtype=np.uint8)
    text = np.concatenate([dna[rng.integers(0, 4, 600_000)], np.full(200_000, ord("A"), np.uint8),
                           dna[rng.integers(0, 4, 600_000)], np.frombuffer(b"CA" * 100_000, np.uint8),
                           [ord("$")]]).astype(np.uint8)
    ref = oracle.suffix_array(text)
    devs, _ = _emulated_shard_build(hk, text, nranks, flags)
    assert devs[0].shard_scheme() == 1
    parts = [d.shard_sa() for d in devs]
    assert np.array_equal(np.concatenate(parts), ref)
    assert np.array_equal(np.concatenate([d.shard_bwt() for d in devs]), oracle.bwt(text, ref))
    for d in devs:
        d.close()


def _repetitive(name):
    rng = np.random.default_rng(99)
    if name == "periodic_64K":
        return np.frombuffer(b"abc" * 21845 + b"$", dtype=np.uint8)
    if name == "run_a_20K":
        return np.frombuffer(b"a" * 20000 + b"$", dtype=np.uint8)
    if name == "repeats_200K":
        base = rng.integers(0, 4, size=5000).astype(np.uint8) + ord("A")
        rep = np.tile(base, 40)
        rep[rng.integers(0, len(rep), size=50)] = ord("T")
        return np.concatenate([rep, [ord("$")]]).astype(np.uint8)
    if name == "run_a_8M":     # longer than 200,000 refinement rounds x ~30 symbols
        return np.frombuffer(b"a" * (1 << 23) + b"$", dtype=np.uint8)
    raise KeyError(name)


def _expected_sa(name, text):
    if name.startswith("run_a"):   # 'a'^N '$': '$' < 'a', so SA = n-1, n-2, ..., 0
        return np.arange(len(text) - 1, -1, -1, dtype=np.uint64)
    return oracle.suffix_array(text)


def _emulated_shard_build(hk, text, nranks, flags):
    from hkcsa.shard import emulated_doubling
    devs = [hk.DeviceIndex.from_bytes(text, device=0, flags=flags) for _ in range(nranks)]
    g = sum(d.shard_histogram(nranks, r) for r, d in enumerate(devs))
    below = sum(d.shard_counts(g, nranks, r) for r, d in enumerate(devs))
    for r, d in enumerate(devs):
        d.shard_build(g, below, nranks, r)
    rounds = emulated_doubling(devs)
    return devs, rounds


@pytest.mark.parametrize("name,nranks,flags", [
    ("periodic_64K", 2, 0), ("periodic_64K", 5, 1), ("run_a_20K", 3, 0), ("run_a_20K", 8, 1),
    ("repeats_200K", 4, 0), ("repeats_200K", 7, 1), ("repeats_200K", 2, 3),
    ("run_a_8M", 2, 0), ("run_a_8M", 4, 1)])
def test_shard_doubling_emulated(hk, name, nranks, flags):
    """Repetitive texts whose slices stay tied after the chunk rounds: prefix doubling with the ISA
    rank exchange (hkcsa_shard_isa_segment / _updates / _apply / _round), ranks emulated on one GPU,
    u32 and u64 positions.  Bit-exact against the oracle SA (the analytic SA for the runs)."""
    text = _repetitive(name)
    ref = _expected_sa(name, text)
    devs, rounds = _emulated_shard_build(hk, text, nranks, flags)
    assert rounds > 0, "the text should need the doubling exchange"
    parts, bw = [], []
    for d in devs:
        assert d.shard_status()[2] == 0
        parts.append(d.shard_sa())
        bw.append(d.shard_bwt())
    sa = np.concatenate(parts)
    assert np.array_equal(sa, ref), name
    assert np.array_equal(np.concatenate(bw), oracle.bwt(text, ref)), name
    for d in devs:
        d.close()


@pytest.mark.parametrize("name,flags", [("dna_200K", 0), ("printable_200K", 0), ("printable_200K", 1),
                                        ("printable_200K", 3), ("periodic_64K", 0), ("run_a_20K", 1),
                                        ("repeats_200K", 0), ("run_a_8M", 0)])
def test_shard_rccl_single_rank(hk, name, flags):
    if name == "dna_200K":
        text = oracle.synth_text(200001, b"ACGT", seed=13)
    elif name == "printable_200K":
        text = oracle.synth_text(200001, bytes(range(0x20, 0x7F)), seed=13)
    else:
        text = _repetitive(name)
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=flags)
    dev.build_sa_sharded(hk.comm_unique_id(), 1, 0)
    assert dev.shard_range() == (0, len(text))
    sa = _expected_sa(name, text)
    assert np.array_equal(dev.shard_sa(), sa)
    assert np.array_equal(dev.shard_bwt(), oracle.bwt(text, sa))
    dev.close()


def _query_set(text, seed, count=600):
    rng = np.random.default_rng(seed)
    n = len(text)
    pats = [b"", b"$", bytes(text[-3:])]
    for _ in range(count):
        m = int(rng.integers(1, 24))
        st = int(rng.integers(0, max(1, n - m)))
        pats.append(text[st:st + m].tobytes())
    for _ in range(100):
        pats.append(bytes(rng.choice(np.unique(text), size=int(rng.integers(1, 6)))))
    return pats


def _check_queries(dev, text, sa, seed):
    fm = oracle.FM(text, sa)
    pats = _query_set(text, seed)
    assert np.array_equal(dev.count_ranges(pats), fm.find_range(pats))
    offs, pos = dev.locate(pats)
    got = [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(pats))]
    assert got == fm.find(pats)


@pytest.mark.parametrize("name,flags", [("dna_300K", 0), ("dna_300K", 1), ("repeats_200K", 1)])
def test_shard_replicate_queries(hk, name, flags):
    """Replicas for batched queries: RCCL all-gather of the SA slices and BWT rows (one rank), then
    the wavelet tree and count / locate (u64 SA gather with flags=1) against the oracle FM index."""
    text = oracle.synth_text(300001, b"ACGT", seed=17) if name == "dna_300K" else _repetitive(name)
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=flags)
    dev.build_sa_sharded(hk.comm_unique_id(), 1, 0)
    with pytest.raises(hk.HkcsaError):
        dev.build_wt()                      # a sharded handle holds only its slice
    dev.shard_replicate()
    dev.build_wt()
    sa = oracle.suffix_array(text)
    assert np.array_equal(dev.sa(), sa)
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa))
    _check_queries(dev, text, sa, seed=len(text))
    dev.close()


@pytest.mark.parametrize("name,rate", [("dna_300K", 6), ("repeats_200K", 3)])
def test_sampled_replicated_u64(hk, name, rate):
    """The epsilon contract over a replicated index whose SA is u64 (flags=1, as every rank's replica
    of a text with >= 2^32 suffixes): 8-byte samples, then SA, BWT, text, extract, count and locate by
    LF walks equal the full arrays and the oracle."""
    text = oracle.synth_text(300001, b"ACGT", seed=18) if name == "dna_300K" else _repetitive(name)
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=1)
    dev.build_sa_sharded(hk.comm_unique_id(), 1, 0)
    dev.shard_replicate()
    dev.build_wt()
    sa = oracle.suffix_array(text)
    dev.build_samples(rate)
    dev.compact()
    sp = dev.space()
    assert sp["sa"] == 0 and sp["text"] == 0 and sp["sampled"] == 1 and sp["sample_rate"] == rate
    n = len(text)
    assert sp["samples"] == (2 * ((n + rate - 1) // rate) + int(np.count_nonzero(text == text[-1]))) * 8
    assert np.array_equal(dev.sa(), sa)
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa))
    assert np.array_equal(dev.text(), text)
    rng = np.random.default_rng(rate)
    for _ in range(20):
        i = int(rng.integers(0, n))
        j = int(rng.integers(i, min(n, i + 5000) + 1))
        assert dev.extract(i, j) == text[i:j].tobytes()
    _check_queries(dev, text, sa, seed=n)
    dev.close()


@pytest.mark.parametrize("nranks,flags", [(3, 0), (4, 1)])
def test_shard_adopt_queries(hk, nranks, flags):
    """Host-assembled replica after an emulated sharded build (hkcsa_shard_adopt)."""
    text = oracle.synth_text(250001, b"ACGT", seed=19)
    devs, _ = _emulated_shard_build(hk, text, nranks, flags)
    sa = np.concatenate([d.shard_sa() for d in devs])
    bwt = np.concatenate([d.shard_bwt() for d in devs])
    ref = oracle.suffix_array(text)
    assert np.array_equal(sa, ref)
    dev = devs[0]
    dev.shard_adopt(sa, bwt)
    dev.build_wt()
    _check_queries(dev, text, ref, seed=nranks)
    for d in devs:
        d.close()


def test_sharded_handle_refuses_full_index_calls(hk):
    """A sharded handle holds SA[lo:hi) and its BWT rows only: whole-index calls fail with
    HKCSA_E_STATE instead of reading past the slice."""
    text = oracle.synth_text(100001, b"ACGT", seed=23)
    devs, _ = _emulated_shard_build(hk, text, 2, 0)
    d = devs[1]
    for call in (d.build_wt, lambda: d.bwt(0, 10), lambda: d.locate([b"AC"]), lambda: d.count_ranges([b"A"]),
                 lambda: d.rank(np.array([65], np.uint8), np.array([5], np.uint64)), lambda: d.sa(0, 4),
                 lambda: d.entropy(2)):
        with pytest.raises(hk.HkcsaError) as e:
            call()
        assert e.value.code == -3
    for x in devs:
        x.close()


def test_entropy_after_compact_refused(hk):
    dev = _build(hk, oracle.synth_text(5001, b"ACGT", seed=3).tobytes())
    h0 = dev.entropy(0)
    dev.build_samples(4)
    dev.compact()
    assert dev.entropy(0) == h0
    with pytest.raises(hk.HkcsaError) as e:
        dev.entropy(2)
    assert e.value.code == -3
    dev.close()


def test_entropy_keeps_wavelet_tree(hk):
    text = oracle.synth_text(20001, b"ACGT", seed=5)
    dev = hk.DeviceIndex.from_bytes(text, device=0)
    dev.build_sa()
    dev.build_wt()
    e1 = dev.entropy(3)
    dev.build_sa()          # fresh SA, then H_k rebuilds nothing and the WT stays usable
    dev.build_wt()
    assert dev.entropy(3) == e1
    _check_queries(dev, text, oracle.suffix_array(text), seed=1)
    dev.close()


def test_timing_stats(hk):
    dev = hk.DeviceIndex.synthetic(1 << 20, b"ACGT", seed=1)
    dev.timing(True)
    dev.build_sa()
    dev.synchronize()
    # whole-symbol buckets: the cursor partition (pre-pass counts, pass A builds the keys from the
    # text, pass B when the bucket has more than 8 bits), no onesweep pass over the text
    l, ms, b = dev.kernel_stats("sa_bucket_hist")
    assert l == 1 and ms > 0 and b > 0
    l, ms, b = dev.kernel_stats("radix_part_text")
    assert l == 1 and ms > 0 and b > 0
    assert dev.kernel_stats("radix_part")[0] <= 1
    assert dev.kernel_stats("radix_onesweep_text_small")[0] == 0
    l, ms, b = dev.kernel_stats("sa_bucket_sort")
    assert l == 1 and ms > 0 and b > 0
    assert dev.kernel_stats("sa_pack_keys")[0] == 0
    dev.close()


def _sampled_texts():
    yield "dna_200K", oracle.synth_text(200_001, b"ACGT", seed=41)
    yield "bytes_64K", oracle.synth_text(65_537, bytes(range(256)), seed=42)
    t = oracle.synth_text(50_001, b"AC$G", seed=43)            # '$' inside the text: LF fix rows
    yield "dollars_50K", t
    yield "periodic_30K", np.frombuffer(b"abcab" * 6000 + b"$", dtype=np.uint8)
    yield "run_5K", np.frombuffer(b"a" * 5000 + b"$", dtype=np.uint8)
    yield "two", np.frombuffer(b"z$", dtype=np.uint8)
    yield "single", np.frombuffer(b"$", dtype=np.uint8)


@pytest.mark.parametrize("name,text", list(_sampled_texts()))
@pytest.mark.parametrize("rate", [1, 3, 6, 32])
def test_sampled_compressed_mode(hk, name, text, rate):
    """hkcsa_build_samples + hkcsa_compact: SA, BWT, text, extract, count and locate answered by
    LF walks equal the full arrays (and the oracle)."""
    n = len(text)
    dev = _build(hk, text.tobytes())
    sa = dev.sa()
    bwt = dev.bwt()
    assert np.array_equal(sa, oracle.suffix_array(text)), name
    rng = np.random.default_rng(rate * 1000 + n)
    pats = [b"", b"$", bytes(text[-2:])]
    for _ in range(300):
        m = int(rng.integers(1, 12))
        s = int(rng.integers(0, max(1, n - m)))
        pats.append(text[s:s + m].tobytes())
    lr_full = dev.count_ranges(pats)
    offs_full, pos_full = dev.locate(pats)
    dev.build_samples(rate)
    dev.compact()
    sp = dev.space()
    assert sp["sa"] == 0 and sp["text"] == 0 and sp["bwt"] == 0 and sp["sampled"] == 1
    assert sp["sample_rate"] == rate
    assert np.array_equal(dev.sa(), sa), name
    assert np.array_equal(dev.bwt(), bwt), name
    assert np.array_equal(dev.text(), text), name
    for _ in range(50):
        i = int(rng.integers(0, n))
        j = int(rng.integers(i, n + 1))
        assert dev.extract(i, j) == text[i:j].tobytes(), (name, i, j)
    assert np.array_equal(dev.count_ranges(pats), lr_full), name
    offs, pos = dev.locate(pats)
    assert np.array_equal(offs, offs_full) and np.array_equal(pos, pos_full), name
    with pytest.raises(hk.HkcsaError):
        dev.build_sa()
    dev.close()


def test_compact_needs_samples(hk):
    dev = _build(hk, b"banana$")
    with pytest.raises(hk.HkcsaError):
        dev.compact()
    dev.close()


def test_entropy_golden(hk, random_cases):
    """hkcsa_entropy against calculate_high_order_entropy's own outputs (golden), k = 0..3."""
    for name in random_cases.names:
        c = random_cases.get(name)
        t = c["text"]
        if len(t) == 0:
            continue
        dev = hk.DeviceIndex.from_bytes(t.tobytes(), device=0)
        for k in range(4):
            assert dev.entropy(k) == pytest.approx(float(c["entropy"][k]), rel=1e-9, abs=1e-12), (name, k)
        dev.close()


@pytest.mark.parametrize("name,text,ks", [
    ("dna_4M", oracle.synth_text(1 << 22, b"ACGT", seed=51), [1, 2, 5, 8, 13]),
    ("bytes_1M", oracle.synth_text(1 << 20, bytes(range(256)), seed=52), [1, 2, 3]),
    ("binary_1M", oracle.synth_text(1 << 20, b"ab", seed=53), [1, 7, 20, 30]),
    ("periodic", np.frombuffer(b"abcab" * 20000, dtype=np.uint8), [1, 3, 6]),
    ("run", np.frombuffer(b"a" * 5000, dtype=np.uint8), [0, 1, 4]),
])
def test_entropy_vs_oracle(hk, name, text, ks):
    dev = hk.DeviceIndex.from_bytes(text.tobytes(), device=0)
    for k in [0] + ks:
        assert dev.entropy(k) == pytest.approx(oracle.entropy(text, k), rel=1e-9, abs=1e-12), (name, k)
    assert dev.entropy(-1) == 0.0 and dev.entropy(len(text)) == 0.0
    dev.close()


def test_entropy_64MiB(hk):
    n = 1 << 26
    dev = hk.DeviceIndex.synthetic(n, b"ACGT", seed=54, terminator=ord("A"))
    text = oracle.synth_text(n, b"ACGT", seed=54, terminator=ord("A"))
    for k in (2, 6):
        assert dev.entropy(k) == pytest.approx(oracle.entropy(text, k), rel=1e-9), k
    dev.close()
