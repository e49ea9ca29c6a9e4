"""GPU parity at the sizes bench.py times ("what's missing" #2).

* configs[4] at N = 1: the 4 GiB + 1 sigma=4 text on one handle (hkcsa_build_sa builds it as slices of
  ~2^30 suffixes inside the library, 64-bit positions), iid and with long planted repeats;
* the geometry of every N >= 2 weak-scaling rank: a 2 GiB + 1 text split over two emulated ranks
  (two ~1 GiB slices, host-driven two-phase API);
* the configs[2] stand-in shape: 200 MiB of iid printable bytes (sigma = 95), full build, 20k
  batched 20-symbol counts.

Each concatenated SA is checked by the O(n) oracle checker (a checked SA is build_suffix_array's
output, csa/suffix_array.py:131-134 — the SA is unique), the BWT against the oracle's gather
(csa/bwt.py:3-13) and the counts against the oracle FM index (csa/enhanced_fm_index.py:21-32).
"""
import os
import sys
import time

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu

_T0 = [time.perf_counter()]


def _say(msg):
    """Progress on stdout (run with -s): the 4 GiB checks spend minutes in host-side oracle work."""
    print(f"  [{time.perf_counter() - _T0[0]:7.1f} s] {msg}", flush=True)

if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


@pytest.fixture(scope="module")
def hk():
    import hkcsa
    if hkcsa.device_count() < 1:
        pytest.fail("no GPU visible: the HIP path is required (there is no CPU fallback)")
    return hkcsa


def test_config4_4GiB_single_handle_build(hk):
    """configs[4]'s 4 GiB + 1 text on ONE handle (VERDICT r3 missing #1): hkcsa_build_all builds the full
    u64 SA and BWT in HBM (slices inside the library), checked by the O(n) checker and the oracle BWT;
    then the wavelet tree, locate with the full SA, CompressedSuffixArray's epsilon = 0.5 samples,
    compaction (SA, BWT and text released) and the same locate by LF walks, SA rows and an extract
    across 2^32: identical answers.  (csa/suffix_array.py:131-134, csa/enhanced_fm_index.py:8-13,
    tests/benchmark.py:25,32)"""
    from csa.csa import sample_rate
    from oracle import oracle
    n = (1 << 32) + 1
    _T0[0] = time.perf_counter()
    dev = hk.DeviceIndex.synthetic(n, b"ACGT", seed=2)
    dev.build_all()
    info = dev.build_info()
    _say(f"built SA + BWT + WT, info {info[:10]}")
    assert info[7] & 4, info[:10]                 # keyed coarse slices
    sa = dev.sa()
    _say("SA downloaded")
    text = oracle.synth_text(n, b"ACGT", seed=2)
    assert oracle.check_sa(text, sa) == 0
    _say("SA checked")
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa))
    _say("BWT checked")
    del text
    rng = np.random.default_rng(4)
    win = dev.text((1 << 32) - (1 << 20), (1 << 32))
    starts = rng.integers(0, len(win) - 13, size=400)
    pats = [win[s:s + 12].tobytes() for s in starts] + [b"ACGTACGTACGTACGTACGT", b"$", b""]
    offs_full, pos_full = dev.locate(pats)
    tail = dev.text((1 << 32) - 100, (1 << 32) + 1)
    rows = rng.integers(0, n, size=64)
    rate = sample_rate(n, 0.5)
    dev.build_samples(rate)
    dev.compact()
    _say("samples + compact")
    sp = dev.space()
    assert sp["sa"] == 0 and sp["text"] == 0 and sp["sample_rate"] == rate
    offs, pos = dev.locate(pats)
    assert np.array_equal(offs, offs_full) and np.array_equal(pos, pos_full)
    for r in rows:
        assert int(dev.sa(int(r), int(r) + 1)[0]) == int(sa[r])
    assert dev.extract((1 << 32) - 100, (1 << 32) + 1) == tail.tobytes()
    _say("sampled locate / rows / extract checked")
    dev.close()


def test_4GiB_planted_repeats_single_handle(hk):
    """A 4 GiB + 1 text with long planted repeats (copies of 10 KiB - 4 MiB passages, one 64 MiB passage
    twice) on one handle: ties outlast the slices' chunk rounds and the cross-slice prefix doubling over
    the full ISA finishes them; the O(n) checker and the oracle BWT."""
    from oracle import oracle
    n = (1 << 32) + 1
    _T0[0] = time.perf_counter()
    text = oracle.synth_text(n, b"ACGT", seed=6)
    rng = np.random.default_rng(6)
    for _ in range(48):
        L = int(rng.integers(10 << 10, 4 << 20))
        src = int(rng.integers(0, n - 1 - L))
        dst = int(rng.integers(0, n - 1 - L))
        text[dst:dst + L] = text[src:src + L].copy()
    text[(3 << 30):(3 << 30) + (64 << 20)] = text[(1 << 30):(1 << 30) + (64 << 20)].copy()
    _say("text planted")
    dev = hk.DeviceIndex.from_bytes(text, device=0)
    dev.build_sa()
    info = dev.build_info()
    _say(f"built SA + BWT, info {info[:12]}")
    assert info[2] >> 32 > 0, info[:12]        # prefix-doubling rounds ran
    sa = dev.sa()
    assert oracle.check_sa(text, sa) == 0
    _say("SA checked")
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa))
    _say("BWT checked")
    dev.close()


def test_weak_rank_geometry_2GiB_two_ranks(hk):
    from hkcsa.shard import slice_bounds, split_buckets
    from oracle import oracle
    n = (1 << 31) + 1
    devs = [hk.DeviceIndex.synthetic(n, b"ACGT", seed=5) for _ in range(2)]
    assert devs[0].shard_scheme() == 1
    g = sum(d.shard_histogram(2, r) for r, d in enumerate(devs))
    assert int(g.sum()) == n
    below = sum(d.shard_counts(g, 2, r) for r, d in enumerate(devs))
    B = split_buckets(g, 2, aligned=True)
    cum = np.concatenate(([0], np.cumsum(g)))
    assert [int(cum[b]) for b in B] == [int(x) for x in below]
    sa = np.empty(n, dtype=np.uint64)
    bwt = np.empty(n, dtype=np.uint8)
    for r, d in enumerate(devs):
        d.shard_build(g, below, 2, r)
        lo, hi = d.shard_range()
        assert (lo, hi) == slice_bounds(below, 2)[r]
        assert d.shard_status()[2] == 0
        info = d.build_info()
        assert info[7] & 4 and info[7] & 2, info[:10]   # keyed scheme, packed records
        d.shard_sa(out=sa[lo:hi])
        d.shard_bwt(out=bwt[lo:hi])
        d.close()
    text = oracle.synth_text(n, b"ACGT", seed=5)
    assert oracle.check_sa(text, sa) == 0
    assert np.array_equal(bwt, oracle.bwt(text, sa))


def test_printable_200MiB_count_20sym(hk):
    from oracle import oracle
    n = 200 * (1 << 20) + 1
    alpha = bytes(range(0x20, 0x7F))
    dev = hk.DeviceIndex.synthetic(n, alpha, seed=20)
    dev.build_all()
    sa = dev.sa()
    text = oracle.synth_text(n, alpha, seed=20)
    assert oracle.check_sa(text, sa) == 0
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa))
    rng = np.random.default_rng(21)
    starts = rng.integers(0, n - 21, size=20000)
    pats = [text[s:s + 20].tobytes() for s in starts]
    pats += [bytes(rng.integers(0x20, 0x7F, size=20).astype(np.uint8)) for _ in range(2000)]   # mostly absent
    fm = oracle.FM(text, sa)
    got = dev.count_ranges(pats)
    assert np.array_equal(got, fm.find_range(pats))
    # substrings are found (the printable alphabet holds '$': patterns with it follow the reference's
    # wrapped-row quirk, csa/bwt.py:9-10, so only '$'-free ones must occur)
    plain = np.array([b"$" not in p for p in pats[:20000]])
    assert (got[:20000, 0][plain] >= 0).all()
    dev.close()
