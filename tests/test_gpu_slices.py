"""The single-GPU multi-slice build (hkcsa_build_sa for n >= 2^32 - 1; HKCSA_FLAG_SLICES at any n).

The reference's build_suffix_array has no size limit (csa/suffix_array.py:131-134), and
EnhancedFMIndex(text) / CompressedSuffixArray(text, epsilon) build whatever text they are given
(csa/enhanced_fm_index.py:8-13).  A text of >= 2^32 - 1 symbols needs 64-bit positions, which one
handle builds as slices of the final SA, one after another, straight into one full SA and BWT;
ties that outlast a slice's chunk rounds finish by prefix doubling over one ISA of the full SA.
HKCSA_FLAG_SLICES runs that path at every size, so the small texts below (repeats, runs, periodic,
printable, skewed) drive its cross-slice doubling and its non-keyed partition; the 4 GiB + 1 cases
are configs[4]'s text on one GPU.  Bit-exact checks: the SA by the oracle (or its O(n) checker),
the BWT, the WT levels, count / locate against the oracle FM index.
"""
import numpy as np
import pytest

from oracle import oracle
from test_gpu_parity import _texts

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hk():
    import hkcsa
    if hkcsa.device_count() < 1:
        pytest.fail("no GPU visible: the HIP path is required (there is no CPU fallback)")
    return hkcsa


def _check(dev, text, npat=300, seed=0, wt=True):
    sa = dev.sa()
    assert oracle.check_sa(text, sa) == 0
    bwt = dev.bwt()
    assert np.array_equal(bwt, oracle.bwt(text, sa))
    if wt:
        full = oracle.wt_levels(bwt)
        assert dev.wt_levels() == len(full)
        for lv in range(len(full)):
            assert np.array_equal(dev.wt_level_bits(lv), full[lv]), lv
    rng = np.random.default_rng(seed)
    n = len(text)
    pats = [b"", b"$", bytes(text[-3:])]
    for _ in range(npat):
        m = int(rng.integers(1, 24))
        s = int(rng.integers(0, max(1, n - m)))
        pats.append(text[s:s + m].tobytes())
    fm = oracle.FM(text, sa)
    assert np.array_equal(dev.count_ranges(pats), fm.find_range(pats))
    offs, pos = dev.locate(pats)
    assert [[int(x) for x in pos[offs[i]:offs[i + 1]]] for i in range(len(pats))] == fm.find(pats)
    return sa


@pytest.mark.parametrize("pos64", [False, True])
@pytest.mark.parametrize("name,text", list(_texts()))
def test_slices_flag_vs_oracle(hk, name, text, pos64):
    from hkcsa.index import FLAG_POS64, FLAG_SLICES
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=FLAG_SLICES | (FLAG_POS64 if pos64 else 0))
    dev.build_all()
    sa = _check(dev, text, seed=len(text))
    if len(text) <= (1 << 20) + 1 and not name.startswith(("run_", "periodic", "repeats")):
        assert np.array_equal(sa, oracle.suffix_array(text)), name
    assert dev.space()["sa"] == len(text) * (8 if pos64 else 4)
    dev.close()


def test_slices_english_like_doubling(hk):
    """24 MiB of natural-language-like text (utils/textgen.py) in 4 slices: long copies leave every slice
    tied after its chunk rounds, so the cross-slice prefix doubling over the full ISA finishes them."""
    from hkcsa.index import FLAG_POS64, FLAG_SLICES
    from utils.textgen import english_like_text
    text = english_like_text(24 * (1 << 20) + 1, seed=12, copy_frac=0.5, min_copy=100, max_copy=20000)
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=FLAG_SLICES | FLAG_POS64)
    dev.build_all()
    info = dev.build_info()
    assert info[2] >> 32 > 0, info[:12]        # doubling rounds ran
    _check(dev, text, npat=2000, seed=12)
    # the same handle again: the full arrays are reused, the result is identical
    a = dev.sa()
    dev.build_sa()
    assert np.array_equal(dev.sa(), a)
    dev.close()


def test_slices_dna_24MiB_flag_matches_default(hk):
    """The sliced build of a 24 MiB DNA text equals the default single-pass build, u32 and u64 positions."""
    from hkcsa.index import FLAG_POS64, FLAG_SLICES
    text = oracle.synth_text(24 * (1 << 20) + 1, b"ACGT", seed=13)
    ref = hk.DeviceIndex.from_bytes(text, device=0)
    ref.build_sa()
    want, wbwt = ref.sa(), ref.bwt()
    ref.close()
    assert oracle.check_sa(text, want) == 0
    for flags in (FLAG_SLICES, FLAG_SLICES | FLAG_POS64):
        dev = hk.DeviceIndex.from_bytes(text, device=0, flags=flags)
        dev.build_sa()
        assert np.array_equal(dev.sa(), want), flags
        assert np.array_equal(dev.bwt(), wbwt), flags
        dev.close()


@pytest.mark.parametrize("var", ["HKCSA_BS_TRACE", "HKCSA_SL_TRACE"])
def test_trace_builds_identical(hk, var, monkeypatch, capfd):
    """The two diagnostic switches the library still reads: phase-stamped builds of
    the bucket sort / the slice pass A.  They print cycle stamps and must leave the result unchanged."""
    from hkcsa.index import FLAG_SLICES
    text = oracle.synth_text(8 * (1 << 20) + 1, b"ACGT", seed=14)
    want = oracle.suffix_array(text)
    monkeypatch.setenv(var, "1")
    for flags in (0, FLAG_SLICES):
        dev = hk.DeviceIndex.from_bytes(text, device=0, flags=flags | 16)   # 16: HKCSA_FLAG_MAX_BUCKETS
        dev.build_sa()
        assert np.array_equal(dev.sa(), want), flags
        assert np.array_equal(dev.bwt(), oracle.bwt(text, want)), flags
        dev.close()
    err = capfd.readouterr().err
    assert "trace]" in err


@pytest.mark.parametrize("rec", ["1", "0"])
@pytest.mark.parametrize("alpha,n", [(b"ACGT", 8 << 20), (b"ab", 3 << 20), (b"ACGTNRYK", 5 << 20),
                                     (b"ACGT", 1 << 16)])
def test_record_sort_switch_identical(hk, rec, alpha, n, monkeypatch, capfd):
    """HKCSA_BS_REC=0 (read per call) keeps the fast LDS sort where the record-plane sort would run; both
    give the oracle's SA and BWT.  Small texts have the sym field below bit 32 (the u64 prologue), so this
    covers the non-X32 record sort; the trace line names the sort that ran."""
    text = oracle.synth_text(n + 1, alpha, seed=len(alpha) + n % 97)
    want = oracle.suffix_array(text)
    monkeypatch.setenv("HKCSA_BS_REC", rec)
    monkeypatch.setenv("HKCSA_BS_TRACE", "1")
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=16)   # 16: HKCSA_FLAG_MAX_BUCKETS
    dev.build_sa()
    assert np.array_equal(dev.sa(), want)
    assert np.array_equal(dev.bwt(), oracle.bwt(text, want))
    dev.close()
    err = capfd.readouterr().err
    if rec == "0":
        assert "record-plane" not in err, err[-400:]
    elif alpha == b"ACGT" and n >= 1 << 20:   # (sigma 2 runs 1024-thread items here: the fast sort)
        assert "record-plane" in err, err[-400:]


@pytest.mark.parametrize("nranks", [2, 3, 8])
@pytest.mark.parametrize("alpha", [b"ACGT", bytes(range(256)), b"ab"])
def test_keyed_below_rule_matches_host(hk, nranks, alpha):
    """the keyed scheme's slice bounds (hkcsa_build_sa_sharded's `below` from the exact coarse
    histogram alone: splitters(..., aligned) + prefix sums, the rule build_sa_slices uses too) equal the
    host restatement (hkcsa/shard.py split_buckets) and the summed per-block counts at N = 2, 3, 8."""
    from hkcsa.shard import split_buckets
    text = oracle.synth_text(3 * (1 << 20) + 1, alpha, seed=nranks)
    devs = [hk.DeviceIndex.from_bytes(text, device=0) for _ in range(nranks)]
    assert devs[0].shard_scheme() == 1
    g = sum(d.shard_histogram(nranks, r) for r, d in enumerate(devs))
    assert int(g.sum()) == len(text)
    cum = np.concatenate(([0], np.cumsum(g, dtype=np.uint64)))
    host = np.array([cum[b] for b in split_buckets(g, nranks, aligned=True)], dtype=np.uint64)
    dev_below = sum(d.shard_counts(g, nranks, r) for r, d in enumerate(devs))
    assert np.array_equal(dev_below, host)
    for d in devs:
        d.close()
