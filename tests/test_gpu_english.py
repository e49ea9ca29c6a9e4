"""GPU parity on natural-language-like and protein-like text: the configs[2] shape and the proteins corpus
of the reference's dataset bench (tests/dataset_benchmark.py:13).

english.200MB (BASELINE.json configs[2]; the reference's corpora, tests/dataset_benchmark.py:10-16)
is absent offline, so utils.textgen.english_like stands in for its structure: Zipf words over a
skewed latin-1 alphabet, sentence punctuation, 25 % of the bytes verbatim copies of earlier passages
(50 - 5000 symbols) and a few 64 KiB - 1 MiB copies.  These texts tie far beyond any fixed key, so
they run the chunk refinement and the prefix-doubling fallback that iid text never reaches.

Checks (all bit-exact): the SA by the O(n) checker (a checked SA is build_suffix_array's output,
csa/suffix_array.py:131-134), the BWT against the oracle's gather (csa/bwt.py:3-13), every WT level
against the oracle's levelwise tree (csa/wavelet_tree.py:72-100), batched 20-symbol counts and a
locate sample against the oracle FM index (csa/enhanced_fm_index.py:15-32).
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def hk():
    import hkcsa
    if hkcsa.device_count() < 1:
        pytest.fail("no GPU visible: the HIP path is required (there is no CPU fallback)")
    return hkcsa


def _full_check(hk, text, npat, seed, flags=0, wt=True, fm=True):
    dev = hk.DeviceIndex.from_bytes(text, device=0, flags=flags)
    dev.build_all()
    info = dev.build_info()
    sa = dev.sa()
    assert oracle.check_sa(text, sa) == 0, info[:12]
    bwt = dev.bwt()
    assert np.array_equal(bwt, oracle.bwt(text, sa))
    if wt:
        want = oracle.wt_levels(bwt)
        assert dev.wt_levels() == len(want)
        for d in range(len(want)):
            assert np.array_equal(dev.wt_level_bits(d), want[d]), d
        del want
    if not fm:
        dev.close()
        return info
    rng = np.random.default_rng(seed)
    n = len(text)
    starts = rng.integers(0, n - 21, size=npat)
    pats = [text[s:s + 20].tobytes() for s in starts]
    pats += [text[s:s + 5].tobytes() + b"qzx" for s in starts[:200]]   # mostly absent
    fm = oracle.FM(text, sa)
    got = dev.count_ranges(pats)
    assert np.array_equal(got, fm.find_range(pats))
    assert (got[:npat, 0] >= 0).all()          # substrings (no '$' in the text body) occur
    few = pats[:300]
    offs, pos = dev.locate(few)
    assert [list(map(int, pos[offs[i]:offs[i + 1]])) for i in range(len(few))] == fm.find(few)
    dev.close()
    return info


def test_english_like_200MiB_full_build(hk):
    """configs[2] shape at its size: 200 MiB + '$', full build, all WT levels, 1M 20-symbol counts (the
    bench leg's batch size) and 300 locates against the oracle FM index."""
    from utils.textgen import english_like_text
    text = english_like_text(200 * (1 << 20) + 1, seed=3)
    info = _full_check(hk, text, 1_000_000, seed=31)
    assert info[2] >> 32 > 0, info[:12]         # the prefix-doubling fallback ran (long copies)


@pytest.mark.parametrize("seed,kw", [
    (5, dict(copy_frac=0.6, min_copy=200, max_copy=20000, long_copies=16)),
    (6, dict(copy_frac=0.05, long_copies=0)),
    (7, dict(copy_frac=0.4, min_copy=20, max_copy=400, long_copies=2, vocab=300)),
])
def test_english_like_24MiB_variants(hk, seed, kw):
    """Heavier and lighter repetition, a 300-word vocabulary: 24 MiB, full checks."""
    from utils.textgen import english_like_text
    text = english_like_text(24 * (1 << 20) + 1, seed=seed, **kw)
    _full_check(hk, text, 4000, seed=seed + 100)


def test_english_like_global_sort_flag(hk):
    """The same text through HKCSA_FLAG_GLOBAL_SORT (full-width LSD sort instead of bucket sorts)."""
    from utils.textgen import english_like_text
    text = english_like_text(6 * (1 << 20) + 1, seed=8)
    _full_check(hk, text, 2000, seed=108, flags=hk.index.FLAG_GLOBAL_SORT, wt=False)


def test_protein_like_1GiB_full_build(hk):
    """The proteins corpus shape (tests/dataset_benchmark.py:13) at 1 GiB: sigma = 25 + newline + '$' (not a
    power of two, so the stable onesweep pair instead of the cursor passes), skewed letter frequencies,
    35 % family members (copies with 8 % substitutions) and 5 % exact duplicates.  SA by the O(n) checker,
    BWT by the oracle's gather, every WT level, 100k 20-symbol counts and 300 locates against the oracle."""
    from utils.textgen import protein_like_text
    text = protein_like_text((1 << 30) + 1, seed=4)
    _full_check(hk, text, 100_000, seed=41)


def test_protein_like_24MiB_wt(hk):
    """The same generator at 24 MiB with every WT level checked."""
    from utils.textgen import protein_like_text
    text = protein_like_text(24 * (1 << 20) + 1, seed=9, family_frac=0.6, mut_rate=0.02)
    _full_check(hk, text, 4000, seed=91)


@pytest.mark.parametrize("kind,flag", [("english", "FLAG_NO_LINKS"), ("protein", "FLAG_LINKS"),
                                       ("periodic", "FLAG_LINKS"), ("repeats", "FLAG_LINKS")])
def test_doubling_links_both_ways(hk, kind, flag):
    """Doubling links (a group that maps whole onto one tied group leaves the list; hk_seground.hpp) forced on
    or off against the default rule (on when a third of the suffixes reach prefix doubling): the English-like
    text without them, protein-like, periodic and planted-repeat texts with them.  Full checks."""
    from utils.textgen import english_like_text, protein_like_text
    rng = np.random.default_rng(77)
    if kind == "english":
        text = english_like_text(12 * (1 << 20) + 1, seed=12)
    elif kind == "protein":
        text = protein_like_text(16 * (1 << 20) + 1, seed=13, family_frac=0.6, mut_rate=0.02)
    elif kind == "periodic":
        unit = rng.integers(97, 101, size=37, dtype=np.uint8)
        body = np.tile(unit, (3 << 20) // 37 + 1)[: 3 << 20]
        body[1 << 20] = 120                                  # one break in the period
        text = np.concatenate([body, np.frombuffer(b"$", np.uint8)])
    else:
        body = rng.integers(65, 69, size=4 << 20, dtype=np.uint8)
        for _ in range(40):                                  # planted copies of 10K - 200K symbols
            ln = int(rng.integers(10_000, 200_000))
            src, dst = (int(x) for x in rng.integers(0, len(body) - ln, size=2))
            body[dst:dst + ln] = body[src:src + ln].copy()
        text = np.concatenate([body, np.frombuffer(b"$", np.uint8)])
    _full_check(hk, text, 3000, seed=171, flags=getattr(hk.index, flag), wt=False)
