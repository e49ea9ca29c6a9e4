"""BASELINE.json configs[0] exactly as it is quoted: a 1 MiB iid DNA text (sigma = 4) through the
drop-in `csa.CSA` / `CompressedSuffixArray(text, epsilon=0.5)` surface (tests/benchmark.py:25-52,
the class the reference's harness expects), SA + BWT + WT built, then 1,000 seeded 16-symbol
`locate()` calls, each one a separate call as the reference's harness makes them
(tests/benchmark.py:39-52), checked against the oracle FM index (csa/enhanced_fm_index.py:15-32).

This module sorts first in the GPU suite (conftest.pytest_collection_modifyitems), so a `-x` stop
later in the multi-process tests cannot hide it.
"""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

N0 = 1 << 20


def _dna_text(n, seed):
    rng = np.random.default_rng(seed)
    return np.frombuffer(b"ACGT", np.uint8)[rng.integers(0, 4, size=n)]


@pytest.mark.parametrize("epsilon,compact", [(0.5, True), (0.5, False)])
def test_config0_csa_1MiB_dna_1k_locate(epsilon, compact):
    from csa import CompressedSuffixArray
    from utils.patterns import sample_substrings
    t = _dna_text(N0, seed=0)
    text = t.tobytes().decode("latin-1")
    csa = CompressedSuffixArray(text, epsilon=epsilon, compact=compact)
    tp = np.concatenate([t, np.frombuffer(b"$", np.uint8)])
    fm = oracle.FM(tp)
    assert oracle.check_sa(tp, fm.sa) == 0
    # whole-structure parity: SA, BWT (SA order) and C
    assert np.array_equal(np.asarray(csa.fm_index.device_index.sa(), np.uint64), fm.sa)
    assert np.array_equal(csa.fm_index.device_index.bwt(), fm.bwt)
    data, offs = sample_substrings(t, 1000, 16, seed=1)
    pats = [data[offs[i]:offs[i + 1]].tobytes() for i in range(1000)]
    want = fm.find(pats)
    for p, w in zip(pats, want):
        assert csa.locate(p.decode("latin-1")) == w
    assert sum(len(w) for w in want) >= 1000       # every sampled pattern occurs
    # count() agrees with the same backward search
    lr = fm.find_range(pats[:100])
    for p, (l, r) in zip(pats[:100], lr):
        assert csa.count(p.decode("latin-1")) == (0 if l < 0 else int(r - l + 1))
