"""GPU parity of the single-GPU bucket build (hk_bucket.hip) and of the global-sort path
(HKCSA_FLAG_GLOBAL_SORT): the keyed suffix keys (no end-of-text code, a unique terminal left out
of the radix), the short-suffix boundary keys, LDS bucket sorts (narrow and wide local keys), big
buckets on the global path, and the tie list feeding refinement / prefix doubling.
SA bit-exact against the oracle (naive sort up to 1 MiB, the O(n) checker above), BWT and C
recomputed by the oracle from the checked SA."""
import numpy as np
import pytest

from oracle import oracle

pytestmark = pytest.mark.gpu

GLOBAL_SORT = 4
MAX_BUCKETS = 16   # 2^17 buckets at any n: the 1 GiB pipeline (half items, packed records)


@pytest.fixture(scope="module")
def hk():
    import hkcsa
    if hkcsa.device_count() < 1:
        pytest.fail("no GPU visible: the HIP path is required (there is no CPU fallback)")
    return hkcsa


def _rand(n, alphabet, seed, p=None):
    rng = np.random.default_rng(seed)
    a = np.frombuffer(alphabet, dtype=np.uint8)
    return a[rng.choice(len(a), size=n, p=p)]


def _cases():
    rng = np.random.default_rng(5)
    yield "dna_4M", oracle.synth_text((1 << 22) + 1, b"ACGT", seed=21)
    yield "dna_20K", oracle.synth_text(20001, b"ACGT", seed=22)           # two buckets
    yield "dna_18K", oracle.synth_text(18000, b"ACGT", seed=23)           # one LDS sort, no passes
    # a long run inside random DNA: one bucket far above the LDS capacity (the big-bucket path)
    t = _rand(1 << 21, b"ACGT", 24)
    t[700000:1000000] = ord("A")
    yield "dna_run_2M", np.concatenate([t, [ord("$")]]).astype(np.uint8)
    # terminal above every symbol, in the middle, and not unique
    yield "term_top", np.concatenate([_rand(300000, b"abc", 25), [ord("~")]]).astype(np.uint8)
    yield "term_mid", np.concatenate([_rand(300000, b"az", 26), [ord("m")]]).astype(np.uint8)
    yield "term_mid4", np.concatenate([_rand(300000, b"acgt", 35), [ord("m")]]).astype(np.uint8)
    yield "term_repeated", np.concatenate([_rand(300000, b"$AC", 27), [ord("$")]]).astype(np.uint8)
    yield "term_lowest_byte", np.concatenate([_rand(100000, b"\x01\x02\x03", 28), [0]]).astype(np.uint8)
    # skewed binary: wide local keys and big buckets (most suffixes start with a's)
    yield "skewed_binary_4M", np.concatenate([_rand(1 << 22, b"ab", 29, p=[0.9, 0.1]),
                                              [ord("$")]]).astype(np.uint8)
    # keyed radix 2^3 and 2^5 (codes do not tile a 32-bit word) and 2^4
    yield "radix8_1M", oracle.synth_text((1 << 20) + 1, b"ACDEFGHI", seed=32)
    yield "radix16_1M", oracle.synth_text((1 << 20) + 1, b"ABCDEFGHIJKLMNOP", seed=33)
    yield "radix32_1M", oracle.synth_text((1 << 20) + 1, bytes(range(0x41, 0x61)), seed=34)
    yield "bytes_2M", oracle.synth_text((1 << 21) + 1, bytes(range(256)), seed=30)
    yield "printable_3M", oracle.synth_text(3 * (1 << 20) + 1, bytes(range(0x20, 0x7F)), seed=31)
    base = rng.integers(0, 4, size=3000).astype(np.uint8) + ord("A")
    yield "repeats_600K", np.concatenate([np.tile(base, 200), [ord("$")]]).astype(np.uint8)
    yield "short_2", np.frombuffer(b"a$", dtype=np.uint8)
    yield "short_3", np.frombuffer(b"ba$", dtype=np.uint8)
    yield "all_same_70", np.frombuffer(b"q" * 70, dtype=np.uint8)


@pytest.mark.parametrize("flags", [0, GLOBAL_SORT, MAX_BUCKETS])
@pytest.mark.parametrize("name,text", list(_cases()))
def test_bucket_build_vs_oracle(hk, name, text, flags):
    dev = hk.DeviceIndex.from_bytes(text.tobytes(), device=0, flags=flags)
    dev.build_sa()
    dev.build_bwt()
    sa = dev.sa()
    assert oracle.check_sa(text, sa) == 0, name
    if len(text) <= (1 << 20) + 1 and not name.startswith(("repeats", "all_same")):
        assert np.array_equal(sa, oracle.suffix_array(text)), name
    assert np.array_equal(dev.bwt(), oracle.bwt(text, sa)), name
    info = dev.build_info()
    if flags == 0 and name in ("dna_4M", "bytes_2M", "printable_3M"):
        assert info[7] == 0 and info[4] > 0 and info[5] == 0, (name, info[:8])
    if flags == 0 and name == "dna_run_2M":
        assert info[7] == 0 and info[5] >= 1, (name, info[:8])
    if flags == MAX_BUCKETS and name in ("dna_4M", "dna_run_2M", "term_mid4", "radix16_1M"):
        # packed records (bit 1) with the prev field re-coded without the terminal ('$' lowest in
        # dna_*, 'm' inside the alphabet in term_mid4)
        assert info[7] & 2, (name, info[:8])
    dev.close()


def test_bucket_build_rebuild_identical(hk):
    text = oracle.synth_text((1 << 21) + 1, b"ACGT", seed=40)
    dev = hk.DeviceIndex.from_bytes(text.tobytes(), device=0)
    dev.build_sa()
    a = dev.sa().copy()
    dev.build_sa()
    assert np.array_equal(a, dev.sa())
    dev.close()
