"""The C-ABI library loads and exports every symbol include/hkcsa.h declares (no GPU needed)."""
import os
import re

import hkcsa
from hkcsa import _native

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "hkcsa.h")


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hkcsa_[A-Za-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = header_functions()
    assert "hkcsa_build_sa" in names and "hkcsa_locate_batch" in names
    assert len(names) >= 40


def test_library_exports_every_declared_symbol():
    lib = hkcsa.load()
    missing = [n for n in header_functions() if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_table_matches_header():
    assert sorted(_native.EXPORTED) == header_functions()


def test_abi_version_and_errors_without_device():
    lib = hkcsa.load()
    assert lib.hkcsa_abi_version() == 1
    # argument validation happens before any device work
    rc = lib.hkcsa_create(None, 0, None, None)
    assert rc == -1
    assert b"null" in lib.hkcsa_last_error()


def test_library_is_gfx950():
    so = hkcsa.LIB_PATH
    data = open(so, "rb").read()
    assert b"gfx950" in data


def test_flag_constants_match_header():
    """hkcsa.index.FLAG_* and _native.E_RANGE mirror the header's #defines."""
    from hkcsa import index
    src = open(HEADER).read()
    flags = {m.group(1): int(m.group(2)) for m in re.finditer(r"#define HKCSA_FLAG_([A-Z0-9_]+) (\d+)u", src)}
    assert {"POS64", "GLOBAL_SORT", "MUL_BINS", "MAX_BUCKETS", "SLICES"} <= set(flags)
    for name, v in flags.items():
        if hasattr(index, "FLAG_" + name):
            assert getattr(index, "FLAG_" + name) == v, name
    assert int(re.search(r"#define HKCSA_E_RANGE \((-\d+)\)", src).group(1)) == _native.E_RANGE


def test_slice_bounds_planner_refuses_oversized_slice():
    """hkcsa_slice_bounds (host only, no device): the slice bounds hkcsa_build_sa's slice build takes from
    an exact coarse histogram equal hkcsa/shard.py's restatement of the splitter rule; a histogram with one
    dominant coarse bucket of >= 2^32 - 1 suffixes (a long run in a text of n > 2^32) is refused with
    HKCSA_E_TOOBIG instead of wrapping the 32-bit slots inside a slice."""
    import ctypes as C

    import numpy as np

    from hkcsa import shard
    from hkcsa.index import _ptr
    lib = hkcsa.load()
    nb = 65536
    rng = np.random.default_rng(3)
    for k in (1, 2, 3, 4, 8):
        h = rng.integers(0, 70000, size=nb).astype(np.uint64)
        below = np.zeros(k + 1, dtype=np.uint64)
        assert lib.hkcsa_slice_bounds(_ptr(h), nb, k, _ptr(below)) == 0
        B = shard.split_buckets(h, k, aligned=True)
        cum = np.concatenate(([0], np.cumsum(h)))
        assert [int(cum[b]) for b in B] == [int(x) for x in below], k
    # 4 GiB + 1 text whose run of one symbol fills one coarse bucket with 2^32 - 1 suffixes
    h = np.zeros(nb, dtype=np.uint64)
    h[0] = (1 << 32) - 1
    h[1:3] = 1
    below = np.zeros(5, dtype=np.uint64)
    assert lib.hkcsa_slice_bounds(_ptr(h), nb, 4, _ptr(below)) == -6
    assert b"2^32" in lib.hkcsa_last_error()
    h[0] = (1 << 32) - 2                     # one fewer: a single slice of 2^32 - 2 is still addressable
    assert lib.hkcsa_slice_bounds(_ptr(h), nb, 4, _ptr(below)) == 0
    assert int(below[1]) == (1 << 32) - 2
    assert lib.hkcsa_slice_bounds(None, nb, 4, _ptr(below)) == -1
    assert lib.hkcsa_slice_bounds(_ptr(h), nb, 0, _ptr(below)) == -1
    del C
