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
