import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "high-order-entropy-compressed-suffix-array_amd")
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path through the C-ABI)")


# GPU modules run in this order: the BASELINE config tests first (configs[0], then configs[1]/[3]/1 GiB,
# then configs[4]), the multi-process gloo tests last, so a `-x` stop in a fragile multi-process test
# cannot leave the config rows unreached.  Modules not listed keep their place between the two groups.
_FIRST = ["test_gpu_configs", "test_gpu_parity", "test_gpu_scale", "test_gpu_english", "test_gpu_dropin"]
_LAST = ["test_gpu_dist"]


def pytest_collection_modifyitems(session, config, items):
    def key(item):
        mod = item.module.__name__.rsplit(".", 1)[-1] if item.module else ""
        if mod in _FIRST:
            return _FIRST.index(mod)
        if mod in _LAST:
            return len(_FIRST) + 1 + _LAST.index(mod)
        return len(_FIRST)
    items.sort(key=key)      # stable: the order inside a module is kept


@pytest.fixture(scope="session")
def kat():
    with open(os.path.join(GOLDEN, "kat.json")) as f:
        return json.load(f)


class Cases:
    def __init__(self, path):
        self.z = np.load(path, allow_pickle=False)
        self.names = [str(x) for x in self.z["cases"]]

    def get(self, name):
        pre = name + "/"
        return {k[len(pre):]: self.z[k] for k in self.z.files if k.startswith(pre)}


@pytest.fixture(scope="session")
def random_cases():
    return Cases(os.path.join(GOLDEN, "random_cases.npz"))


@pytest.fixture(scope="session")
def large_cases():
    return Cases(os.path.join(GOLDEN, "large_cases.npz"))


def patterns_of(case, prefix="pat"):
    d, o = case[f"{prefix}_data"], case[f"{prefix}_offs"]
    return [d[o[i]:o[i + 1]].tobytes() for i in range(len(o) - 1)]


def locs_of(case):
    d, o = case["loc_data"], case["loc_offs"]
    return [[int(x) for x in d[o[i]:o[i + 1]]] for i in range(len(o) - 1)]


def wt_golden_levels(case):
    L = int(case["wt_levels"][0]) if "wt_levels" in case else 0
    out = []
    for lv in range(L):
        nb = int(case[f"wt{lv}_nbits"][0])
        bits = np.unpackbits(case[f"wt{lv}_bits"])[:nb]
        ng = int(case[f"wt{lv}_ngolomb"][0])
        gol = np.unpackbits(case[f"wt{lv}_golomb"])[:ng]
        out.append({"bits": bits, "golomb": gol, "left": case[f"wt{lv}_left"].tobytes(),
                    "right": case[f"wt{lv}_right"].tobytes(), "next": case[f"wt{lv}_next"].tobytes()})
    return out
