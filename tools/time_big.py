"""Times each step of the 1 GiB parity check (tests/test_gpu_parity.py::test_full_size_bench_1GiB_sigma4)
with a line per step, so a slow oracle step shows up (diagnostic)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "high-order-entropy-compressed-suffix-array_amd"))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

import hkcsa  # noqa: E402
from oracle import oracle  # noqa: E402

T0 = time.time()


def step(msg):
    print(f"{time.time() - T0:8.2f}s {msg}", flush=True)


n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 30) + 1
step("start")
dev = hkcsa.DeviceIndex.synthetic(n, b"ACGT", seed=2)
dev.build_sa()
dev.build_bwt()
dev.synchronize()
step("gpu build")
sa = dev.sa()
step("dev.sa()")
text = oracle.synth_text(n, b"ACGT", seed=2)
step("oracle.synth_text")
r = oracle.check_sa(text, sa)
step(f"check_sa -> {r}")
bwt = oracle.bwt(text, sa)
step("oracle.bwt")
ok = np.array_equal(dev.bwt(), bwt)
step(f"bwt equal {ok}")
dev.build_wt()
step("build_wt")
fm = oracle.FM(text, sa)
step("oracle.FM")
rng = np.random.default_rng(5)
pats = [text[s:s + 16].tobytes() for s in rng.integers(0, n - 16, size=2000)]
a = dev.count_ranges(pats)
step("dev.count_ranges")
b = fm.find_range(pats)
step(f"fm.find_range equal {np.array_equal(a, b)}")
