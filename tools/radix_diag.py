"""Diagnostic: per-pass time of onesweep variants at n keys (prints one JSON line)."""
import ctypes as C, json, sys, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "high-order-entropy-compressed-suffix-array_amd"))
import numpy as np
from hkcsa import _native as N
lib = N.load()
n = int(sys.argv[1]) if len(sys.argv) > 1 else (1 << 30)
out = np.zeros(8)
N.check(lib.hkcsa_debug_radix_bench(n, 5, out.ctypes.data_as(C.c_void_p), 8))
names = ["512x16_w16", "512x16_nolookback", "1024x16_w4", "1024x12_w4", "512x16_w4", "1024x16_nolookback", "copy", "err"]
gb = n * 24 / 1e9
print(json.dumps({k: (round(v, 4) if k != "err" else v) for k, v in zip(names, out)}))
print(json.dumps({k + "_GBps": round(gb / (v / 1e3), 1) for k, v in zip(names[:7], out[:7])}))
