"""Kernel gaps of one bench step: rocprofv3 kernel trace of `bench.py --steps 2 --warmup 1` (SA build
only), printed in dispatch order with each kernel's duration and the idle gap before it (us)."""
import os
import sqlite3
import sys

db = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gap/run_results.db"
c = sqlite3.connect(db)
rows = c.execute("select name, start, end from kernels order by start").fetchall()
# the last step: from the last byte-histogram dispatch on
starts = [i for i, r in enumerate(rows) if "k_byte_hist" in r[0]]
i0 = starts[-1] if starts else 0
prev = None
tot_gap = 0.0
for name, st, en in rows[i0:]:
    gap = (st - prev) / 1000 if prev is not None else 0.0
    tot_gap += gap
    short = name.replace("hk::(anonymous namespace)::", "").split("(")[0][:70]
    print(f"{gap:9.1f} {((en - st) / 1000):9.1f}  {short}")
    prev = en
print("total gap us", round(tot_gap, 1), "span us", round((rows[-1][2] - rows[i0][1]) / 1000, 1))
