"""Kernel gaps of the last build step: a rocprofv3 kernel trace (CSV) of `bench.py --steps 2 --warmup 1`
(SA build only), printed in dispatch order with each kernel's duration and the idle gap before it (us),
over one whole build step (between the last two byte-histogram dispatches); --csv OUT also writes the rows."""
import csv
import sys

src = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/gap/run_kernel_trace.csv"
out = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
               for r in csv.DictReader(open(src))), key=lambda r: r[1])
starts = [i for i, r in enumerate(rows) if "k_byte_hist" in r[0]]
# one whole build step: from the second-to-last byte histogram to the last (the last step is followed by
# the WT build and queries); a single step: from its histogram to the end
i0, i1 = (starts[-2], starts[-1]) if len(starts) >= 2 else ((starts[-1] if starts else 0), len(rows))
prev = None
tot_gap = 0.0
lines = []
for name, st, en in rows[i0:i1]:
    gap = (st - prev) / 1000 if prev is not None else 0.0
    gap = max(gap, 0.0)   # (overlapping dispatches on the auxiliary stream)
    tot_gap += gap
    short = name.replace("hk::(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
    lines.append(((st - rows[i0][1]) / 1000, (en - rows[i0][1]) / 1000, gap, short))
    print(f"{gap:9.1f} {((en - st) / 1000):9.1f}  {short}")
    prev = en if prev is None else max(prev, en)
span = (max(r[2] for r in rows[i0:i1]) - rows[i0][1]) / 1000
print("total gap us", round(tot_gap, 1), "span us", round(span, 1))
if out:
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["start_us", "end_us", "gap_before_us", "kernel"])
        for r in lines:
            w.writerow([round(r[0], 1), round(r[1], 1), round(r[2], 1), r[3]])
        w.writerow(["total_gap_us", round(tot_gap, 1), "span_us", round(span, 1)])
