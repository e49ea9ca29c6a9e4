"""Diagnostic: the per-rank work of an N-GPU sharded build, emulated on one GPU.

The global key histogram of the whole text equals the sum of the ranks' histograms, so one
device can play rank r of N with the two-phase API (hkcsa_shard_histogram over all of T',
then hkcsa_shard_build(global, N, r)).  Prints one JSON line per emulated rank with the
slice size, wall time and the per-kernel breakdown (HIP events).

  python tools/shard_emulate.py --per-rank 1073741824 --nranks 8 --ranks 0 7
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                "high-order-entropy-compressed-suffix-array_amd"))
from hkcsa import DeviceIndex  # noqa: E402

STAGES = ["shard_hist", "shard_slice_hist", "shard_slice_part", "shard_select_count", "shard_pack_select",
          "sa_bucket_hist", "radix_part_keys", "radix_part",
          "sa_bin_starts", "sa_bucket_sort", "radix_hist",
          "radix_onesweep", "radix_onesweep_small", "shard_split_join", "sa_refine_stats", "sa_refine_apply",
          "sa_refine_keys"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--per-rank", type=int, default=1 << 30)
    ap.add_argument("--nranks", type=int, default=8)
    ap.add_argument("--ranks", type=int, nargs="*", default=[0])
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--pos64", action="store_true")
    args = ap.parse_args()
    N = args.nranks
    n = args.per_rank * N + 1
    dev = DeviceIndex.synthetic(n, b"ACGT", seed=2, device=0, flags=1 if args.pos64 else 0)
    g = dev.shard_histogram(1, 0)
    below = sum(dev.shard_counts(g, N, r) for r in range(N))   # every rank's block, summed
    for r in args.ranks:
        dev.shard_build(g, below, N, r)  # warm-up (workspace growth)
        dev.synchronize()
        dev.timing_reset()
        dev.timing(True)
        t0 = time.perf_counter()
        for _ in range(args.reps):
            dev.shard_build(g, below, N, r)
        dev.synchronize()
        wall = (time.perf_counter() - t0) / args.reps
        dev.timing(False)
        stages = {}
        for s in STAGES:
            l, ms, b = dev.kernel_stats(s)
            if l:
                stages[s] = {"launches_per_build": l // args.reps, "ms_per_build": round(ms / args.reps, 3)}
        lo, hi = dev.shard_range()
        print(json.dumps({"n": n, "nranks": N, "rank": r, "slice": [lo, hi], "build_ms": round(wall * 1e3, 2),
                          "info": dev.build_info()[:8], "stages": stages}), flush=True)
    dev.close()


if __name__ == "__main__":
    main()
