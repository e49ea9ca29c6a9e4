#!/usr/bin/env python3
"""Headline benchmark: SA build MB/s + batched locate() patterns/s (BASELINE.json).

N = 1 (default): configs[1]'s pipeline on the metric's 1 GiB sigma=4 text — one "step" is the
  SA + BWT build of T' = 2^30 iid ACGT symbols + '$' (text resident in HBM before timing): keyed
  suffix keys, bucket histogram, two LSD radix passes over the bucket bits (the first builds the
  keys from the text), LDS bucket sorts that write SA and BWT, refinement of the tied suffixes.
  After the timed steps the wavelet tree is built and 1M random 16-symbol substrings are located in
  batches (count + SA gather), reported as locate_patterns_per_s.
N > 1 (torchrun, one process per GPU): the sharded construction (hkcsa_build_sa_sharded: RCCL
  all-reduce of the partition histogram and of the slice counts, independent slice sorts, RCCL
  all-gather of the slice bounds) of an N GiB text, i.e. weak scaling at 1 GiB of suffixes per GPU;
  value = all ranks' text MB / max-over-ranks time.

The JSON line also carries:
  roofline      — the dominant kernel of the timed steps (largest summed time among the bucket
                  sort and the two radix passes) timed with HIP events on the library's stream:
                  achieved = its algorithmic bytes per launch / mean launch time, peak = 8000 GB/s
                  (MI355X HBM3E), traffic = PMC-measured HBM bytes per launch (profiles/
                  pmc_kernels.json); the other two kernels under roofline["others"].
  cpu_baseline  — the pure-Python restatement of the reference (oracle/ref_port.py:
                  naive suffix sort, dense occ, dict backward search), one core, on a
                  bounded sample (rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "high-order-entropy-compressed-suffix-array_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

from hkcsa import DeviceIndex, comm_unique_id  # noqa: E402

METRIC = "SA build MB/s + batched locate() patterns/s, 1 GiB text, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
DNA = b"ACGT"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(sample_n: int, npat: int, seed: int = 3) -> dict:
    """Reference algorithm restated in pure Python, timed on this host (1 core)."""
    from oracle import ref_port
    rng = np.random.default_rng(seed)
    text = np.frombuffer(DNA, np.uint8)[rng.integers(0, 4, size=sample_n)].tobytes().decode("latin-1")
    times = []
    idx = None
    for _ in range(3):
        gc.collect()
        t0 = time.perf_counter()
        idx = ref_port.FMIndexPort(text)
        times.append(time.perf_counter() - t0)
    t_build = float(np.median(times))
    tp = idx.text
    starts = rng.integers(0, len(tp) - 16, size=npat)
    pats = [tp[s:s + 16] for s in starts]
    gc.collect()
    t0 = time.perf_counter()
    for p in pats:
        idx.find(p)
    t_q = time.perf_counter() - t0
    return {
        "value": round(len(tp) / 2**20 / t_build, 6),
        "unit": "MB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"EnhancedFMIndex restatement (naive SA + BWT + dense occ + C) on {len(tp)} iid ACGT "
                  f"symbols, median of 3; find() of {npat} 16-symbol substrings",
        "build_s": round(t_build, 4),
        "locate_patterns_per_s": round(npat / t_q, 1),
        "host_cpus": os.cpu_count(),
    }


# kernels whose roofline bench.py reports: the dominant one (largest summed time) as `roofline`,
# the others under roofline["others"]
ROOF_KERNELS = ("sa_bucket_sort", "radix_onesweep_text", "radix_onesweep")


def pmc_traffic_gb(name: str) -> float | None:
    """HBM GB per launch of timer `name`'s kernel, measured with rocprofv3 PMC counters on this config
    (tools/gpu_pmc.sh + tools/pmc_summary.py -> profiles/pmc_kernels.json; FETCH_SIZE x2 gfx950 correction)."""
    p = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    try:
        with open(p) as f:
            return float(json.load(f)[name]["traffic_gb_per_launch"])
    except Exception:
        return None


def kernel_roofline(dev: DeviceIndex, name: str) -> dict | None:
    launches, ms, alg_bytes = dev.kernel_stats(name)
    if not launches:
        return None
    per_launch_bytes = alg_bytes / launches
    avg_s = ms / launches / 1e3
    achieved = per_launch_bytes / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic_gb(name), "kernel": name,
            "launches": launches, "avg_launch_ms": round(ms / launches, 4), "total_ms": round(ms, 3),
            "alg_bytes_per_launch": per_launch_bytes}


def roofline(dev: DeviceIndex, traffic_gb: float | None) -> dict:
    rows = [r for r in (kernel_roofline(dev, k) for k in ROOF_KERNELS) if r]
    if not rows:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None}
    dom = max(rows, key=lambda r: r["total_ms"])
    if traffic_gb is not None:
        dom["traffic"] = traffic_gb
    dom["others"] = [{k: r[k] for k in ("kernel", "achieved", "frac", "traffic", "avg_launch_ms")}
                     for r in rows if r is not dom]
    return dom


def stage_breakdown(dev: DeviceIndex, names) -> dict:
    out = {}
    for nm in names:
        l, ms, b = dev.kernel_stats(nm)
        if l:
            out[nm] = {"launches": l, "ms": round(ms, 3)}
    return out


def run_single(args) -> dict:
    n = args.text_bytes + 1
    dev = DeviceIndex.synthetic(n, DNA, seed=args.seed, device=0, flags=4 if args.global_sort else 0)
    log(f"[bench] text n={n} resident on device")
    for _ in range(args.warmup):
        dev.build_sa()
        dev.build_bwt()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    try:
        import torch
        torch.cuda.synchronize()
    except Exception:
        pass
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dev.build_sa()
        dev.build_bwt()
    dev.synchronize()
    t1 = time.perf_counter()
    dev.timing(False)
    wall = t1 - t0
    value = args.steps * n / 2**20 / wall
    info = dev.build_info()
    roof = roofline(dev, args.traffic_gb)
    stages = stage_breakdown(dev, ["sa_bucket_hist", "sa_digit_hist", "sa_bin_starts", "sa_bucket_sort",
                                   "sa_big_gather", "radix_onesweep_text",
                                   "radix_table_text", "radix_tile_hist",
                                   "radix_hist", "radix_onesweep", "radix_onesweep_small", "sa_pack_keys",
                                   "sa_refine_stats", "sa_refine_apply", "sa_refine_keys", "sa_isa_scatter",
                                   "sa_group_stats", "sa_group_apply", "sa_pair_keys", "bwt_gather", "byte_hist"])
    log(f"[bench] SA+BWT {wall / args.steps * 1e3:.2f} ms/step -> {value:.1f} MB/s; info={info[:8]}")

    # full build (adds the wavelet tree) and batched locate
    t0 = time.perf_counter()
    dev.build_wt()
    dev.synchronize()
    t_wt = time.perf_counter() - t0
    loc = None
    if args.patterns > 0:
        rng = np.random.default_rng(args.seed + 1)
        starts = np.sort(rng.integers(0, n - 1 - args.plen, size=args.patterns)).astype(np.uint64)
        lo, hi = int(starts[0]), int(starts[-1]) + args.plen
        txt = dev.text(lo, hi)
        idx = (starts - lo)[:, None] + np.arange(args.plen, dtype=np.uint64)[None, :]
        data = txt[idx].reshape(-1)
        rng.shuffle(data.reshape(-1, args.plen))
        offs = np.arange(args.patterns + 1, dtype=np.uint64) * args.plen
        q = dev.queries(data=data, offs=offs)
        q.locate()
        dev.synchronize()
        t0 = time.perf_counter()
        reps = args.query_reps
        total = 0
        for _ in range(reps):
            total = q.locate()
        dev.synchronize()
        t_loc = (time.perf_counter() - t0) / reps
        t0 = time.perf_counter()
        for _ in range(reps):
            q.count()
        dev.synchronize()
        t_cnt = (time.perf_counter() - t0) / reps
        loc = {"patterns": args.patterns, "plen": args.plen, "occurrences": int(total),
               "locate_patterns_per_s": round(args.patterns / t_loc, 1),
               "count_patterns_per_s": round(args.patterns / t_cnt, 1)}
        q.close()
    res = {
        "metric": METRIC,
        "value": round(value, 2),
        "unit": "MB/s",
        "n_gpus": 1,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(wall / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": "1 GiB synthetic sigma=4 text: SA + BWT by the HIP bucket build (LSD "
                               "radix passes over the bucket bits, LDS bucket sorts writing SA and BWT, "
                               "tie refinement; configs[1] pipeline at the metric's 1 GiB), then WT + "
                               f"1M batched {args.plen}-symbol locate()",
                   "text_symbols": n, "sigma": 4, "positions": "u32"},
        "roofline": roof,
        "locate_patterns_per_s": loc["locate_patterns_per_s"] if loc else None,
        "full_build_MBps": round(n / 2**20 / (wall / args.steps + t_wt), 2),
        "detail": {"wt_build_ms": round(t_wt * 1e3, 2), "locate": loc, "stages_ms_total": stages,
                   "build_info": info[:16]},
    }
    dev.close()
    return res


def run_sharded(args, rank: int, world: int, local_rank: int) -> dict | None:
    import torch
    import torch.distributed as dist
    torch.cuda.set_device(local_rank)
    per = args.text_bytes
    n = per * world + 1
    dev = DeviceIndex.synthetic(n, DNA, seed=args.seed, device=local_rank, flags=1 if args.pos64 else 0)
    uid = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    uid = uid[0]
    for _ in range(args.warmup):
        dev.build_sa_sharded(uid, world, rank)
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        dev.build_sa_sharded(uid, world, rank)
    dev.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    dev.timing(False)
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    wall = float(el.item())
    lo, hi = dev.shard_range()
    roof = roofline(dev, args.traffic_gb)
    # the PMC summaries in profiles/ are of the single-GPU launches: not this slice's kernels
    if args.traffic_gb is None:
        roof["traffic"] = None
        for o in roof.get("others", []):
            o["traffic"] = None
    stages = stage_breakdown(dev, ["shard_hist", "shard_below", "shard_select_count", "shard_pack_select",
                                   "rccl_allreduce_hist", "rccl_allreduce_counts", "rccl_allgather_bounds",
                                   "sa_bin_starts", "sa_bucket_sort", "radix_hist", "radix_onesweep",
                                   "radix_onesweep_small", "shard_split_join", "sa_refine_stats",
                                   "sa_refine_apply", "sa_refine_keys"])
    res = None
    if rank == 0:
        value = args.steps * n / 2**20 / wall
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{world} GiB synthetic sigma=4 text sharded over {world} GPUs: partition "
                                   "histogram + slice counts by RCCL all-reduce, per-rank slice selection, LSD "
                                   "passes over the slice's bucket bits, LDS bucket sorts, tie refinement, RCCL "
                                   "all-gather of the slice bounds", "text_symbols": n, "sigma": 4,
                       "parallelism": f"sa-slices x{world}",
                       "positions": "u64" if (n >= 2**32 - 1 or args.pos64) else "u32"},
            "roofline": roof,
            "locate_patterns_per_s": None,
            "detail": {"rank0_slice": [lo, hi], "stages_ms_total": stages, "build_info": dev.build_info()[:16]},
        }
    dev.close()
    return res


def _stdout_for_result():
    """Route fd 1 to stderr for the run (RCCL / gloo print banners on stdout) and return a
    stream on the original stdout, so the result stays the only line there."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def main():
    result_out = _stdout_for_result()
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--text-bytes", type=int, default=1 << 30, help="text symbols per GPU (before '$')")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--patterns", type=int, default=1_000_000)
    ap.add_argument("--plen", type=int, default=16)
    ap.add_argument("--query-reps", type=int, default=5)
    ap.add_argument("--cpu-sample", type=int, default=1 << 17)
    ap.add_argument("--cpu-patterns", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--sharded", action="store_true", help="use the sharded (multi-GPU) build even at N=1")
    ap.add_argument("--pos64", action="store_true", help="sharded build with 64-bit positions at any n")
    ap.add_argument("--global-sort", action="store_true",
                    help="single-GPU build by full-width LSD sort of the keys (no LDS bucket sorts)")
    ap.add_argument("--traffic-gb", type=float, default=None,
                    help="PMC-measured HBM GB per launch of the dominant kernel; default: profiles/pmc_kernels.json")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or args.gpus > 1 or args.sharded:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(backend="gloo")
        world = dist.get_world_size()
        rank = dist.get_rank()
        res = run_sharded(args, rank, world, local_rank)
        dist.barrier()
        dist.destroy_process_group()
    else:
        res = run_single(args)
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_patterns)
    if res is not None:
        if "cpu_baseline" not in res:
            res["cpu_baseline"] = None
        print(json.dumps(res), file=result_out, flush=True)


if __name__ == "__main__":
    main()
