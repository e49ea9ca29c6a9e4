#!/usr/bin/env python3
"""Headline benchmark: SA build MB/s + batched locate() patterns/s (BASELINE.json).

N = 1 (default): configs[1]'s pipeline on the metric's 1 GiB sigma=4 text — one "step" is the
  SA + BWT build of T' = 2^30 iid ACGT symbols + '$' (text resident in HBM before timing): byte
  histogram / C array, keyed suffix keys, two LSD radix passes over the bucket bits (the first builds
  the keys from the text), LDS bucket sorts that write SA and BWT, refinement of the tied suffixes.
  After the timed steps the wavelet tree is built (warm, timed over repeats) and 1M random 16-symbol
  substrings are located in batches (count + SA gather), reported as locate_patterns_per_s.
  Extra legs under detail (skip with --no-legs):
    sigma256          configs[3]: 1 GiB iid bytes (sigma=256): SA + BWT steps, 8-level WT, roofline of
                      the radix passes and WT kernels;
    printable_200MiB  a clearly labelled stand-in for configs[2] (english.200MB is not available
                      offline): 200 MiB iid printable bytes (sigma=95), full build + 1M 20-symbol count().
N > 1: one process per GPU (torchrun, or spawned here when WORLD_SIZE is unset): the sharded
  construction (hkcsa_build_sa_sharded: RCCL all-reduce of the partition histogram and of the slice
  counts, independent slice sorts, RCCL all-gather of per-rank status; ISA rank exchange by RCCL
  all-gather only for texts whose ties outlast the chunk refinement).
    default (weak):   N GiB of text on N GPUs (1 GiB of suffixes per GPU);
    --strong:         a fixed --strong-bytes text (default 4 GiB = configs[4]) on N GPUs; at N = 1 a text
                      with >= 2^32 - 1 suffixes is one hkcsa_build_sa call (the library builds it as slices
                      of ~2^30 suffixes one after another into one full u64 SA / BWT).
  value = all suffixes' MB / max-over-ranks time.  After the timed steps every rank all-gathers the
  SA slices and BWT rows (replicas), builds its wavelet tree and locates its 1/N of the patterns;
  locate_patterns_per_s = all patterns / max-over-ranks time.

The JSON line also carries:
  roofline      — the dominant kernel of the timed steps (largest summed time among the bucket
                  sort and the two radix passes) timed with HIP events on the library's stream:
                  achieved = its algorithmic bytes per launch / mean launch time, peak = 8000 GB/s
                  (MI355X HBM3E), traffic = PMC-measured HBM bytes per launch (profiles/
                  pmc_kernels.json); the other kernels under roofline["others"].
  cpu_baseline  — the pure-Python restatement of the reference (oracle/ref_port.py: naive suffix
                  sort, dense occ, left-spine WT, dict backward search), one core, on bounded
                  samples (rank 0, N = 1 only): the unmodified pipeline end to end at 2^17 symbols
                  and configs[0]'s reference stages at 1 MiB with the suffix array substituted.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "high-order-entropy-compressed-suffix-array_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "SA build MB/s + batched locate() patterns/s, 1 GiB text, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0
DNA = b"ACGT"
PRINTABLE = bytes(range(0x20, 0x7F))
BYTES256 = bytes(range(256))
PATTERN_WINDOW = 256 << 20   # patterns are drawn from a window of this many symbols at a seeded offset


def log(*a):
    print(*a, file=sys.stderr, flush=True)


# ---------------------------------------------------------------------------- CPU baseline
def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(sample_n: int, npat: int, c0_n: int, seed: int = 3) -> dict:
    """Reference algorithms restated in pure Python (oracle/ref_port.py), timed on this host, 1 core."""
    from oracle import oracle, ref_port
    rng = np.random.default_rng(seed)
    # (1) the unmodified reference pipeline (naive suffix sort) end to end at sample_n symbols
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
    del idx
    # (2) configs[0]: the reference stages at 1 MiB with the suffix array substituted (the naive
    # sort would need ~512 GiB there); the SA comes from the oracle's C suffix sort (not timed)
    t1 = oracle.synth_text(c0_n + 1, DNA, seed=seed + 1)
    t1s = t1.tobytes().decode("latin-1")
    sa = oracle.suffix_array(t1).tolist()
    stages = {}
    gc.collect()
    t0 = time.perf_counter()
    bwt = ref_port.bwt_of(t1s, sa)
    stages["bwt_s"] = time.perf_counter() - t0
    gc.collect()
    t0 = time.perf_counter()
    ref_port.left_spine_levels(bwt)
    stages["wt_s"] = time.perf_counter() - t0
    gc.collect()
    t0 = time.perf_counter()
    occ = ref_port.occ_table(bwt)
    stages["occ_s"] = time.perf_counter() - t0
    gc.collect()
    t0 = time.perf_counter()
    ref_port.count_table(t1s)
    stages["C_s"] = time.perf_counter() - t0
    port = ref_port.FMIndexPort.__new__(ref_port.FMIndexPort)
    port.text, port.suffix_array, port.bwt, port.occ = t1s, sa, bwt, occ
    port.count = ref_port.count_table(t1s)
    st1 = rng.integers(0, len(t1s) - 16, size=npat)
    pats1 = [t1s[s:s + 16] for s in st1]
    gc.collect()
    t0 = time.perf_counter()
    for p in pats1:
        port.find(p)
    t_q1 = time.perf_counter() - t0
    build1 = sum(stages.values())
    return {
        "value": round(len(tp) / 2**20 / t_build, 6),
        "unit": "MB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"EnhancedFMIndex restatement (naive SA + BWT + dense occ + C) on {len(tp)} iid ACGT "
                  f"symbols, median of 3; find() of {npat} 16-symbol substrings; plus configs[0]'s "
                  f"stages at {c0_n + 1} symbols with the SA substituted",
        "build_s": round(t_build, 4),
        "locate_patterns_per_s": round(npat / t_q, 1),
        "config0_1MiB": {"symbols": c0_n + 1, **{k: round(v, 4) for k, v in stages.items()},
                         "stages_MBps": round((c0_n + 1) / 2**20 / build1, 4),
                         "find_patterns_per_s": round(npat / t_q1, 1),
                         "sa": "substituted (oracle C suffix sort, not timed)"},
        "host_cpus": os.cpu_count(),
        "cpu_model": cpu_model(),
        "note": "1 of host_cpus cores used (the reference is single-threaded pure Python)",
    }


# ---------------------------------------------------------------------------- rooflines
# kernels whose roofline bench.py reports: the dominant one (largest summed time) as `roofline`,
# the others under roofline["others"]
ROOF_KERNELS = ("sa_bucket_sort", "radix_part_text", "radix_part", "radix_part_keys", "shard_slice_part",
                "radix_onesweep_text", "radix_onesweep", "byte_hist")
WT_KERNELS = ("wt_bits", "wt_partition")


def pmc_traffic_gb(name: str, leg: str = "") -> float | None:
    """HBM GB per launch of timer `name`'s kernel, measured with rocprofv3 PMC counters on this config
    (tools/kprof.py --pmc-json profiles/pmc_kernels.json, separate FETCH_SIZE / WRITE_SIZE passes; FETCH_SIZE
    x2 gfx950 correction for the wide streaming reads)."""
    p = os.path.join(ROOT, "profiles", "pmc_kernels.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return float((d[leg] if leg else d)[name]["traffic_gb_per_launch"])
    except Exception:
        return None


def kernel_roofline(dev, name: str, leg: str = "") -> dict | None:
    launches, ms, alg_bytes = dev.kernel_stats(name)
    if not launches:
        return None
    per_launch_bytes = alg_bytes / launches
    avg_s = ms / launches / 1e3
    achieved = per_launch_bytes / avg_s / 1e9
    return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": pmc_traffic_gb(name, leg), "kernel": name,
            "launches": launches, "avg_launch_ms": round(ms / launches, 4), "total_ms": round(ms, 3),
            "alg_bytes_per_launch": per_launch_bytes}


def roofline(dev, names=ROOF_KERNELS, leg: str = "", traffic_gb: float | None = None) -> dict:
    rows = [r for r in (kernel_roofline(dev, k, leg) for k in names) if r]
    if not rows:
        return {"bound": "hbm", "achieved": None, "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": None,
                "traffic": None}
    dom = max(rows, key=lambda r: r["total_ms"])
    if traffic_gb is not None:
        dom["traffic"] = traffic_gb
    dom["others"] = [{k: r[k] for k in ("kernel", "achieved", "frac", "traffic", "avg_launch_ms")}
                     for r in rows if r is not dom]
    return dom


def stage_breakdown(dev, names) -> dict:
    out = {}
    for nm in names:
        l, ms, b = dev.kernel_stats(nm)
        if l:
            out[nm] = {"launches": l, "ms": round(ms, 3)}
    return out


BUILD_STAGES = ["byte_hist", "sa_bucket_hist", "radix_part_text", "radix_part_keys", "radix_part", "sa_digit_hist",
                "sa_bin_starts",
                "sa_bucket_sort", "sa_big_gather", "radix_onesweep_text", "radix_table_text", "radix_tile_hist", "radix_hist", "radix_onesweep",
                "radix_onesweep_small", "sa_pack_keys", "sa_refine_stats", "sa_refine_apply", "sa_refine_keys", "sa_refine_segsort",
                "sa_isa_scatter", "sa_group_stats", "sa_group_apply", "sa_pair_keys", "sa_pair_segsort", "sa_big_groups",
                "sa_round_plan", "sa_round_chunk", "sa_round_dbl", "sa_link", "bwt_gather"]
SHARD_STAGES = ["shard_hist", "shard_below", "shard_slice_hist", "shard_slice_part", "shard_select_count",
                "shard_pack_select", "rccl_allreduce_bytes",
                "rccl_allreduce_hist",
                "rccl_allreduce_counts", "rccl_allgather_status", "rccl_allgather_sa", "rccl_allgather_pairs",
                "sa_isa_update", "shard_split_join"] + BUILD_STAGES


# ---------------------------------------------------------------------------- pattern sets
def pattern_batch(dev, n: int, count: int, plen: int, seed: int) -> tuple[np.ndarray, np.ndarray]:
    """count substrings of length plen drawn uniformly from a seeded window of the device text."""
    rng = np.random.default_rng(seed)
    win = min(n - 1, PATTERN_WINDOW)
    w0 = int(rng.integers(0, n - win)) if n - win > 0 else 0
    txt = dev.text(w0, w0 + win)
    starts = rng.integers(0, win - plen, size=count).astype(np.int64)
    data = txt[starts[:, None] + np.arange(plen)[None, :]].reshape(-1)
    offs = np.arange(count + 1, dtype=np.uint64) * plen
    return np.ascontiguousarray(data), offs


def time_queries(dev, data, offs, reps: int) -> dict:
    q = dev.queries(data=data, offs=offs)
    P = len(offs) - 1
    total = q.locate()
    q.count()
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        total = q.locate()
    dev.synchronize()
    t_loc = (time.perf_counter() - t0) / reps
    t0 = time.perf_counter()
    for _ in range(reps):
        q.count()
    dev.synchronize()
    t_cnt = (time.perf_counter() - t0) / reps
    q.close()
    return {"patterns": P, "plen": int(offs[1] - offs[0]) if P else 0, "occurrences": int(total),
            "locate_s": t_loc, "count_s": t_cnt,
            "locate_patterns_per_s": round(P / t_loc, 1), "count_patterns_per_s": round(P / t_cnt, 1)}


def pmc_row(name: str) -> dict:
    """The PMC row of timer `name` in profiles/pmc_kernels.json (tools/kprof.py --pmc-json), or {}."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_kernels.json")) as f:
            return json.load(f).get(name, {})
    except Exception:
        return {}


def count_roofline(dev, data, offs, reps: int, sigma_codes: int) -> dict:
    """The batched count kernel (k_count, one lane per pattern) against HBM: its algorithmic bytes per pattern
    are the pattern, the k-mer table entry of its last K symbols, two 64-B occ-directory lines (+ an 8-B
    superblock prefix each) per remaining LF step and the (l, r) + count outputs; the time is the kernel's own
    HIP events.  L2 hit rate, HBM traffic and occupancy come from the committed rocprofv3 row (pmc_row)."""
    P = len(offs) - 1
    plen = int(offs[1] - offs[0]) if P else 0
    K, tot = 0, 1
    while K < 12 and tot * sigma_codes <= (1 << 21):   # hk_wt.hip build_wt: sigma^K <= 2^21 with a directory
        tot *= sigma_codes
        K += 1
    steps = max(plen - K, 0)
    occ = sigma_codes <= 9   # sigma <= 8 (+ '$'): the flat occ directory, one line per rank; else two (16-ary)
    per_pat = plen + 16 + steps * 2 * ((64 if occ else 128) + 8) + 16 + 8
    q = dev.queries(data=data, offs=offs)
    q.count()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    for _ in range(reps):
        q.count()
    dev.synchronize()
    launches, ms, _ = dev.kernel_stats("fm_count")
    dev.timing(False)
    q.close()
    if not launches:
        return {}
    avg_s = ms / launches / 1e3
    achieved = P * per_pat / avg_s / 1e9
    pmc = pmc_row("fm_count")
    return {"kernel": "k_count<16,1> (occ directory + k-mer table)" if occ else "k_count<16,2> (16-ary directory)",
            "bound": "hbm", "patterns": P, "plen": plen,
            "kmer_k": K, "lf_steps": steps, "alg_bytes_per_pattern": per_pat, "avg_launch_ms": round(avg_s * 1e3, 4),
            "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc.get("traffic_gb_per_launch"), "l2_hit": pmc.get("l2_hit"),
            "waves_per_cu": pmc.get("waves_per_cu"), "pmc_source": "profiles/pmc_kernels.json" if pmc else None,
            "note": "random 64-B line reads: the line count, not the bytes used, is the HBM cost"}


def time_wt(dev, reps: int) -> float:
    dev.build_wt()            # warm: first-call allocations happen here
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dev.build_wt()
    dev.synchronize()
    return (time.perf_counter() - t0) / reps


# ---------------------------------------------------------------------------- single GPU
def build_leg(alpha: bytes, n: int, steps: int, warmup: int, seed: int, flags: int = 0):
    from hkcsa import DeviceIndex
    dev = DeviceIndex.synthetic(n, alpha, seed=seed, device=0, flags=flags)
    for _ in range(warmup):
        dev.build_sa()
        dev.build_bwt()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    t0 = time.perf_counter()
    for _ in range(steps):
        dev.build_sa()          # includes the byte histogram / C array of every build
        dev.build_bwt()         # no-op: the bucket sorts write the BWT with the SA
    dev.synchronize()
    wall = time.perf_counter() - t0
    return dev, wall


def pcie_inclusive(n: int, alpha: bytes, seed: int) -> dict:
    """The host-buffer boundary once, after the timed steps (never the bench value):
    host text -> HBM (hkcsa_create), SA + BWT build, SA and BWT back to host buffers."""
    from hkcsa import DeviceIndex
    rng = np.random.default_rng(seed)
    sym = np.frombuffer(alpha, dtype=np.uint8)
    text = np.empty(n, dtype=np.uint8)
    text[:-1] = sym[rng.integers(0, len(alpha), n - 1, dtype=np.uint8)]
    text[-1] = ord("$")
    t0 = time.perf_counter()
    dev = DeviceIndex.from_bytes(text, device=0)
    t1 = time.perf_counter()
    dev.build_sa()
    dev.synchronize()
    t2 = time.perf_counter()
    sa = dev.sa()
    bwt = dev.bwt()
    t3 = time.perf_counter()
    dev.close()
    del sa, bwt, text
    return {"upload_ms": round((t1 - t0) * 1e3, 2), "build_ms": round((t2 - t1) * 1e3, 2),
            "download_ms": round((t3 - t2) * 1e3, 2), "MBps": round(n / 2**20 / (t3 - t0), 2),
            "note": "one cold run from a host text to host SA (u64, widened on the GPU) + BWT buffers: "
                    "includes the handle's first allocations and both PCIe copies"}


def run_single(args) -> dict:
    n = args.text_bytes + 1
    alpha = {4: DNA, 95: PRINTABLE, 256: BYTES256}[args.sigma]
    dev, wall = build_leg(alpha, n, args.steps, args.warmup, args.seed, flags=4 if args.global_sort else 0)
    value = args.steps * n / 2**20 / wall
    info = dev.build_info()
    leg = "" if args.sigma == 4 else f"sigma{args.sigma}"
    roof = roofline(dev, ROOF_KERNELS, leg, args.traffic_gb)
    stages = stage_breakdown(dev, BUILD_STAGES)
    log(f"[bench] sigma={args.sigma} SA+BWT {wall / args.steps * 1e3:.2f} ms/step -> {value:.1f} MB/s; "
        f"info={info[:8]}")
    dev.timing_reset()
    t_wt = time_wt(dev, args.wt_reps)
    wt_roof = roofline(dev, WT_KERNELS, leg)
    dev.timing(False)
    loc = eps = loc_host = cnt_roof = None
    if args.patterns > 0:
        data, offs = pattern_batch(dev, n, args.patterns, args.plen, args.seed + 1)
        loc = time_queries(dev, data, offs, args.query_reps)
        cnt_roof = count_roofline(dev, data, offs, args.query_reps, len(set(alpha)) + 1)
        loc_host = locate_host_leg(dev, data, offs, args.query_reps, loc)
        log(f"[bench] locate at the host boundary: {loc_host['locate_patterns_per_s']:.3g} patterns/s")
        if args.eps:
            eps = epsilon_leg(dev, n, data, offs, args.query_reps, loc)
    dev.close()
    pcie = pcie_inclusive(n, alpha, args.seed + 7) if args.pcie else None
    harness = harness_leg(n, args.seed + 8) if args.harness and args.sigma == 4 else None
    if harness:
        log(f"[bench] harness: construction {harness['construction_s']:.3f} s, locate by length "
            f"{harness['locate_s_by_length']}")
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
        "config": {"workload": f"{n - 1} iid sigma={args.sigma} symbols + '$': SA + BWT by the HIP bucket "
                               "build (byte histogram, bucket counts + two cursor scatter passes over the "
                               "bucket bits, LDS bucket sorts writing SA and BWT, tie refinement; configs[1] "
                               "pipeline at the "
                               "metric's 1 GiB), then warm WT build + batched "
                               f"{args.plen}-symbol locate()",
                   "text_symbols": n, "sigma": args.sigma, "positions": "u32"},
        "roofline": roof,
        "locate_patterns_per_s": loc["locate_patterns_per_s"] if loc else None,
        "full_build_MBps": round(n / 2**20 / (wall / args.steps + t_wt), 2),
        "detail": {"wt_build_ms": round(t_wt * 1e3, 3), "wt_roofline": wt_roof, "locate": loc,
                   "count_roofline": cnt_roof,
                   "pattern_source": f"uniform substrings of a {PATTERN_WINDOW >> 20} MiB window of the text",
                   "stages_ms_total": stages, "build_info": info[:16], "pcie_inclusive": pcie,
                   "epsilon": eps, "locate_host": loc_host, "harness": harness},
    }
    return res


def epsilon_leg(dev, n: int, data, offs, reps: int, full: dict) -> dict:
    """CompressedSuffixArray(text, epsilon=0.5)'s compact mode on the bench index (tests/benchmark.py:25,
    32,47): SA/ISA samples every ceil(log2(n) ** 0.5) positions + compact (the SA, BWT and text leave
    HBM), timed once, then the same patterns located by LF walks over the wavelet tree (identical
    answers: tests/test_gpu_parity.py test_sampled_*).  Runs last: the index keeps only samples."""
    from csa.csa import sample_rate
    rate = sample_rate(n, 0.5)
    dev.synchronize()
    # EnhancedFMIndex.__init__ drops the construction workspace after every build (csa/enhanced_fm_index.py);
    # timed on its own, then the epsilon part: samples + compaction (SA, BWT array and text released)
    t0 = time.perf_counter()
    dev.release_workspace()
    t_ws = time.perf_counter() - t0
    dev.timing_reset()
    dev.timing(True)
    t0 = time.perf_counter()
    dev.build_samples(rate)
    dev.synchronize()
    t_smp = time.perf_counter() - t0
    dev.compact()
    dev.synchronize()
    t_s = time.perf_counter() - t0
    smp_ms = {k: round(dev.kernel_stats(k)[1], 3) for k in ("smp_mark", "smp_fill", "smp_fix")}
    sp = dev.space()
    dev.timing_reset()
    qq = time_queries(dev, data, offs, reps)
    l, ms, _ = dev.kernel_stats("fm_locate_sampled")
    dev.timing(False)
    if qq["occurrences"] != full["occurrences"]:
        raise RuntimeError("sampled locate disagrees with the full-SA locate")
    log(f"[bench] epsilon=0.5 (rate {rate}): samples+compact {t_s * 1e3:.2f} ms, "
        f"locate {qq['locate_patterns_per_s']:.3g} patterns/s")
    return {"epsilon": 0.5, "sample_rate": rate, "samples_compact_ms": round(t_s * 1e3, 3),
            "samples_ms": round(t_smp * 1e3, 3), "compact_ms": round((t_s - t_smp) * 1e3, 3),
            "workspace_release_ms": round(t_ws * 1e3, 3),
            "sample_kernels_ms": smp_ms, "space_bytes": sp,
            "locate_patterns_per_s": qq["locate_patterns_per_s"], "count_patterns_per_s": qq["count_patterns_per_s"],
            "locate_sampled_kernel_ms": round(ms / max(1, l), 4), "occurrences": qq["occurrences"],
            "patterns": qq["patterns"], "plen": qq["plen"],
            "vs_full_sa_locate": round(qq["locate_patterns_per_s"] / full["locate_patterns_per_s"], 4)}


def run_extra_legs(args, res: dict):
    """configs[3] (sigma=256, 1 GiB) and the configs[2] stand-in (sigma=95, 200 MiB)."""
    legs = {}
    if args.sigma != 256:
        n = (1 << 30) + 1
        dev, wall = build_leg(BYTES256, n, args.leg_steps, 1, args.seed + 10)
        roof = roofline(dev, ROOF_KERNELS, "sigma256")
        stages = stage_breakdown(dev, BUILD_STAGES)
        dev.timing_reset()
        t_wt = time_wt(dev, args.wt_reps)
        wt_roof = roofline(dev, WT_KERNELS, "sigma256")
        dev.timing(False)
        info = dev.build_info()
        dev.close()
        legs["sigma256"] = {"config": "configs[3]: 1 GiB iid bytes sigma=256 + '$': SA + BWT steps, 8-level WT",
                            "text_symbols": n, "steps": args.leg_steps,
                            "ms_per_step": round(wall / args.leg_steps * 1e3, 3),
                            "sa_bwt_MBps": round(args.leg_steps * n / 2**20 / wall, 2),
                            "wt_build_ms": round(t_wt * 1e3, 3),
                            "full_build_MBps": round(n / 2**20 / (wall / args.leg_steps + t_wt), 2),
                            "roofline": roof, "wt_roofline": wt_roof, "stages_ms_total": stages,
                            "build_info": info[:16]}
        log(f"[bench] sigma256 leg: {legs['sigma256']['ms_per_step']} ms/step, WT {t_wt * 1e3:.2f} ms")
    legs["english_like_200MiB"] = english_leg(args)
    legs["protein_like_1GiB"] = protein_leg(args)
    n = 200 * (1 << 20) + 1
    dev, wall = build_leg(PRINTABLE, n, args.leg_steps, 1, args.seed + 20)
    dev.timing_reset()
    t_wt = time_wt(dev, args.wt_reps)
    data, offs = pattern_batch(dev, n, args.patterns or 1_000_000, 20, args.seed + 21)
    dev.timing_reset()
    dev.timing(True)
    qq = time_queries(dev, data, offs, args.query_reps)
    l, ms, _ = dev.kernel_stats("fm_count")
    dev.timing(False)
    dev.close()
    legs["printable_200MiB"] = {
        "config": "stand-in for configs[2] (english.200MB absent offline: not run): 200 MiB iid printable "
                  "bytes (sigma=95) + '$', full build + batched 20-symbol count()",
        "text_symbols": n, "ms_per_step": round(wall / args.leg_steps * 1e3, 3),
        "wt_build_ms": round(t_wt * 1e3, 3),
        "full_build_MBps": round(n / 2**20 / (wall / args.leg_steps + t_wt), 2),
        "count_patterns_per_s": qq["count_patterns_per_s"], "locate_patterns_per_s": qq["locate_patterns_per_s"],
        "fm_count_kernel_ms": round(ms / max(1, l), 4), "patterns": qq["patterns"], "plen": 20}
    log(f"[bench] printable leg: count {qq['count_patterns_per_s']:.3g} patterns/s")
    res["detail"]["legs"] = legs


def english_leg(args) -> dict:
    """configs[2]'s shape without its corpus (english.200MB is absent offline): 200 MiB of seeded
    natural-language-like latin-1 text (utils/textgen.py: Zipf words, punctuation, 25 % verbatim copies of
    50 - 5000 symbols plus a few of 64 KiB - 1 MiB), generated on the host (untimed) and uploaded; SA + BWT
    steps with the refinement / prefix-doubling stage times, the WT, 1M batched 20-symbol count()."""
    from hkcsa import DeviceIndex
    from utils.textgen import english_like_text
    n = 200 * (1 << 20) + 1
    t0 = time.perf_counter()
    text = english_like_text(n, seed=args.seed + 30)
    gen_s = time.perf_counter() - t0
    dev = DeviceIndex.from_bytes(text, device=0)
    del text
    dev.build_sa()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    t0 = time.perf_counter()
    for _ in range(args.leg_steps):
        dev.build_sa()
        dev.build_bwt()
    dev.synchronize()
    wall = time.perf_counter() - t0
    stages = stage_breakdown(dev, BUILD_STAGES)
    info = dev.build_info()
    dev.timing_reset()
    t_wt = time_wt(dev, args.wt_reps)
    data, offs = pattern_batch(dev, n, args.patterns or 1_000_000, 20, args.seed + 31)
    dev.timing_reset()
    qq = time_queries(dev, data, offs, args.query_reps)
    l, ms, _ = dev.kernel_stats("fm_count")
    dev.timing(False)
    dev.close()
    refine = ("sa_refine_stats", "sa_refine_apply", "sa_refine_keys", "sa_refine_segsort", "radix_onesweep_small",
              "radix_hist", "radix_onesweep", "sa_round_chunk")
    dbl = ("sa_isa_scatter", "sa_pair_keys", "sa_pair_segsort", "sa_group_stats", "sa_group_apply", "sa_round_dbl",
           "sa_round_plan", "sa_big_groups", "sa_link")
    per = lambda names: round(sum(stages.get(k, {}).get("ms", 0.0) for k in names) / args.leg_steps, 3)
    log(f"[bench] english-like leg: {wall / args.leg_steps * 1e3:.2f} ms/step, refinement {per(refine)} ms, "
        f"doubling {per(dbl)} ms, count {qq['count_patterns_per_s']:.3g} patterns/s")
    return {"config": "configs[2] shape (english.200MB absent offline): 200 MiB natural-language-like latin-1 text "
                      "(utils/textgen.py english_like, seed %d) + '$': SA + BWT steps, WT, batched 20-symbol count()"
                      % (args.seed + 30),
            "text_symbols": n, "generate_s": round(gen_s, 2), "steps": args.leg_steps,
            "ms_per_step": round(wall / args.leg_steps * 1e3, 3),
            "sa_bwt_MBps": round(args.leg_steps * n / 2**20 / wall, 2),
            "refinement_ms_per_step": per(refine), "doubling_ms_per_step": per(dbl),
            "chunk_rounds": info[2] & 0xFFFFFFFF, "doubling_rounds": info[2] >> 32,
            "tied_after_round": info[9:9 + 24], "wt_build_ms": round(t_wt * 1e3, 3),
            "full_build_MBps": round(n / 2**20 / (wall / args.leg_steps + t_wt), 2),
            "count_patterns_per_s": qq["count_patterns_per_s"], "locate_patterns_per_s": qq["locate_patterns_per_s"],
            "fm_count_kernel_ms": round(ms / max(1, l), 4), "patterns": qq["patterns"], "plen": 20,
            "stages_ms_total": stages, "build_info": info[:9]}


def protein_leg(args) -> dict:
    """The proteins corpus shape of the reference's dataset bench (tests/dataset_benchmark.py:13), absent
    offline: 1 GiB of seeded protein-database-like text (utils/textgen.py protein_like: 25 amino-acid letters
    at natural frequencies + newlines, 35 % family members with 8 % substitutions, 5 % duplicates), generated
    on the host (untimed) and uploaded; SA + BWT steps (non-power-of-two alphabet: the stable onesweep
    pair, LDS bucket sorts, refinement)."""
    from hkcsa import DeviceIndex
    from utils.textgen import protein_like_text
    n = int(os.environ.get("BENCH_PROTEIN_MIB", "1024")) * (1 << 20) + 1   # (size override: experiments)
    t0 = time.perf_counter()
    text = protein_like_text(n, seed=args.seed + 40)
    gen_s = time.perf_counter() - t0
    dev = DeviceIndex.from_bytes(text, device=0)
    del text
    dev.build_sa()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    t0 = time.perf_counter()
    for _ in range(args.leg_steps):
        dev.build_sa()
        dev.build_bwt()
    dev.synchronize()
    wall = time.perf_counter() - t0
    stages = stage_breakdown(dev, BUILD_STAGES)
    info = dev.build_info()
    dev.timing(False)
    dev.close()
    log(f"[bench] protein-like leg: {wall / args.leg_steps * 1e3:.2f} ms/step")
    return {"config": "proteins corpus shape (tests/dataset_benchmark.py:13; absent offline): 1 GiB protein-like "
                      "text (utils/textgen.py protein_like, seed %d) + '$': SA + BWT steps" % (args.seed + 40),
            "text_symbols": n, "generate_s": round(gen_s, 2), "steps": args.leg_steps,
            "ms_per_step": round(wall / args.leg_steps * 1e3, 3),
            "sa_bwt_MBps": round(args.leg_steps * n / 2**20 / wall, 2),
            "tied_after_round": info[9:9 + 24], "stages_ms_total": stages, "build_info": info[:9]}


def locate_host_leg(dev, data, offs, reps: int, full: dict) -> dict:
    """hkcsa_locate_batch at the host boundary: the same patterns from host buffers, CSR offsets and
    positions back into caller-owned host arrays (tests/benchmark.py:39-52 times csa.locate(p) returning
    a list; this is its batched C-ABI form).  PCIe copies and the allocations inside the call included."""
    occ, pos = dev.locate_batch(data, offs)            # warm; also learns the size
    cap = len(pos)
    if len(pos) != full["occurrences"]:
        raise RuntimeError("host-boundary locate disagrees with the device-resident locate")
    dev.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        occ, pos = dev.locate_batch(data, offs, cap=cap)
    t = (time.perf_counter() - t0) / reps
    P = len(offs) - 1
    return {"patterns": P, "plen": full["plen"], "occurrences": int(len(pos)), "call_s": round(t, 6),
            "locate_patterns_per_s": round(P / t, 1),
            "in_bytes": int(data.nbytes + offs.nbytes), "out_bytes": int(occ.nbytes + pos.nbytes),
            "vs_device_resident": round(P / t / full["locate_patterns_per_s"], 4),
            "note": "one hkcsa_locate_batch call per batch (cap known): H2D patterns, count, scan, SA gather, "
                    "D2H offsets + positions into pageable numpy arrays"}


def harness_leg(n: int, seed: int, lengths=(5, 10, 50, 100, 500, 1000), iterations: int = 3) -> dict:
    """The reference harness (tests/benchmark.py:54-89) as utils.benchmark.run_full_benchmark on the
    bench text (1 GiB iid ACGT, epsilon = 0.5): construction through the str API (codec, upload, SA, BWT, WT,
    samples, compaction), then `iterations` csa.locate(p) calls per pattern length, each returning a list."""
    from hkcsa import DeviceIndex
    from utils.benchmark import run_full_benchmark
    dev = DeviceIndex.synthetic(n, DNA, seed=seed, device=0)
    text = dev.text(0, n - 1).tobytes().decode("latin-1")   # the text without the '$' the class appends
    dev.close()
    res = run_full_benchmark(text, lengths, iterations, epsilon=0.5, seed=seed, verbose=False)
    del text
    gc.collect()
    return {"text_symbols": n, "epsilon": 0.5, "construction_s": round(res.construction_time, 4),
            "construction_MBps": round(n / 2**20 / res.construction_time, 2),
            "device_bytes": int(res.device_bytes),
            "locate_s_by_length": {int(k): round(v, 6) for k, v in sorted(res.pattern_times.items())},
            "occurrences_by_length": {int(k): int(v) for k, v in sorted(res.occurrences.items())},
            "iterations": iterations,
            "note": "run_full_benchmark(text) over csa.CompressedSuffixArray: per-length mean of csa.locate(p), "
                    "host str in, Python list out"}


# ---------------------------------------------------------------------------- sharded / multi-GPU
def strong_leg(args, rank: int, world: int, local_rank: int, uid) -> dict:
    """configs[4]'s fixed text (--strong-bytes, 4 GiB + '$') over the same ranks after the weak-scaling line
    (SURVEY.md §8e's 1 -> 8 curve in both modes): one warm-up and up to three timed sharded builds,
    barrier-bracketed, max over ranks."""
    import torch
    import torch.distributed as dist
    from hkcsa import DeviceIndex
    n = args.strong_bytes + 1
    dev = DeviceIndex.synthetic(n, DNA, seed=args.seed, device=local_rank, flags=1 if args.pos64 else 0)
    steps = max(1, min(args.steps, 3))
    single = world == 1 and n >= (1 << 32) - 1   # (one rank: the library's own slices, as run_sharded)

    def step():
        if single:
            dev.build_sa()
        else:
            dev.build_sa_sharded(uid, world, rank)

    step()
    dev.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    dev.synchronize()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.barrier()
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    lo, hi = (0, n) if single else dev.shard_range()
    dev.close()
    wall = float(el.item())
    return {"text_symbols": n, "scaling": "strong", "n_gpus": world, "steps": steps,
            "ms_per_step": round(wall / steps * 1e3, 3), "MBps": round(steps * n / 2**20 / wall, 2),
            "rank0_slice": [lo, hi], "note": "configs[4]: the same 4 GiB text at every N (strong scaling)"}


def run_sharded(args, rank: int, world: int, local_rank: int) -> dict | None:
    import torch
    import torch.distributed as dist
    from hkcsa import DeviceIndex, comm_unique_id
    torch.cuda.set_device(local_rank)
    n = (args.strong_bytes if args.strong else args.text_bytes * world) + 1
    flags = 1 if args.pos64 else 0
    dev = DeviceIndex.synthetic(n, DNA, seed=args.seed, device=local_rank, flags=flags)
    uid = [comm_unique_id() if rank == 0 else None]
    dist.broadcast_object_list(uid, src=0)
    uid = uid[0]
    # one slice per rank; at N = 1 a text of >= 2^32 - 1 suffixes is the single-GPU library build
    # (hkcsa_build_sa: slices of ~2^30 suffixes one after another into one full u64 SA / BWT)
    single = world == 1 and n >= (1 << 32) - 1
    per_gpu = max(2, (n + (1 << 29)) >> 30) if single else 1   # (hk_shard.hip slices_for)

    def step():
        if single:
            dev.build_sa()
        else:
            dev.build_sa_sharded(uid, world, rank)

    for _ in range(args.warmup):
        step()
    dev.synchronize()
    dev.timing_reset()
    dev.timing(True)
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dev.synchronize()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    dist.barrier()
    dev.timing(False)
    el = torch.tensor([t1 - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX)
    wall = float(el.item())
    lo, hi = (0, n) if single else dev.shard_range()
    roof = roofline(dev, ROOF_KERNELS, "", args.traffic_gb)
    if args.traffic_gb is None:   # the PMC summaries in profiles/ are of the single-GPU launches
        roof["traffic"] = None
        for o in roof.get("others", []):
            o["traffic"] = None
    stages = stage_breakdown(dev, SHARD_STAGES)
    info = dev.build_info()[:16]
    # ---- replicas + batched locate (patterns split P/N over the ranks)
    loc = None
    if args.patterns > 0:
        dev.release_workspace()
        dist.barrier()
        t0 = time.perf_counter()
        if not single:
            dev.shard_replicate()
        dev.synchronize()
        t_rep = time.perf_counter() - t0
        t_wt = time_wt(dev, args.wt_reps)
        data, offs = pattern_batch(dev, n, args.patterns, args.plen, args.seed + 1)
        P = args.patterns
        a, b = P * rank // world, P * (rank + 1) // world
        mine_d = data[int(offs[a]):int(offs[b])]
        mine_o = offs[a:b + 1] - offs[a]
        dist.barrier()
        qq = time_queries(dev, mine_d, mine_o, args.query_reps)
        ts = torch.tensor([qq["locate_s"], qq["count_s"], t_rep, t_wt], dtype=torch.float64)
        dist.all_reduce(ts, op=dist.ReduceOp.MAX)
        occ = torch.tensor([qq["occurrences"]], dtype=torch.int64)
        dist.all_reduce(occ)
        loc = {"patterns": P, "plen": args.plen, "occurrences": int(occ.item()),
               "locate_patterns_per_s": round(P / float(ts[0]), 1), "count_patterns_per_s": round(P / float(ts[1]), 1),
               "replicate_ms": round(float(ts[2]) * 1e3, 2), "wt_build_ms": round(float(ts[3]) * 1e3, 2),
               "split": f"P/{world} patterns per rank, max-over-ranks time"}
    dev.close()
    strong = None
    if (world > 1 or args.sharded) and not args.strong and not single and args.strong_leg:
        strong = strong_leg(args, rank, world, local_rank, uid)
    res = None
    if rank == 0:
        value = args.steps * n / 2**20 / wall
        scaling = "strong" if args.strong else "weak"
        res = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "MB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic",
            "config": {"workload": f"{n - 1} iid sigma=4 symbols + '$' sharded over {world} GPUs"
                                   + (f" (one handle: hkcsa_build_sa builds {per_gpu} slices one after another "
                                      "into the full u64 SA / BWT)" if single else "")
                                   + ": partition histogram + slice counts by RCCL all-reduce, per-rank slice "
                                   "selection, LSD passes over the slice's bucket bits, LDS bucket sorts, tie "
                                   "refinement, RCCL all-gather of per-rank status (ISA rank exchange only for "
                                   "ties that outlast the chunk rounds); then replicas + batched locate",
                       "text_symbols": n, "sigma": 4, "parallelism": f"sa-slices x{world}",
                       "positions": "u64" if (n >= 2**32 - 1 or args.pos64) else "u32"},
            "roofline": roof,
            "locate_patterns_per_s": loc["locate_patterns_per_s"] if loc else None,
            "detail": {"rank0_slice": [lo, hi], "slices_per_gpu": per_gpu, "locate": loc,
                       "stages_ms_total": stages, "build_info": info, "strong_4GiB": strong},
        }
        if not args.no_cpu_baseline:   # rank 0's host cores, after every timed region (the other ranks wait)
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_patterns, args.cpu_config0)
    dist.barrier()
    return res


# ---------------------------------------------------------------------------- launch
def _stdout_for_result():
    """Route fd 1 to stderr for the run (RCCL / gloo print banners on stdout) and return a
    stream on the original stdout, so the result stays the only line there."""
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    return os.fdopen(saved, "w")


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_check(rank: int, world: int) -> dict | None:
    """--launch-check: the rendezvous and max-over-ranks reduction of a multi-GPU run, no GPU work
    (CPU test of the launch logic, tests/test_bench_cpu.py)."""
    import torch
    import torch.distributed as dist
    dist.barrier()
    t = torch.tensor([float(rank)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    if rank:
        return None
    return {"metric": METRIC, "value": None, "unit": "MB/s", "n_gpus": world, "launch_check":
            {"world": world, "max_rank": int(t.item()), "local_rank": int(os.environ.get("LOCAL_RANK", "-1"))}}


def _rank_entry(argv, rank, world, port, q):
    """Spawned worker (one process per GPU): fresh interpreter, no GPU state inherited."""
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank), "LOCAL_WORLD_SIZE": str(world)})
    args = parse_args(argv)
    import torch.distributed as dist
    dist.init_process_group(backend="gloo")
    try:
        res = launch_check(rank, world) if args.launch_check else run_sharded(args, rank, world, rank)
        if rank == 0:
            q.put(res)
        dist.barrier()
    finally:
        dist.destroy_process_group()


def spawn_ranks(argv, world: int) -> dict:
    """--gpus N without a launcher: start N worker processes (before this process touches the GPU)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_entry, args=(argv, r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = None
    while res is None:
        try:
            res = q.get(timeout=5)
        except Exception:
            dead = [p for p in procs if p.exitcode not in (None, 0)]
            if dead or all(p.exitcode is not None for p in procs):
                for p in procs:
                    if p.exitcode is None:
                        p.terminate()
                raise SystemExit(f"bench: a rank failed (exit codes {[p.exitcode for p in procs]})")
    for p in procs:
        p.join(timeout=300)
        if p.exitcode != 0:
            raise SystemExit(f"bench: rank exited with {p.exitcode}")
    return res


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--text-bytes", type=int, default=1 << 30, help="text symbols per GPU (before '$')")
    ap.add_argument("--sigma", type=int, default=4, choices=(4, 95, 256), help="alphabet of the headline text")
    ap.add_argument("--seed", type=int, default=2)
    ap.add_argument("--patterns", type=int, default=1_000_000)
    ap.add_argument("--plen", type=int, default=16)
    ap.add_argument("--query-reps", type=int, default=5)
    ap.add_argument("--wt-reps", type=int, default=3)
    ap.add_argument("--leg-steps", type=int, default=3)
    ap.add_argument("--no-legs", action="store_true", help="skip the sigma=256 and printable legs (N = 1)")
    ap.add_argument("--cpu-sample", type=int, default=1 << 17)
    ap.add_argument("--cpu-config0", type=int, default=1 << 20)
    ap.add_argument("--cpu-patterns", type=int, default=1000)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-eps", dest="eps", action="store_false",
                    help="skip the epsilon=0.5 compact-mode leg (samples + LF-walk locate) at N = 1")
    ap.add_argument("--no-pcie", dest="pcie", action="store_false",
                    help="skip the host-buffer (PCIe-inclusive) build after the timed steps")
    ap.add_argument("--no-harness", dest="harness", action="store_false",
                    help="skip run_full_benchmark (the reference harness) on the 1 GiB text at N = 1")
    ap.add_argument("--sharded", action="store_true", help="use the sharded (multi-GPU) build even at N=1")
    ap.add_argument("--strong", action="store_true", help="fixed text of --strong-bytes over the N GPUs")
    ap.add_argument("--strong-bytes", type=int, default=1 << 32)
    ap.add_argument("--pos64", action="store_true", help="sharded build with 64-bit positions at any n")
    ap.add_argument("--no-strong-leg", dest="strong_leg", action="store_false",
                    help="N > 1: skip configs[4]'s fixed 4 GiB (strong-scaling) leg after the weak-scaling line")
    ap.add_argument("--global-sort", action="store_true",
                    help="single-GPU build by full-width LSD sort of the keys (no LDS bucket sorts)")
    ap.add_argument("--only-leg", choices=("english", "protein"), default=None,
                    help="run only this detail leg (profiling): english = the 200 MiB English-like leg, "
                         "protein = the 1 GiB protein-like leg")
    ap.add_argument("--launch-check", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--traffic-gb", type=float, default=None,
                    help="PMC-measured HBM GB per launch of the dominant kernel; default: profiles/pmc_kernels.json")
    return ap.parse_args(argv)


def main():
    result_out = _stdout_for_result()
    argv = sys.argv[1:]
    args = parse_args(argv)
    launched = "WORLD_SIZE" in os.environ
    if args.gpus > 1 and not launched:
        res = spawn_ranks(argv, args.gpus)
    elif launched or args.gpus > 1 or args.sharded or args.strong:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        os.environ.setdefault("RANK", "0")
        os.environ.setdefault("WORLD_SIZE", "1")
        dist.init_process_group(backend="gloo")
        world = dist.get_world_size()
        rank = dist.get_rank()
        if world != args.gpus and rank == 0:
            log(f"[bench] note: WORLD_SIZE={world} (launcher) with --gpus {args.gpus}")
        if args.launch_check:
            res = launch_check(rank, world)
        else:
            res = run_sharded(args, rank, world, int(os.environ.get("LOCAL_RANK", "0")))
        dist.barrier()
        dist.destroy_process_group()
    elif args.only_leg == "english":
        res = {"leg": "english_like_200MiB", **english_leg(args)}
    elif args.only_leg == "protein":
        res = {"leg": "protein_like_1GiB", **protein_leg(args)}
    else:
        res = run_single(args)
        if not args.no_legs:
            run_extra_legs(args, res)
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(args.cpu_sample, args.cpu_patterns, args.cpu_config0)
    if res is not None:
        if "cpu_baseline" not in res:
            res["cpu_baseline"] = None
        print(json.dumps(res), file=result_out, flush=True)


if __name__ == "__main__":
    main()
