"""The reference's benchmark harness (tests/benchmark.py:1-112) over the GPU csa.CSA.

run_full_benchmark(text, pattern_lengths, iterations) builds CompressedSuffixArray(text,
epsilon) once, draws one pattern per length with generate_random_patterns, and times
`iterations` locate() calls per pattern — the reference's procedure (:54-89) and result fields
(BenchmarkResults, :15-22), with the memory columns as host RSS deltas (psutil, :10-13) and the
index's resident HBM bytes added as `device_bytes`.  print_benchmark_summary prints the
reference's summary table (:91-106).  memory_profiler (:5) is not used: it is not installed here
and only decorates the functions.
"""
from __future__ import annotations

import gc
import os
import time

from utils.patterns import generate_random_patterns


def get_process_memory() -> float:
    """Current RSS in MB (tests/benchmark.py:10-13)."""
    try:
        import psutil
        return psutil.Process(os.getpid()).memory_info().rss / 1024 / 1024
    except ImportError:
        return 0.0


class BenchmarkResults:
    def __init__(self):
        self.construction_time = 0
        self.construction_memory = 0
        self.pattern_times = {}
        self.pattern_memory = {}
        self.total_time = 0
        self.peak_memory = 0
        self.device_bytes = 0
        self.occurrences = {}


def benchmark_construction(text, epsilon=0.5):
    from csa.csa import CompressedSuffixArray
    gc.collect()
    m0 = get_process_memory()
    t0 = time.time()
    csa = CompressedSuffixArray(text, epsilon=epsilon)
    return csa, time.time() - t0, get_process_memory() - m0


def benchmark_pattern_search(csa, pattern):
    gc.collect()
    m0 = get_process_memory()
    t0 = time.time()
    locations = csa.locate(pattern)
    return locations, time.time() - t0, get_process_memory() - m0


def run_full_benchmark(text, pattern_lengths=(5, 10, 50, 100, 500, 1000), iterations=3, epsilon=0.5, seed=None,
                       verbose=True):
    say = print if verbose else (lambda *a, **k: None)
    res = BenchmarkResults()
    say("\nBenchmarking CSA Construction...")
    csa, res.construction_time, res.construction_memory = benchmark_construction(text, epsilon)
    say(f"Construction Time: {res.construction_time:.4f} seconds")
    say(f"Construction Memory: {res.construction_memory:.2f} MB")
    res.device_bytes = sum(v for k, v in csa.space().items() if k not in ("sample_rate", "sampled"))
    patterns = generate_random_patterns(text, list(pattern_lengths), seed=seed)
    say("\nBenchmarking Pattern Searches...")
    for pattern in patterns:
        times, mems = [], []
        say(f"\nPattern length: {len(pattern)}")
        for i in range(iterations):
            locations, t, m = benchmark_pattern_search(csa, pattern)
            times.append(t)
            mems.append(m)
            say(f"Iteration {i + 1}: Time={t:.4f}s, Memory={m:.2f}MB")
            say(f"Found {len(locations)} occurrences")
        res.pattern_times[len(pattern)] = sum(times) / iterations
        res.pattern_memory[len(pattern)] = sum(mems) / iterations
        res.occurrences[len(pattern)] = len(locations)
    res.total_time = res.construction_time + sum(res.pattern_times.values())
    res.peak_memory = max([res.construction_memory] + list(res.pattern_memory.values()))
    return res


def print_benchmark_summary(results):
    print("\n=== Benchmark Summary ===")
    print("\nConstruction:")
    print(f"Time: {results.construction_time:.4f} seconds")
    print(f"Memory: {results.construction_memory:.2f} MB")
    print("\nPattern Search (averages):")
    print("Pattern Length | Time (s) | Memory (MB)")
    print("-" * 40)
    for length in sorted(results.pattern_times.keys()):
        print(f"{length:>13} | {results.pattern_times[length]:>8.4f} | {results.pattern_memory[length]:>10.2f}")
    print("\nOverall:")
    print(f"Total Time: {results.total_time:.4f} seconds")
    print(f"Peak Memory: {results.peak_memory:.2f} MB")
