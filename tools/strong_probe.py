"""Wall time of hkcsa_build_sa on configs[4]'s 4 GiB + 1 DNA text on one GPU, per call, with the kernel
time the library's own timers saw (the difference is host time: allocation, read-backs)."""
import os, sys, time
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "high-order-entropy-compressed-suffix-array_amd"))
from hkcsa import DeviceIndex

n = (1 << 32) + 1
dev = DeviceIndex.synthetic(n, b"ACGT", seed=2, device=0)
dev.timing(True)
for i in range(4):
    dev.timing_reset()
    t0 = time.perf_counter()
    dev.build_sa()
    dev.synchronize()
    wall = (time.perf_counter() - t0) * 1e3
    names = ("shard_hist", "shard_slice_hist", "shard_slice_part", "byte_hist", "radix_part", "sa_bucket_sort",
             "radix_hist", "radix_onesweep_small", "sa_refine_stats", "sa_refine_apply", "sa_refine_keys",
             "sa_refine_segsort", "sa_isa_scatter", "sa_pair_keys", "sa_group_stats", "sa_group_apply")
    ker = sum(dev.kernel_stats(k)[1] for k in names)
    print(f"build {i}: wall {wall:.1f} ms, timed kernels {ker:.1f} ms", flush=True)
dev.close()
