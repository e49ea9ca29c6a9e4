// hk_entropy.hip — empirical k-th order entropy H_k of T.
//
// Restates csa/high_order_entropy.py:4-32:
//   H_0 = -sum_c (n_c/n) log2(n_c/n)
//   H_k = sum over contexts w (|w| = k) of (n_w/n) * H_0(symbols following w), over the n-k
//         positions i < n-k (note: divided by n, not n-k), 0 when n <= k.
// With n_w the context total and n_wc the count of (w, c) pairs,
//   n·H_k = sum_w n_w log2 n_w - sum_(w,c) n_wc log2 n_wc,
// so only the run lengths of two groupings are needed, and the suffix array provides both: the
// suffixes i < n-k sorted, equal (k+1)-prefixes (w, c) and equal k-prefixes (w) are contiguous
// runs.  Suffixes shorter than k+1 are removed first (they sort ahead of their group, so the
// remaining runs stay contiguous).  Passes: compact valid SA entries; per adjacent pair the
// common prefix length capped at k+1 (random text reads); two run-length reductions in double.
// Floating point: per-block partial sums in double, summed on the host in block order —
// deterministic; parity with the reference is to a relative tolerance (test: 1e-9).
#include <cmath>

#include "hk_index.hpp"

namespace hk {
namespace {

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

__global__ __launch_bounds__(256) void k_hk_valid(const uint32_t* __restrict__ sa, uint64_t n, uint64_t lim,
                                                  uint32_t* __restrict__ flag) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256)
    flag[j] = sa[j] < lim ? 1u : 0u;
}

__global__ __launch_bounds__(256) void k_hk_compact(const uint32_t* __restrict__ sa, uint64_t n, uint64_t lim,
                                                    const uint64_t* __restrict__ pos, uint32_t* __restrict__ out) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256)
    if (sa[j] < lim) out[pos[j]] = sa[j];
}

// common prefix of suffixes a and b capped at cap (both have at least cap symbols)
__device__ __forceinline__ uint32_t lcp_capped(const uint8_t* __restrict__ t, uint64_t a, uint64_t b, uint32_t cap) {
  uint32_t l = 0;
  while (l < cap && t[a + l] == t[b + l]) ++l;
  return l;
}

// starts of runs: s0[j] = 1 if j opens a k-run (context), s1[j] = 1 if it opens a (k+1)-run
__global__ __launch_bounds__(256) void k_hk_bounds(const uint32_t* __restrict__ v, uint64_t m,
                                                   const uint8_t* __restrict__ t, uint32_t k,
                                                   uint32_t* __restrict__ s0, uint32_t* __restrict__ s1) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256) {
    const uint32_t l = j ? lcp_capped(t, v[j - 1], v[j], k + 1) : 0u;
    s0[j] = l < k ? 1u : 0u;
    s1[j] = l < k + 1 ? 1u : 0u;
  }
}

__global__ __launch_bounds__(256) void k_hk_starts(const uint32_t* __restrict__ s, const uint64_t* __restrict__ pos,
                                                   uint64_t m, uint64_t* __restrict__ starts) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256)
    if (s[j]) starts[pos[j]] = j;
}

// per-block partial of sum over runs of len * log2(len)
__global__ __launch_bounds__(256) void k_hk_runsum(const uint64_t* __restrict__ starts, uint64_t runs, uint64_t m,
                                                   double* __restrict__ part) {
  double acc = 0;
  for (uint64_t r = (uint64_t)blockIdx.x * 256 + threadIdx.x; r < runs; r += (uint64_t)gridDim.x * 256) {
    const uint64_t e = r + 1 < runs ? starts[r + 1] : m;
    const double len = (double)(e - starts[r]);
    acc += len * log2(len);
  }
  __shared__ double red[256];
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if ((int)threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
    __syncthreads();
  }
  if (threadIdx.x == 0) part[blockIdx.x] = red[0];
}

double run_log_sum(Index& ix, const uint32_t* d_flags, uint64_t m, hipStream_t s) {
  // exclusive scan of the start flags -> run index of every start; total = number of runs
  ix.tile_a.ensure((m + 1) * 8);
  scan_exclusive_u32_to_u64(ix.sw, d_flags, ix.tile_a.as<uint64_t>(), m, true, s);
  uint64_t runs = 0;
  HK_HIP(hipMemcpyAsync(&runs, ix.tile_a.as<uint64_t>() + m, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  ix.tile_c.ensure((runs + 1) * 8);
  k_hk_starts<<<grid_for(m), 256, 0, s>>>(d_flags, ix.tile_a.as<uint64_t>(), m, ix.tile_c.as<uint64_t>());
  HK_HIP(hipGetLastError());
  const unsigned g = grid_for(runs, 256, 2048);
  ix.tile_d.ensure((size_t)g * 8);
  k_hk_runsum<<<g, 256, 0, s>>>(ix.tile_c.as<uint64_t>(), runs, m, ix.tile_d.as<double>());
  HK_HIP(hipGetLastError());
  std::vector<double> part(g);
  HK_HIP(hipMemcpyAsync(part.data(), ix.tile_d.p, (size_t)g * 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  double sum = 0;
  for (double p : part) sum += p;
  return sum;
}

}  // namespace

double entropy_k(Index& ix, int k) {
  const uint64_t n = ix.n;
  if (k < 0 || n == 0) return 0.0;
  // H_0 needs only the byte histogram (kept after compact); H_k reads the text
  if (!ix.have_text && (k > 0 || !ix.have_alpha)) throw ApiError{-3, "entropy: text released by compact"};
  compute_alphabet(ix);
  if (k == 0) {   // csa/high_order_entropy.py:11-16
    double h = 0;
    for (int c = 0; c < 256; ++c)
      if (ix.byte_hist[c]) {
        const double p = (double)ix.byte_hist[c] / (double)n;
        h -= p * std::log2(p);
      }
    return h;
  }
  if (n <= (uint64_t)k) return 0.0;                // :18-19
  if (ix.sharded) throw ApiError{-3, "entropy: a sharded index holds only a slice"};
  if (!ix.have_sa) {   // the SA of the same text: an existing BWT / wavelet tree stays valid
    const bool wt = ix.have_wt;
    build_sa(ix);
    ix.have_wt = wt;
  }
  if (ix.sa_pos64) throw ApiError{-6, "entropy: 64-bit suffix arrays not supported"};
  hipStream_t s = ix.stream;
  const uint64_t m = n - (uint64_t)k;              // positions i < n - k
  const uint32_t* sa = ix.sa.as<uint32_t>();
  ix.seq[0].ensure(n * 4 + 16);                    // valid flags, then start flags (k)
  ix.seq[1].ensure(n * 4 + 16);                    // start flags (k+1)
  ix.isa.ensure(m * 4 + 16);                       // compacted suffixes
  ix.tile_b.ensure((n + 1) * 8);
  uint32_t* flag = ix.seq[0].as<uint32_t>();
  {
    TimedLaunch t(ix.timer, "hk_compact", (double)n * 16);
    k_hk_valid<<<grid_for(n), 256, 0, s>>>(sa, n, m, flag);
    HK_HIP(hipGetLastError());
    scan_exclusive_u32_to_u64(ix.sw, flag, ix.tile_b.as<uint64_t>(), n, false, s);
    k_hk_compact<<<grid_for(n), 256, 0, s>>>(sa, n, m, ix.tile_b.as<uint64_t>(), ix.isa.as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  {
    TimedLaunch t(ix.timer, "hk_bounds", (double)m * (4 + 8 + 2.0 * (k + 1)));
    k_hk_bounds<<<grid_for(m), 256, 0, s>>>(ix.isa.as<uint32_t>(), m, ix.text.as<uint8_t>(), (uint32_t)k,
                                            ix.seq[0].as<uint32_t>(), ix.seq[1].as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  const double ctx = run_log_sum(ix, ix.seq[0].as<uint32_t>(), m, s);
  const double pair = run_log_sum(ix, ix.seq[1].as<uint32_t>(), m, s);
  const double h = (ctx - pair) / (double)n;
  return h < 0 ? 0.0 : h;
}

}  // namespace hk
