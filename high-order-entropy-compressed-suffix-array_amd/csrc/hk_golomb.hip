// hk_golomb.hip — Golomb-Rice code of a wavelet-tree level.
//
// Restates csa/wavelet_tree.py:27-63 (GolombRiceEncoder) as applied by build_tree (:84-86):
//   m     = 1 if the level has no ones, else max(1, int(log2(1 / (ones / len))))  — host double
//           arithmetic, the same IEEE operations and libm log2 as CPython's math.log2;
//   code  = for every maximal run of L ones, left to right: L // m zeros, a one, then L % m in
//           exactly m binary digits, most significant first; zeros emit nothing.
// The bit stream is packed LSB-first into u64 words (bit j -> word j/64, bit j%64), the layout of
// hkcsa_wt_level.
//
// Three word-parallel passes over the level's rank lines (8 u64 per line: ones-before + 7 data
// words), each reading the level once (n/8 bytes):
//   1. k_gr_starts: per data word, 1 + absolute position of its last run start (0 if none), and
//      the popcount of the prefix (one atomic per block) — then an exclusive max-scan gives, for
//      every word, the start of a run that enters it from the left;
//   2. k_gr_sizes: per word, the code length of the runs that END in it;  exclusive sum-scan ->
//      each word's output bit offset (and the total);
//   3. k_gr_write: each run ORs its (1, remainder) field — at most m + 1 <= 64 bits, two words —
//      into the zeroed output; the L // m zeros are implicit.
#include <cmath>

#include "hk_index.hpp"

namespace hk {
namespace {

// data word w of a level, restricted to the first nbits bits
__device__ __forceinline__ uint64_t level_word(const uint64_t* __restrict__ lines, uint64_t w, uint64_t nbits) {
  const uint64_t nw = (nbits + 63) / 64;
  if (w >= nw) return 0;
  uint64_t x = lines[(w / 7) * 8 + 1 + (w % 7)];
  const uint64_t rem = nbits - w * 64;
  if (rem < 64) x &= (1ull << rem) - 1;
  return x;
}

__device__ __forceinline__ void word_runs(const uint64_t* __restrict__ lines, uint64_t w, uint64_t nbits,
                                          uint64_t& x, uint64_t& starts, uint64_t& ends) {
  x = level_word(lines, w, nbits);
  const uint64_t prev = w ? level_word(lines, w - 1, nbits) >> 63 : 0;
  const uint64_t next = level_word(lines, w + 1, nbits) & 1;
  starts = x & ~((x << 1) | prev);
  ends = x & ~((x >> 1) | (next << 63));
}

__global__ __launch_bounds__(256) void k_gr_starts(const uint64_t* __restrict__ lines, uint64_t nbits,
                                                   uint64_t nw, uint64_t* __restrict__ last_start,
                                                   unsigned long long* __restrict__ ones) {
  uint64_t cnt = 0;
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256) {
    uint64_t x, st, en;
    word_runs(lines, w, nbits, x, st, en);
    last_start[w] = st ? w * 64 + (63 - __clzll(st)) + 1 : 0;
    cnt += __popcll(x);
  }
  cnt = wave_sum(cnt);
  __shared__ uint64_t red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t t = red[0] + red[1] + red[2] + red[3];
    if (t) atomicAdd(ones, (unsigned long long)t);
  }
}

// visits every run ending in word w as (run length L, absolute end position)
template <typename F>
__device__ __forceinline__ void for_runs_ending(const uint64_t* __restrict__ lines, uint64_t w, uint64_t nbits,
                                                uint64_t carry_start1, F&& f) {
  uint64_t x, st, en;
  word_runs(lines, w, nbits, x, st, en);
  while (en) {
    const int e = __ffsll((unsigned long long)en) - 1;
    en &= en - 1;
    const uint64_t below = e == 63 ? st : st & ((2ull << e) - 1);
    const uint64_t s = below ? w * 64 + (63 - __clzll(below)) : carry_start1 - 1;
    f(w * 64 + e - s + 1);
  }
}

__global__ __launch_bounds__(256) void k_gr_sizes(const uint64_t* __restrict__ lines, uint64_t nbits, uint64_t nw,
                                                  const uint64_t* __restrict__ carry, uint32_t m,
                                                  uint64_t* __restrict__ size) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256) {
    uint64_t bits = 0;
    for_runs_ending(lines, w, nbits, carry[w], [&](uint64_t L) { bits += L / m + 1 + m; });
    size[w] = bits;
  }
}

__device__ __forceinline__ void or_bits(unsigned long long* out, uint64_t pos, uint64_t v, int width) {
  const uint64_t wi = pos >> 6;
  const int sh = (int)(pos & 63);
  atomicOr(out + wi, (unsigned long long)(v << sh));
  if (sh && sh + width > 64) atomicOr(out + wi + 1, (unsigned long long)(v >> (64 - sh)));
}

__global__ __launch_bounds__(256) void k_gr_write(const uint64_t* __restrict__ lines, uint64_t nbits, uint64_t nw,
                                                  const uint64_t* __restrict__ carry, uint32_t m,
                                                  const uint64_t* __restrict__ off,
                                                  unsigned long long* __restrict__ out) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256) {
    uint64_t o = off[w];
    for_runs_ending(lines, w, nbits, carry[w], [&](uint64_t L) {
      const uint64_t q = L / m, r = L % m;
      // field = the terminating one, then r in m digits MSB first, written LSB-first
      const uint64_t field = 1ull | ((__brevll(r) >> (64 - m)) << 1);
      or_bits(out, o + q, field, (int)m + 1);
      o += q + 1 + m;
    });
  }
}

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace

uint32_t golomb_m(uint64_t ones, uint64_t total) {
  if (ones == 0) return 1;
  const double ratio = (double)ones / (double)total;
  const int m = (int)std::log2(1.0 / ratio);
  return m < 1 ? 1u : (uint32_t)m;
}

GolombResult wt_golomb(Index& ix, int depth, uint64_t nbits, uint32_t m_override, bool write) {
  if (!ix.have_wt) throw ApiError{-3, "golomb: wavelet tree not built"};
  if (depth < 0 || depth >= ix.wt_levels) throw ApiError{-4, "golomb: level out of range"};
  if (nbits > ix.n) throw ApiError{-4, "golomb: prefix longer than the level"};
  if (m_override > 63) throw ApiError{-4, "golomb: m must be below 64"};
  hipStream_t s = ix.stream;
  GolombResult res;
  const uint64_t nw = ceil_div(nbits, 64);
  if (!nw) {
    res.m = m_override ? m_override : 1;
    return res;
  }
  const uint64_t* lines = ix.wt_lines[depth].as<uint64_t>();
  ix.gr_tmp[0].ensure((nw + 1) * 8);
  ix.gr_tmp[1].ensure((nw + 1) * 8);
  ix.small.ensure(8192);
  uint64_t* A = ix.gr_tmp[0].as<uint64_t>();
  uint64_t* B = ix.gr_tmp[1].as<uint64_t>();
  unsigned long long* d_ones = ix.small.as<unsigned long long>() + 900;
  HK_HIP(hipMemsetAsync(d_ones, 0, 8, s));
  {
    TimedLaunch t(ix.timer, "golomb_starts", (double)nw * 8 * 3 + nw * 8);
    k_gr_starts<<<grid_for(nw), 256, 0, s>>>(lines, nbits, nw, A, d_ones);
    HK_HIP(hipGetLastError());
  }
  uint64_t ones = 0;
  HK_HIP(hipMemcpyAsync(&ones, d_ones, 8, hipMemcpyDeviceToHost, s));
  scan_exclusive_max_u64(ix.sw, A, B, nw, s);    // B = carry (1 + start of the run entering word w)
  HK_HIP(hipStreamSynchronize(s));
  res.ones = ones;
  res.m = m_override ? m_override : golomb_m(ones, nbits);
  {
    TimedLaunch t(ix.timer, "golomb_sizes", (double)nw * 8 * 5);
    k_gr_sizes<<<grid_for(nw), 256, 0, s>>>(lines, nbits, nw, B, res.m, A);
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_u64(ix.sw, A, A, nw, true, s);   // A[w] = output offset of word w, A[nw] = total
  HK_HIP(hipMemcpyAsync(&res.bits, A + nw, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (write) {
    const uint64_t ow = ceil_div(res.bits, 64) + 1;
    ix.gr_out.ensure(ow * 8);
    HK_HIP(hipMemsetAsync(ix.gr_out.p, 0, ow * 8, s));
    TimedLaunch t(ix.timer, "golomb_write", (double)nw * 8 * 5 + (double)res.bits / 8);
    k_gr_write<<<grid_for(nw), 256, 0, s>>>(lines, nbits, nw, B, res.m, A,
                                              ix.gr_out.as<unsigned long long>());
    HK_HIP(hipGetLastError());
  }
  return res;
}

}  // namespace hk
