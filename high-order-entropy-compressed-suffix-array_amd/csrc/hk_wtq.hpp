// hk_wtq.hpp — device-side wavelet-tree walks shared by the query kernels (hk_wt.hip) and the
// sampled-SA kernels (hk_sample.hip).  Layout and LF identities: see hk_wt.hip's header.
#pragma once

#include "hk_index.hpp"

namespace hk {

__device__ __forceinline__ uint64_t rank1(const uint64_t* __restrict__ lines, uint64_t x) {
  const uint32_t x6 = (uint32_t)(x >> 6);
  const uint64_t li = x6 / 7u;
  const uint32_t off = (uint32_t)(x - li * kLineBits);
  const ulonglong2* L = reinterpret_cast<const ulonglong2*>(lines + li * 8);
  const ulonglong2 a = L[0], b = L[1], c = L[2], d = L[3];
  const uint64_t w[7] = {a.y, b.x, b.y, c.x, c.y, d.x, d.y};
  const uint32_t wi = off >> 6, bi = off & 63u;
  const uint64_t pm = (1ull << bi) - 1ull;
  uint64_t r = a.x;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const uint64_t m = (uint32_t)k < wi ? ~0ull : ((uint32_t)k == wi ? pm : 0ull);
    r += (uint64_t)__popcll(w[k] & m);
  }
  return r;
}

// rank1 and the bit at x from the same 64-B line
__device__ __forceinline__ uint64_t rank1_bit(const uint64_t* __restrict__ lines, uint64_t x, uint32_t& bit) {
  const uint32_t x6 = (uint32_t)(x >> 6);
  const uint64_t li = x6 / 7u;
  const uint32_t off = (uint32_t)(x - li * kLineBits);
  const ulonglong2* L = reinterpret_cast<const ulonglong2*>(lines + li * 8);
  const ulonglong2 a = L[0], b = L[1], c = L[2], d = L[3];
  const uint64_t w[7] = {a.y, b.x, b.y, c.x, c.y, d.x, d.y};
  const uint32_t wi = off >> 6, bi = off & 63u;
  const uint64_t pm = (1ull << bi) - 1ull;
  uint64_t r = a.x;
  uint64_t cur = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k) {
    const uint64_t m = (uint32_t)k < wi ? ~0ull : ((uint32_t)k == wi ? pm : 0ull);
    r += (uint64_t)__popcll(w[k] & m);
    if ((uint32_t)k == wi) cur = w[k];
  }
  bit = (uint32_t)(cur >> bi) & 1u;
  return r;
}

// Per-level / per-code walk tables in LDS for NC codes (256: any alphabet; 16: sigma <= 16, ~1 KiB
// instead of ~38 KiB, so the query kernels keep more waves in flight).
template <int NC>
struct QSharedT {
  uint64_t obn[kMaxLevels][NC];
  uint64_t rbase[kMaxLevels][NC];
  uint8_t bit[kMaxLevels][NC];
  uint8_t depth[NC];
  int16_t code[256];
  const uint64_t* lines[kMaxLevels];
};
using QShared = QSharedT<256>;

template <int NC>
__device__ __forceinline__ void load_qshared(QSharedT<NC>& q, const WtView& v) {
  const int t = threadIdx.x;  // blockDim == 256
  q.code[t] = v.code[t];
  if (t < NC) q.depth[t] = v.depth[t];
  for (int d = 0; d < v.levels; ++d) {
    if (t < v.sigma && t < NC) {
      q.obn[d][t] = v.obn[d * 256 + t];
      q.rbase[d][t] = v.rbase[d * 256 + t];
    }
    if (t < NC) q.bit[d][t] = v.bit[d * 256 + t];
  }
  if (t < kMaxLevels) q.lines[t] = v.lines[t];
  __syncthreads();
}

// LF step of the pair (xl, xr) for code c: returns the leaf positions
template <class Q>
__device__ __forceinline__ void lf_pair(const Q& q, int c, uint64_t& xl, uint64_t& xr) {
  const int dep = q.depth[c];
  for (int d = 0; d < dep; ++d) {
    const uint64_t* L = q.lines[d];
    const uint64_t rl = rank1(L, xl);
    const uint64_t rr = rank1(L, xr);
    if (q.bit[d][c]) {
      const uint64_t rb = q.rbase[d][c];
      xl = rb + rl;
      xr = rb + rr;
    } else {
      const uint64_t o = q.obn[d][c];
      xl = xl - rl + o;
      xr = xr - rr + o;
    }
  }
}

// LF of row x without knowing its symbol: walk down following the bits (the node's first code
// lo stands for every code of the node in the per-code tables).  Returns the leaf position
// C[c] + occ(c, x) and the dense code c = BWT[x].
template <class Q>
__device__ __forceinline__ uint64_t lf_access(const Q& q, int sigma, uint64_t x, int& code) {
  int lo = 0, hi = sigma;
  for (int d = 0; hi - lo > 1; ++d) {
    const int mid = lo + (hi - lo) / 2;
    uint32_t b;
    const uint64_t r = rank1_bit(q.lines[d], x, b);
    if (b) {
      x = q.rbase[d][mid] + r;
      lo = mid;
    } else {
      x = x - r + q.obn[d][lo];
      hi = mid;
    }
  }
  code = lo;
  return x;
}

}  // namespace hk
