// hk_bucket.hip — single-GPU suffix array + BWT by bucket sort (the default build).
//
// Replaces build_suffix_array (csa/suffix_array.py:131-134) + bwt_transform (csa/bwt.py:3-13) for
// one GPU.  Result identical to the reference's SA (Python str order, '$' an ordinary byte,
// proper prefix first) and BWT (wrap at SA == 0).
//
// Pipeline (HBM bytes per suffix in brackets, 1 GiB sigma=4 figures):
//   1. k_bucket_hist   [1]   histogram of the top D bits of every suffix key, from the text;
//   2. k_pack_keyed    [1+8] u64 key per suffix = [q symbols, radix Rk][code of T'[p-1]];
//   3. two LSD onesweep passes over the top D key bits (hk_sort.hip) [20 + 24]: the suffixes are
//      then grouped by bucket, buckets in order, each bucket a contiguous range;
//   4. k_bucket_sort   [12+5] one workgroup per bucket (<= 18432 suffixes): keys to registers,
//      LDS radix sort over the bits that vary inside the bucket, SA and BWT written in sorted order,
//      suffixes with equal keys appended to a tie list;
//   5. buckets too large for one workgroup (skewed texts) are sorted together on the global
//      path (radix sort of (bucket ordinal, low key bits)); a text whose suffixes mostly fall in
//      such buckets takes the global path whole;
//   6. ties are refined from symbol q on (hk_sa.hip refine_loop), falling back to prefix
//      doubling for long repeats.
// Keyed layout: the sorted field has no end-of-text code and no code for a terminal that occurs
// once at n-1 (see KeyGeom) — sigma=4 DNA + '$' packs 2 bits per symbol, so 24 symbols fit the
// 48 bits that two 8-bit passes + a 32-bit LDS sort cover.

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "hk_bucket.hpp"
#include "hk_index.hpp"
#include "hk_keys.hpp"

namespace hk {
namespace {

// ------------------------------------------------------------ 1. bucket histogram
// One pass over the text, all 2^D <= 65536 bins in LDS as u16 pairs (128 KiB).  A counter that
// reaches 0x8000 is drained to the global histogram by the lane whose add took it there (the lane
// sees 0x7FFF returned); the 32k headroom above covers the adds in flight until its subtract lands.
constexpr int BH_T = 1024;
constexpr int BH_PER = 16;                  // consecutive positions per thread (radix-2^k path)
constexpr int BH_TILE = BH_T * BH_PER;      // 16384 positions per iteration = 2 radix tiles
constexpr int BH_STAGE = 4096;              // staged positions per iteration of the generic path
constexpr uint32_t CP_NAM = 512;           // cursor partition: pass A digit rows (<= 9-bit digits)

__device__ __forceinline__ void bh_add(uint32_t* H, uint32_t b, unsigned long long* __restrict__ hist) {
  const uint32_t sh = 16u * (b & 1u);
  const uint32_t old = atomicAdd(&H[b >> 1], 1u << sh);
  if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
    atomicSub(&H[b >> 1], 0x8000u << sh);
    atomicAdd(&hist[b], 0x8000ull);
  }
}

// Workgroup w covers the positions [w*stride, w*stride + span) (span and stride multiples of BH_TILE;
// stride = 0: span, the whole text; a larger stride samples spans spread over the text).
// DIG (HQ only): only the low 8 bits of the bucket — the first LSD pass's digit — into per-wave
// 256-bin LDS histograms (the bucket counts come from the sorted keys afterwards, k_bin_starts).
template <bool HQ, bool DIG = false>
__global__ __launch_bounds__(BH_T, 1) void k_bucket_hist(const uint8_t* __restrict__ t, uint64_t n,
                                                         const uint16_t* __restrict__ lutk,
                                                         const uint64_t* __restrict__ skey, KeyedArgs g, int bsh,
                                                         int D, unsigned long long* __restrict__ hist,
                                                         uint64_t span, uint64_t stride = 0) {
  __shared__ uint32_t H[DIG ? 1 : 32768];
  __shared__ uint32_t HD[DIG ? BH_T / 64 : 1][256];
  __shared__ uint16_t c[HQ ? 1 : BH_STAGE + kCodePad];
  __shared__ uint16_t L[256];
  __shared__ uint64_t SK[72];
  const uint32_t tid = threadIdx.x;
  uint32_t* const hd = &HD[DIG ? tid >> 6 : 0][0];
  auto add = [&](uint32_t b) {
    if (DIG) atomicAdd(&hd[b & 255u], 1u);
    else bh_add(H, b, hist);
  };
  if (DIG) for (uint32_t i = tid; i < (BH_T / 64) * 256; i += BH_T) (&HD[0][0])[i] = 0;
  else for (uint32_t i = tid; i < 32768; i += BH_T) H[i] = 0;
  if (tid < 256) L[tid] = lutk[tid];
  if (tid < 72) SK[tid] = skey[tid];
  __syncthreads();
  const uint64_t lim = n < g.s_start ? n : g.s_start;   // positions with a text window
  const uint64_t lo = (uint64_t)blockIdx.x * (stride ? stride : span);
  const uint64_t hi = lo + span < n ? lo + span : n;
  if (HQ) {
    const int lb = 31 - __clz((uint32_t)g.Rk);
    const uint32_t bmask = (1u << D) - 1;
    uint64_t base = lo;
    uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0;
    if (base + (uint64_t)tid * BH_PER < hi) {
      const uint4* src = reinterpret_cast<const uint4*>(t + base + (uint64_t)tid * BH_PER);
      w0 = src[0];
      w1 = src[1];
    }
    for (; base < hi; base += BH_TILE) {
      const uint64_t p0 = base + (uint64_t)tid * BH_PER;
      const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
      if (p0 + BH_TILE < hi) {   // next iteration's bytes in flight
        const uint4* src = reinterpret_cast<const uint4*>(t + p0 + BH_TILE);
        w0 = src[0];
        w1 = src[1];
      }
      const uint64_t lim2 = lim < hi ? lim : hi;
      if (p0 < lim2) {
        // rolling window over bytes i = 0 .. 30 (static register indices); the window ending at
        // byte i is the bucket of position p0 + i - (hq - 1)
        uint32_t b = 0;
#pragma unroll
        for (int i = 0; i < 2 * BH_PER - 1; ++i) {
          b = ((b << lb) | (L[(wd[i >> 2] >> (8 * (i & 3))) & 255u] & 255u)) & bmask;
          const int j = i - (g.hq - 1);
          if (j >= 0 && j < BH_PER && p0 + j < lim2) add(b);
        }
      }
      for (uint64_t p = p0 > lim ? p0 : lim; p < p0 + BH_PER && p < hi; ++p)
        add((uint32_t)(SK[p - g.s_start] >> bsh));
    }
  } else {
    for (uint64_t base = lo; base < hi; base += BH_STAGE) {
      stage_text_codes<BH_STAGE, BH_T>(c, L, t, n, base);
      __syncthreads();
#pragma unroll
      for (int k = 0; k < BH_STAGE / BH_T; ++k) {
        const int off = k * BH_T + tid;
        const uint64_t p = base + off;
        if (p < hi) bh_add(H, (uint32_t)(keyed_sym(c, off, p, g, SK) >> bsh), hist);
      }
      __syncthreads();
    }
  }
  __syncthreads();
  if (DIG) {
    if (tid < 256) {
      uint64_t v = 0;
#pragma unroll
      for (int w = 0; w < BH_T / 64; ++w) v += HD[w][tid];
      if (v) atomicAdd(&hist[tid], (unsigned long long)v);
    }
    return;
  }
  const uint32_t nb = 1u << D;
  for (uint32_t i = tid; i < 32768; i += BH_T) {
    const uint32_t v = H[i];
    if ((v & 0xFFFFu) && 2 * i < nb) atomicAdd(&hist[2 * i], (unsigned long long)(v & 0xFFFFu));
    if ((v >> 16) && 2 * i + 1 < nb) atomicAdd(&hist[2 * i + 1], (unsigned long long)(v >> 16));
  }
}

// (PkGeom, the packed records' geometry: hk_bucket.hpp)

// a record's key bits below the pass A digit in the full (pb-bit prev) layout
__device__ __forceinline__ uint64_t pk_full_low(uint64_t rec, const PkGeom& g) {
  const uint64_t kr = rec >> g.pbits;
  const uint64_t pos = rec & ((1ull << g.pbits) - 1);
  uint32_t pf = (uint32_t)kr & ((1u << g.pb2) - 1);
  if (g.tcode >= 0) pf = pos == 0 ? (uint32_t)g.tcode : pf + (pf >= (uint32_t)g.tcode ? 1u : 0u);
  return ((kr >> g.pb2) << g.pb) | pf;
}

// ------------------------------------------------------------ 1b. cursor partition
// The bucket grouping needs no stable passes: the LDS bucket sort orders every bucket completely
// and equal keys are refined, so the order inside a bucket is free.  Two scatter passes whose
// destinations are reserved from global cursors therefore replace the two stable onesweep passes:
// no decoupled lookback (2.2 ms of a 7.3 ms 1 GiB pass, tools/radix_diag.py: 512x16 tiles with and
// without it) and one LDS atomic per suffix for its rank instead of the match-mask ranking.
//   pre-pass  k_bucket_hist_spans: the 2^D bucket counts of every workgroup span (u32 partials,
//             reduced by k_bucket_reduce) and the span's counts of pass A's digit (bucket >> sA);
//   pass A    k_cpart<true>: keys from the text, scattered by the bucket's top digit; cursors per
//             (span, digit), started at the digit's start plus the earlier spans' counts;
//   pass B    k_cpart<false> (D > 8): tiles inside one top-digit region, scattered by the bucket's
//             low 8 bits; cursors per bucket, started at the bucket starts.
// Each tile reserves its digit runs with one global atomic per digit (issued before its keys are
// staged; the result is first needed for the write-out).
// end of a span pre-pass: the span's bucket counts as plain u32 stores (reduced by k_bucket_reduce)
// and its counts of pass A's digit (bucket >> sA, incl. the drained parts already in M).  CB = bits
// per LDS counter (16: two per word, 2^D <= 65536; 8: four per word, 2^D <= 131072).  The LDS
// counters hold buckets [boff, boff + nbl) of the 2^D (boff > 0: the second half of an exact
// two-run count, whose digit counts add to the first run's).
template <int CB>
__device__ __forceinline__ void hist_spans_flush(const uint32_t* H, uint32_t* M, uint32_t nbl, uint32_t boff,
                                                 uint32_t stride, int sA, uint32_t* __restrict__ part,
                                                 uint32_t* __restrict__ spanc, uint32_t* fsum = nullptr) {
  constexpr int CPW = 32 / CB;
  constexpr uint32_t CM = (1u << CB) - 1;
  const uint32_t tid = threadIdx.x;
  const uint32_t np = (nbl + CPW - 1) / CPW;
  uint32_t* const pw = part + (uint64_t)blockIdx.x * stride + boff;
  for (uint32_t i = tid; i < np; i += BH_T) {
    const uint32_t v = H[i];
    if (CPW == 2) reinterpret_cast<uint2*>(pw)[i] = make_uint2(v & CM, v >> 16);
    else reinterpret_cast<uint4*>(pw)[i] = make_uint4(v & CM, (v >> 8) & CM, (v >> 16) & CM, v >> 24);
  }
  // pass A digit counts: contiguous words per thread, one LDS add per digit run
  const uint32_t per = (np + BH_T - 1) / BH_T;
  uint32_t acc = 0, cd = 0, fs = 0;
  for (uint32_t i = tid * per; i < np && i < tid * per + per; ++i) {
    const uint32_t v = H[i];
#pragma unroll
    for (int h = 0; h < CPW; ++h) {
      const uint32_t d = (boff + CPW * i + h) >> sA;
      if (d != cd) {
        if (acc) atomicAdd(&M[cd], acc);
        fs += acc;
        acc = 0;
        cd = d;
      }
      acc += (v >> (CB * h)) & CM;
    }
  }
  if (acc) atomicAdd(&M[cd], acc);
  if (fsum && fs + acc) atomicAdd(fsum, fs + acc);
  __syncthreads();
  if (tid < CP_NAM) {
    uint32_t* const sc = spanc + (uint64_t)blockIdx.x * CP_NAM + tid;
    *sc = (boff ? *sc : 0u) + M[tid];
  }
}

// CB = 8 (2^17 buckets): a byte drained at 128 can still pass 255 when ~128+ increments to one
// bucket land before the drain (every thread inside one long run of a symbol); any increment that
// sees a byte at >= 224 raises *ovf, pass A then skips itself and the host recounts exactly with two
// CB = 16 runs over the bucket halves (HB = 0, 1: only buckets with b >> 16 == HB; HB = -1: all).
// LBQ/HQ > 0: the code width and window length fixed at compile time (= log2 g.Rk and g.hq; DNA
// 2/9, bytes 8/3): only the BH_PER + HQ - 1 codes a thread's windows use are mapped, no per-code
// window tests.
template <int CB, int HB = -1, int LBQ = 0, int HQ = 0>
__global__ __launch_bounds__(BH_T, 1) void k_bucket_hist_spans(const uint8_t* __restrict__ t, uint64_t n,
                                                               const uint16_t* __restrict__ lutk,
                                                               const uint64_t* __restrict__ skey, KeyedArgs g,
                                                               int bsh, int D, int sA, uint32_t* __restrict__ part,
                                                               unsigned long long* __restrict__ drain,
                                                               uint32_t* __restrict__ spanc, uint64_t span,
                                                               unsigned long long* __restrict__ ovf) {
  constexpr int hb = HB;
  // CB-bit counters packed in 32768 words (drained at half range, as k_bucket_hist)
  constexpr int CPW = 32 / CB;
  constexpr uint32_t HALF = 1u << (CB - 1);
  const uint32_t boff = hb > 0 ? 65536u : 0u;
  bool bad = false;
  __shared__ uint32_t H[32768];
  __shared__ uint32_t M[CP_NAM];  // pass A digit counts of this span
  __shared__ uint16_t L[256];
  __shared__ uint64_t SK[72];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 32768; i += BH_T) H[i] = 0;
  if (tid < CP_NAM) M[tid] = 0;
  if (tid < 256) L[tid] = lutk[tid];
  if (tid < 72) SK[tid] = skey[tid];
  __syncthreads();
  auto add = [&](uint32_t b) {
    if (hb >= 0 && (b >> 16) != (uint32_t)hb) return;
    const uint32_t bl = b - boff;
    const uint32_t sh = CB * (bl % CPW);
    const uint32_t old = atomicAdd(&H[bl / CPW], 1u << sh);
    const uint32_t ob = (old >> sh) & ((1u << CB) - 1);
    if (CB == 8) bad |= ob >= 224u;
    if (ob == HALF - 1) {
      atomicSub(&H[bl / CPW], HALF << sh);
      atomicAdd(&drain[b], (unsigned long long)HALF);
      atomicAdd(&M[b >> sA], HALF);
    }
  };
  const uint64_t lim = n < g.s_start ? n : g.s_start;   // positions with a text window
  const uint64_t lo = (uint64_t)blockIdx.x * span;
  const uint64_t hi = lo + span < n ? lo + span : n;
  const int lb = LBQ ? LBQ : 31 - __clz((uint32_t)g.Rk);
  const int hq = HQ ? HQ : g.hq;
  constexpr int NI = HQ ? BH_PER + HQ - 1 : 2 * BH_PER - 1;
  static_assert(NI <= 2 * BH_PER, "window past the thread's 32 bytes");
  // the window of hq symbols (hq * lb <= 32 bits); the bucket is its top D bits
  const int wbits = hq * lb, wdrop = wbits - D;
  const uint32_t bmask = wbits >= 32 ? ~0u : (1u << wbits) - 1;
  uint4 w0 = make_uint4(0, 0, 0, 0), w1 = w0;
  if (lo + (uint64_t)tid * BH_PER < hi) {
    const uint4* src = reinterpret_cast<const uint4*>(t + lo + (uint64_t)tid * BH_PER);
    w0 = src[0];
    w1 = src[1];
  }
  for (uint64_t base = lo; base < hi; base += BH_TILE) {
    const uint64_t p0 = base + (uint64_t)tid * BH_PER;
    const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    if (p0 + BH_TILE < hi) {   // next iteration's bytes in flight
      const uint4* src = reinterpret_cast<const uint4*>(t + p0 + BH_TILE);
      w0 = src[0];
      w1 = src[1];
    }
    const uint64_t lim2 = lim < hi ? lim : hi;
    if (p0 < lim2) {
      const bool full = p0 + BH_PER <= lim2;
      uint32_t b = 0;
#pragma unroll
      for (int i = 0; i < NI; ++i) {
        b = ((b << lb) | (L[(wd[i >> 2] >> (8 * (i & 3))) & 255u] & 255u)) & bmask;
        const int j = i - (hq - 1);
        if (j >= 0 && j < BH_PER && (full || p0 + j < lim2)) add(b >> wdrop);
      }
    }
    for (uint64_t p = p0 > lim ? p0 : lim; p < p0 + BH_PER && p < hi; ++p) add((uint32_t)(SK[p - g.s_start] >> bsh));
  }
  if (CB == 8 && bad) atomicOr(ovf, 1ull);
  __syncthreads();
  const uint32_t nbl = hb >= 0 ? 65536u : 1u << D;
  hist_spans_flush<CB>(H, M, nbl, boff, 1u << D, sA, part, spanc);
}

// the pre-pass over the packed keys of a sharded slice: bin = ((key - kbias) >> shift) & (2^D - 1)
__global__ __launch_bounds__(BH_T, 1) void k_key_hist_spans(const uint64_t* __restrict__ keys, uint64_t m, int shift,
                                                            uint64_t kbias, int D, int sA, uint32_t* __restrict__ part,
                                                            unsigned long long* __restrict__ drain,
                                                            uint32_t* __restrict__ spanc, uint64_t span) {
  __shared__ uint32_t H[32768];
  __shared__ uint32_t M[CP_NAM];
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 32768; i += BH_T) H[i] = 0;
  if (tid < CP_NAM) M[tid] = 0;
  __syncthreads();
  const uint32_t bmask = (1u << D) - 1;
  auto add = [&](uint64_t k) {
    const uint32_t b = (uint32_t)((k - kbias) >> shift) & bmask;
    const uint32_t sh = 16u * (b & 1u);
    const uint32_t old = atomicAdd(&H[b >> 1], 1u << sh);
    if (((old >> sh) & 0xFFFFu) == 0x7FFFu) {
      atomicSub(&H[b >> 1], 0x8000u << sh);
      atomicAdd(&drain[b], 0x8000ull);
      atomicAdd(&M[b >> sA], 0x8000u);
    }
  };
  const uint64_t lo = (uint64_t)blockIdx.x * span;
  const uint64_t hi = lo + span < m ? lo + span : m;
  for (uint64_t base = lo; base < hi; base += (uint64_t)BH_T * 8) {   // four 16-B loads in flight
    ulonglong2 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t p = base + ((uint64_t)u * BH_T + tid) * 2;
      v[u] = p + 1 < hi ? *reinterpret_cast<const ulonglong2*>(keys + p)
                        : make_ulonglong2(p < hi ? keys[p] : 0ull, 0ull);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t p = base + ((uint64_t)u * BH_T + tid) * 2;
      if (p < hi) add(v[u].x);
      if (p + 1 < hi) add(v[u].y);
    }
  }
  __syncthreads();
  hist_spans_flush<16>(H, M, 1u << D, 0, 1u << D, sA, part, spanc);
}

// hist[b] = drained counts + the spans' partial counts of bucket b
__global__ __launch_bounds__(256) void k_bucket_reduce(const uint32_t* __restrict__ part,
                                                       const unsigned long long* __restrict__ drain, uint32_t nspan,
                                                       uint32_t stride, uint32_t nb, uint64_t* __restrict__ hist,
                                                       const unsigned long long* __restrict__ only_if = nullptr) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b >= nb || (only_if && !*only_if)) return;
  uint64_t s = drain[b];
#pragma unroll 8
  for (uint32_t w = 0; w < nspan; ++w) s += part[(uint64_t)w * stride + b];
  hist[b] = s;
}

// hist[b] (zeroed) += drain[b] + the spans' partial counts of bucket b: four buckets per thread (16-B
// loads) and the spans split over gridDim.y groups (u64 atomics), so that ~16 MiB of loads are in
// flight (one thread per bucket over every span kept ~4 MiB in flight: 73 us at 1 GiB).  nb % 4 == 0.
__global__ __launch_bounds__(256) void k_bucket_reduce4(const uint32_t* __restrict__ part,
                                                        const unsigned long long* __restrict__ drain, uint32_t nspan,
                                                        uint32_t stride, uint32_t nb,
                                                        unsigned long long* __restrict__ hist) {
  const uint32_t b = (blockIdx.x * 256 + threadIdx.x) * 4;
  if (b >= nb) return;
  const uint32_t per = (nspan + gridDim.y - 1) / gridDim.y, w0 = blockIdx.y * per;
  const uint32_t w1 = w0 + per < nspan ? w0 + per : nspan;
  unsigned long long s0 = 0, s1 = 0, s2 = 0, s3 = 0;
  if (blockIdx.y == 0) {
    const ulonglong2 d0 = *reinterpret_cast<const ulonglong2*>(drain + b);
    const ulonglong2 d1 = *reinterpret_cast<const ulonglong2*>(drain + b + 2);
    s0 = d0.x, s1 = d0.y, s2 = d1.x, s3 = d1.y;
  }
#pragma unroll 8
  for (uint32_t w = w0; w < w1; ++w) {
    const uint4 v = *reinterpret_cast<const uint4*>(part + (uint64_t)w * stride + b);
    s0 += v.x, s1 += v.y, s2 += v.z, s3 += v.w;
  }
  if (s0) atomicAdd(&hist[b], s0);
  if (s1) atomicAdd(&hist[b + 1], s1);
  if (s2) atomicAdd(&hist[b + 2], s2);
  if (s3) atomicAdd(&hist[b + 3], s3);
}

// Cursors of both passes from the counts, in two small kernels over blocks of 64 digits x 16
// span groups (one workgroup scanning every span of every digit took 0.25-0.5 ms of serial loads):
// k_cp_colsum: per digit, the span groups' partial sums (exclusive over groups) and the digit total;
// k_cp_cursors: every block scans the digit totals (digit starts; block 0 publishes them as the
// region bounds of pass B), then each (digit, group) thread walks its spans: pass A's cursor of
// (span, digit) = the digit's start + the earlier spans' counts.  Pass B's cursors (the bucket starts)
// come per digit: each wave scans the 2^sA buckets of four of the block's digits from the digit's start
// (coalesced 32-B loads; one extra workgroup scanning all 2^17 buckets with strided loads took 99 us).
constexpr uint32_t CP_DB = 64, CP_NG = 16;   // digits per block, span groups

// hist = drain + the spans' partial counts (hist zeroed by the caller when nb % 4 == 0)
static void bucket_reduce(const uint32_t* part, const unsigned long long* drain, uint32_t nspan, uint32_t stride,
                          uint32_t nb, uint64_t* hist, hipStream_t s) {
  if (nb % 4 == 0 && stride % 4 == 0) {
    k_bucket_reduce4<<<dim3((nb / 4 + 255) / 256, nspan >= 64 ? 8 : 1), 256, 0, s>>>(
        part, drain, nspan, stride, nb, reinterpret_cast<unsigned long long*>(hist));
  } else {
    k_bucket_reduce<<<(nb + 255) / 256, 256, 0, s>>>(part, drain, nspan, stride, nb, hist);
  }
  HK_HIP(hipGetLastError());
}

__global__ __launch_bounds__(1024) void k_cp_colsum(const uint32_t* __restrict__ spanc, uint32_t nspan, uint32_t ndA,
                                                    uint64_t* __restrict__ gpre, uint64_t* __restrict__ totA) {
  __shared__ uint64_t ps[CP_NG][CP_DB];
  const uint32_t tid = threadIdx.x, dl = tid % CP_DB, g = tid / CP_DB, d = blockIdx.x * CP_DB + dl;
  const uint32_t per = (nspan + CP_NG - 1) / CP_NG, w0 = g * per < nspan ? g * per : nspan;
  const uint32_t w1 = w0 + per < nspan ? w0 + per : nspan;
  uint64_t part = 0;
  if (d < ndA) {
#pragma unroll 8
    for (uint32_t w = w0; w < w1; ++w) part += spanc[(uint64_t)w * CP_NAM + d];
  }
  ps[g][dl] = part;
  __syncthreads();
  if (g == 0 && d < ndA) {
    uint64_t run = 0;
    for (uint32_t q = 0; q < CP_NG; ++q) {
      gpre[(uint64_t)q * CP_NAM + d] = run;
      run += ps[q][dl];
    }
    totA[d] = run;
  }
}

__global__ __launch_bounds__(1024) void k_cp_cursors(const uint64_t* __restrict__ hist, const uint32_t* __restrict__ spanc,
                                                     const uint64_t* __restrict__ gpre, uint32_t nspan, uint32_t nb,
                                                     uint32_t ndA, unsigned long long* __restrict__ curA,
                                                     unsigned long long* __restrict__ curB,
                                                     const uint64_t* __restrict__ totA, uint64_t* __restrict__ startA) {
  __shared__ uint64_t ws[16];
  __shared__ uint64_t st[CP_NAM];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // digit starts (every block; ndA <= CP_NAM, one value per thread of the first CP_NAM)
  const uint64_t tot = tid < ndA ? totA[tid] : 0;
  const uint64_t inc = wave_incl_sum<uint64_t>(tot);
  if (lane == 63 && wv < CP_NAM / 64) ws[wv] = inc;
  __syncthreads();
  if (tid < CP_NAM) {
    uint64_t run = inc - tot;
    for (uint32_t w = 0; w < wv; ++w) run += ws[w];
    st[tid] = run;
    if (blockIdx.x == 0 && tid < ndA) {
      startA[tid] = run;
      if (tid == ndA - 1) startA[ndA] = run + tot;
    }
  }
  __syncthreads();
  if (curB) {   // pass B: bucket starts, four digits per wave (wave-uniform loops: full-wave scans)
    const uint32_t nbk = nb / ndA;   // buckets per digit (2^sA)
    for (uint32_t j = 0; j < CP_DB / 16; ++j) {
      const uint32_t dd = blockIdx.x * CP_DB + wv * (CP_DB / 16) + j;
      if (dd >= ndA) break;
      uint64_t run = st[dd];
      for (uint32_t c = 0; c < nbk; c += 256) {
        const uint32_t i0 = c + 4 * lane;
        const uint64_t b0 = (uint64_t)dd * nbk + i0;
        uint64_t h[4], sum = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          h[i] = i0 + i < nbk ? hist[b0 + i] : 0;
          sum += h[i];
        }
        const uint64_t inc = wave_incl_sum<uint64_t>(sum);
        uint64_t e = run + inc - sum;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (i0 + i < nbk) {
            curB[b0 + i] = e;
            e += h[i];
          }
        run += ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(inc >> 32), 63) << 32) |
               (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)inc, 63);
      }
    }
  }
  const uint32_t dl = tid % CP_DB, g = tid / CP_DB, d = blockIdx.x * CP_DB + dl;
  if (d >= ndA) return;
  const uint32_t per = (nspan + CP_NG - 1) / CP_NG, w0 = g * per < nspan ? g * per : nspan;
  const uint32_t w1 = w0 + per < nspan ? w0 + per : nspan;
  uint64_t run = st[d] + gpre[(uint64_t)g * CP_NAM + d];
#pragma unroll 8
  for (uint32_t w = w0; w < w1; ++w) {
    curA[(uint64_t)w * CP_NAM + d] = run;
    run += spanc[(uint64_t)w * CP_NAM + d];
  }
}

constexpr int CP_T = 512;
constexpr int CP_I = 16;
constexpr int CP_TILE = CP_T * CP_I;   // 8192 suffixes per tile

template <int NB, int T = CP_T, bool SD = false, bool HS = false>
struct CpShared {
  union {
    uint64_t keys[HS ? T * CP_I / 2 : T * CP_I];   // HS: the tile's records staged in two halves
    uint32_t vals[T * CP_I];
    uint16_t codes[T * CP_I + kCodePad];   // pass A: the tile's text codes ...
    struct {                               // ... or packed codes and raw bytes (radix 2^lb)
      uint32_t pk[(T * CP_I + 64) / 4 + 4];
      uint8_t raw[T * CP_I + 64];
    } ft;
  } stage;
  uint8_t sd[SD ? (HS ? T * CP_I / 2 : T * CP_I) : 4];   // packed pass A: low 8 bits of each staged slot's digit
  // destination of the digit's run minus its tile start (packed pass A: u32, single GPU n < 2^32,
  // so that 512-thread tiles fit two workgroups per CU)
  std::conditional_t<SD, uint32_t, uint64_t> gb[NB];
  uint32_t cnt[NB];    // digit counts (ranks by LDS atomics)
  uint32_t tst[NB];    // tile-local exclusive digit starts
  uint32_t wsum[NB / 64];
  uint32_t prev0;
  uint16_t L[256], LP[256];
  uint64_t SK[72];
};

// One tile: ranks by LDS atomics (any order inside a digit), one cursor reservation per digit,
// keys then values staged in digit order and written as runs.  FT: the tile is text positions
// [blockIdx.x * CP_TILE, ...) and builds its keys (values = positions), cursor row = its span's;
// else a tile of one region (from the XCD-group region table) and the row is the region's.
// MODE 0: pass A over the text (builds the keys); 1: pass A over packed keys (a sharded slice's);
// 2: pass B over one region per tile.  digit = ((key - kbias) >> shift) & (NB - 1).
// PK (packed records, single GPU): one u64 per suffix, (key bits below pass A's digit) << pbits |
// position, instead of a key and a value plane.  Pass A (NB = 512) packs after ranking and stages
// each slot's digit (low 8 bits in sd, the 9th from the slot's side of digit 256's start); pass B
// (NB = 256, shift counts the position bits) moves the records unchanged.
// HS (packed records): the tile's records are staged and written in two halves (32 KiB of staging), so
// three workgroups fit a CU instead of two (pass B: 3.52 -> 3.42-3.47 ms at 1 GiB; pass A, whose keys
// then have to be rebuilt or spill, gained nothing and keeps full staging)
template <int MODE, int LB, int NB = 256, int T = CP_T, bool PK = false, bool CS = true, bool HS = false>
__global__ __launch_bounds__(T, T == 1024 ? 1 : (HS ? 3 * T / 256 : 2)) void k_cpart(const uint64_t* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                   uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                   uint64_t n, int shift, uint64_t kbias,
                                                   unsigned long long* __restrict__ cur,
                                                   const uint32_t* __restrict__ gtab,
                                                   const uint64_t* __restrict__ startA, uint64_t span,
                                                   TextKeySrc src, int pbits = 0,
                                                   const unsigned long long* __restrict__ skip = nullptr) {
  constexpr int WSPAN = CP_I * 64;
  constexpr bool FT = MODE == 0;
  constexpr bool SD = PK && MODE == 0;
  static_assert(NB == 256 || NB == 512, "digits per pass");
  static_assert(!PK || MODE == 2 || (MODE == 0 && NB == 512), "packed records: pass A over 9-bit digits");
  static_assert(!HS || PK, "half staging: packed records only");
  constexpr uint32_t DM = NB - 1;
  constexpr int TILE = T * CP_I;
  __shared__ CpShared<NB, T, SD, HS> sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (MODE == 0 && skip && *skip) return;   // the pre-pass counts overflowed: recounted, then relaunched
  uint64_t tbase;
  uint32_t tn;
  unsigned long long* row;
  if (MODE <= 1) {
    // workgroups b, b + 8, ... (one XCD when blocks are dealt round-robin, which only speed relies
    // on) take the spans g, g + 8, ... in order: the runs a cursor row hands out back to back are
    // written from one L2, which merges them into whole lines
    const uint32_t per = (uint32_t)(span / TILE), g = blockIdx.x & 7u, k = blockIdx.x >> 3;
    const uint64_t tile = (uint64_t)(g + 8u * (k / per)) * per + k % per;
    tbase = tile * TILE;
    if (tbase >= n) return;   // past the last span (whole workgroup, before any barrier)
    tn = (uint32_t)(n - tbase < (uint64_t)TILE ? n - tbase : TILE);
    row = cur + (tbase / span) * CP_NAM;
  } else {
    // region table: gtab[g] = first entry of XCD group g (gtab[8] = end), entries {region, first
    // tile}; workgroup b is tile b >> 3 of group b & 7 (see cursor_partition)
    uint32_t* const T2 = reinterpret_cast<uint32_t*>(&sh.stage);   // the table (<= 9 + 2 * CP_NAM words)
    for (uint32_t i = tid; i < 9 + 2 * CP_NAM; i += T) T2[i] = gtab[i];
    __syncthreads();
    if (tid == 0) {
      const uint32_t g = blockIdx.x & 7u, k = blockIdx.x >> 3;
      uint32_t lo = T2[g], hi = T2[g + 1];   // last entry with first tile <= k
      uint32_t d = ~0u, k0 = 0;
      if (lo < hi && T2[9 + 2 * lo + 1] <= k) {
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) / 2;
          if (T2[9 + 2 * mid + 1] <= k) lo = mid; else hi = mid;
        }
        d = T2[9 + 2 * lo];
        k0 = T2[9 + 2 * lo + 1];
      }
      uint64_t tb = 0, tl = 0;
      if (d != ~0u) {
        tb = startA[d] + (uint64_t)(k - k0) * TILE;
        tl = tb < startA[d + 1] ? startA[d + 1] - tb : 0;
      }
      sh.gb[0] = tb;
      sh.gb[1] = tl < (uint64_t)TILE ? tl : (uint64_t)TILE;
      sh.gb[2] = d;
    }
    __syncthreads();
    tbase = sh.gb[0];
    tn = (uint32_t)sh.gb[1];
    if (tn == 0) return;   // past the end of a shorter group (whole workgroup)
    row = cur + sh.gb[2] * NB;
    __syncthreads();   // gb is reused below
  }
  if (tid < NB) sh.cnt[tid] = 0;
  const uint32_t s0 = wv * WSPAN + lane;   // item k of this thread is tile slot s0 + 64 k ...
  // ... or, packed pass A over radix-2^2 codes, slot 16 tid + k
  constexpr bool CONSEC = CS && MODE == 0 && PK && LB == 2 && CP_I == 16;
  const uint32_t c0 = CONSEC ? 16u * tid : s0, cst = CONSEC ? 1u : 64u;
  uint64_t key[CP_I];
  uint32_t val[CP_I];
  if (FT) {
    if (tid < 256) {
      sh.L[tid] = src.lutk[tid];
      sh.LP[tid] = src.lutp[tid];
    }
    if (tid < 72) sh.SK[tid] = src.skey[tid];
    __syncthreads();
    if constexpr (CONSEC)
      text_keys_consec2<T>(key, src, n, tbase, sh.stage.ft.pk, &sh.prev0, sh.L, sh.LP, sh.SK);
    else
      text_keys<T, CP_I, LB>(key, src, n, tbase, tbase + (uint64_t)wv * WSPAN, lane, sh.stage.codes,
                             sh.stage.ft.pk, sh.stage.ft.raw, &sh.prev0, sh.L, sh.LP, sh.SK);
#pragma unroll
    for (int k = 0; k < CP_I; ++k) val[k] = (uint32_t)(tbase + c0 + cst * k);
  } else {
#pragma unroll
    for (int k = 0; k < CP_I; ++k) key[k] = s0 + 64u * k < tn ? kin[tbase + s0 + 64u * k] : ~0ull;
    if (!PK) {
#pragma unroll
      for (int k = 0; k < CP_I; ++k) val[k] = s0 + 64u * k < tn ? vin[tbase + s0 + 64u * k] : 0u;
    }
  }
  __syncthreads();   // counters zeroed; the text staging is read
  uint32_t rk[CP_I];
#pragma unroll
  for (int k = 0; k < CP_I; ++k) {
    const uint32_t d = (uint32_t)((key[k] - kbias) >> shift) & DM;
    const uint32_t r = c0 + cst * k < tn ? atomicAdd(&sh.cnt[d], 1u) : 0u;
    rk[k] = r | (d << 16);
  }
  if (SD) {   // the record: key bits below the digit, then the position
    const uint64_t klmask = (1ull << shift) - 1;
#pragma unroll
    for (int k = 0; k < CP_I; ++k) key[k] = ((key[k] & klmask) << pbits) | val[k];
  }
  __syncthreads();
  unsigned long long g = 0;
  uint32_t c = 0, inc = 0;
  if (tid < NB) {
    c = sh.cnt[tid];
    if (c) g = atomicAdd(&row[tid], (unsigned long long)c);   // the digit run's destination
    inc = wave_incl_sum<uint32_t>(c);
    if (lane == 63) sh.wsum[wv] = inc;
  }
  __syncthreads();
  if (tid < NB) {
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wv; ++w) carry += sh.wsum[w];
    sh.tst[tid] = carry + inc - c;
  }
  __syncthreads();
  if constexpr (HS) {
    // two rounds: the records of final slots [h * TILE / 2, (h + 1) * TILE / 2) staged, then written
    constexpr uint32_t HALF = (uint32_t)TILE / 2;
    if (tid < NB) sh.gb[tid] = (std::remove_reference_t<decltype(sh.gb[0])>)(g - sh.tst[tid]);
    const uint32_t hi256 = SD ? sh.tst[256] : 0u;   // final slots >= hi256 hold digits >= 256
#pragma unroll
    for (uint32_t h = 0; h < 2; ++h) {
      if (h) __syncthreads();   // the first half is written out
#pragma unroll
      for (int k = 0; k < CP_I; ++k)
        if (c0 + cst * k < tn) {
          const uint32_t f = sh.tst[rk[k] >> 16] + (rk[k] & 0xFFFFu);
          if (f - h * HALF < HALF) {
            sh.stage.keys[f - h * HALF] = key[k];
            if (SD) sh.sd[f - h * HALF] = (uint8_t)(rk[k] >> 16);
          }
        }
      __syncthreads();
#pragma unroll
      for (int i = 0; i < CP_I / 2; ++i) {
        const uint32_t s = (uint32_t)i * T + tid, fs = h * HALF + s;
        if (fs < tn) {
          const uint64_t kk = sh.stage.keys[s];
          const uint32_t d = SD ? (uint32_t)sh.sd[s] | (fs >= hi256 ? 256u : 0u) : (uint32_t)((kk - kbias) >> shift) & DM;
          if (SD) kout[(uint32_t)(sh.gb[d] + fs)] = kk;
          else kout[sh.gb[d] + fs] = kk;
        }
      }
    }
    return;
  }
#pragma unroll
  for (int k = 0; k < CP_I; ++k)
    if (c0 + cst * k < tn) {
      const uint32_t f = sh.tst[rk[k] >> 16] + (rk[k] & 0xFFFFu);
      sh.stage.keys[f] = key[k];
      if (SD) sh.sd[f] = (uint8_t)(rk[k] >> 16);
    }
  if (tid < NB) sh.gb[tid] = (std::remove_reference_t<decltype(sh.gb[0])>)(g - sh.tst[tid]);   // first use of the reservation
  __syncthreads();
  uint32_t dg[CP_I / 2] = {};   // digits of the staged slots, two per register
  const uint32_t hi256 = SD ? sh.tst[256] : 0u;   // staged slots >= hi256 hold digits >= 256
#pragma unroll
  for (int i = 0; i < CP_I; ++i) {
    const uint32_t s = (uint32_t)i * T + tid;
    if (s < tn) {
      const uint64_t kk = sh.stage.keys[s];
      const uint32_t d = SD ? (uint32_t)sh.sd[s] | (s >= hi256 ? 256u : 0u) : (uint32_t)((kk - kbias) >> shift) & DM;
      if (!PK) dg[i >> 1] |= d << (16 * (i & 1));
      if (SD) kout[(uint32_t)(sh.gb[d] + s)] = kk;
      else kout[sh.gb[d] + s] = kk;
    }
  }
  if (PK) return;
  __syncthreads();
#pragma unroll
  for (int k = 0; k < CP_I; ++k)
    if (c0 + cst * k < tn) sh.stage.vals[sh.tst[rk[k] >> 16] + (rk[k] & 0xFFFFu)] = val[k];
  __syncthreads();
#pragma unroll
  for (int i = 0; i < CP_I; ++i) {
    const uint32_t s = (uint32_t)i * T + tid;
    if (s < tn) vout[sh.gb[(dg[i >> 1] >> (16 * (i & 1))) & DM] + s] = sh.stage.vals[s];
  }
}

// ------------------------------------------------------------ 1c. sharded slices (keyed coarse splitters)
// A slice of a sharded build owns every suffix whose keyed sym field lies in [base << bsh, (base + nb)
// << bsh): its bin is (sym >> bsh) - base < nb.  With a whole-symbol keyed radix 2^lb, sym >> bsh is the
// first DB = sb - bsh bits of the sym field: a window of hq symbols with its low wdrop bits dropped, so
// the bin comes from the text exactly as the single-GPU cursor pre-pass computes its bucket.  The
// selection is therefore fused into the cursor partition: the pre-pass counts only the slice's suffixes
// (per span: bins and pass A digits), and pass A scans the whole text, keeps the slice's suffixes and
// scatters them by digit - no selection masks, no key planes in position order, no third pass.
// Every rank scans all of T' twice, so for radix 2^2 (DNA) both scans run in registers: a byte maps to
// its keyed code through an 8-entry byte table indexed by 3 bits of the byte (one v_perm_b32 per four
// bytes; the host picks the bit field that separates the keyed bytes), a multiply packs four codes,
// and each position's window is one v_alignbit of the packed words (REG kernels).
// (SliceSel: hk_bucket.hpp)

constexpr uint32_t SL_SUB = 8192;   // positions per sub-tile (= CP_TILE)

// keyed codes (radix 2^2) of 16 text bytes, packed MSB-first (first byte in bits 31..30).  A word's four
// codes (a byte each, from the table) fold into one byte by a dot product with the weights 64 / 16 / 4 / 1
// (v_dot4_u32_u8, full rate; the multiply it replaced is a quarter-rate v_mul_lo_u32).
__device__ __forceinline__ uint32_t pack16_2(const uint4& v, const SliceSel& sl) {
  auto p8 = [&](uint32_t w) -> uint32_t {
    const uint32_t c = __builtin_amdgcn_perm(sl.th, sl.tl, (w >> sl.ps) & 0x07070707u);   // 4 codes, a byte each
    return __builtin_amdgcn_udot4(c, 0x01041040u, 0u, false);   // c0 << 6 | c1 << 4 | c2 << 2 | c3
  };
  return (((p8(v.x) << 8) | p8(v.y)) << 16) | (p8(v.z) << 8) | p8(v.w);
}

// the 32 code bits from position k of the packed stream w0:w1 (k compile-time after unrolling)
__device__ __forceinline__ uint32_t win32(uint32_t w0, uint32_t w1, int k) {
  return k ? __builtin_amdgcn_alignbit(w0, w1, 32 - 2 * k) : w0;
}

// Pre-pass of a slice: for every text span (one workgroup), the slice's bin counts (CB-bit LDS counters
// as k_bucket_hist_spans) and its pass A digit counts.  REG: radix 2^2 in registers; else the LDS code
// table (LBQ / HQ compile-time when given).
// ALL (REG): the slice is the whole sym space (single-GPU build, coarse histogram): no selection test,
// and the add count of a full thread step is its 16 positions.
template <int CB, int HB = -1, int LBQ = 0, int HQ = 0, bool REG = false, bool ALL = false>
__global__ __launch_bounds__(BH_T, 1) void k_slice_hist_spans(const uint8_t* __restrict__ t, uint64_t n,
                                                              const uint16_t* __restrict__ lutk,
                                                              const uint64_t* __restrict__ skey, KeyedArgs g,
                                                              SliceSel sl, int D, uint32_t* __restrict__ part,
                                                              unsigned long long* __restrict__ drain,
                                                              uint32_t* __restrict__ spanc, uint64_t span,
                                                              unsigned long long* __restrict__ ovf) {
  constexpr int hb = HB;
  constexpr uint32_t HALF = 1u << (CB - 1);
  constexpr int CPW = 32 / CB;
  const uint32_t boff = hb > 0 ? 65536u : 0u;
  const int sA = sl.sA;
  bool bad = false;
  __shared__ uint32_t H[32768];
  __shared__ uint32_t M[CP_NAM];
  __shared__ uint16_t L[256];
  __shared__ uint64_t SK[72];
  __shared__ uint32_t KT[2];   // NODRAIN: adds, counter fields
  const uint32_t tid = threadIdx.x;
  for (uint32_t i = tid; i < 32768; i += BH_T) H[i] = 0;
  if (tid < CP_NAM) M[tid] = 0;
  if (tid < 256) L[tid] = lutk[tid];
  if (tid < 72) SK[tid] = skey[tid];
  if (tid < 2) KT[tid] = 0;
  __syncthreads();
  // REG, CB = 8: no drains.  Plain LDS adds (no returned value to wait for) and a count of the adds;
  // a byte that wrapped carries into its neighbour (or off the word), so the span's counter fields
  // then sum to less than the adds: the flush compares the two and raises *ovf (exact recount).
  constexpr bool NODRAIN = REG && CB == 8;
  uint32_t kc = 0;
  uint32_t kcw = 0;   // (REG, not ALL: the wave's adds of whole-wave steps, from the keep ballots)
  auto add = [&](uint32_t b, bool counted = false) {   // b: the slice bin, < sl.nb
    if constexpr (NODRAIN) {
      atomicAdd(&H[b >> 2], 1u << (8 * (b & 3)));
      if constexpr (!ALL) if (!counted) ++kc;
      return;
    }
    if (hb >= 0 && (b >> 16) != (uint32_t)hb) return;
    const uint32_t bl = b - boff;
    const uint32_t sh = CB * (bl % CPW);
    const uint32_t old = atomicAdd(&H[bl / CPW], 1u << sh);
    const uint32_t ob = (old >> sh) & ((1u << CB) - 1);
    if (CB == 8) bad |= ob >= 224u;
    if (ob == HALF - 1) {
      atomicSub(&H[bl / CPW], HALF << sh);
      atomicAdd(&drain[b], (unsigned long long)HALF);
      atomicAdd(&M[b >> sA], HALF);
    }
  };
  const uint64_t lim = n < g.s_start ? n : g.s_start;   // positions with a text window
  const uint64_t lo = (uint64_t)blockIdx.x * span;
  const uint64_t hi = lo + span < n ? lo + span : n;
  const int lb = LBQ ? LBQ : 31 - __clz((uint32_t)g.Rk);
  const int hq = HQ ? HQ : sl.hq;
  constexpr int NI = HQ ? BH_PER + HQ - 1 : 2 * BH_PER - 1;
  static_assert(NI <= 2 * BH_PER, "window past the thread's 32 bytes");
  const int wbits = hq * lb, wdrop = sl.wdrop, dsh = 32 - sl.DB;
  const uint32_t bmask = wbits >= 32 ? ~0u : (1u << wbits) - 1;
  // PF iterations' bytes in flight: slot u's registers are consumed, then reloaded with the bytes PF
  // iterations ahead (a rotating prefetch makes the compiler copy the new registers at the back edge,
  // which waits for the loads just issued)
  // (the loads are unconditional, a position past the span reads the span's first bytes instead: a
  // load under a branch leaves the wait-count pass no exact count, so it waits for all of them)
  constexpr int PF = REG ? 4 : 2;
  uint4 f0[PF], f1[PF];
  auto fetch = [&](uint64_t p, uint4& x0, uint4& x1) {
    const uint4* src = reinterpret_cast<const uint4*>(t + (p < hi ? p : lo));
    x0 = src[0];
    x1 = src[1];
  };
#pragma unroll
  for (int u = 0; u < PF; ++u) fetch(lo + (uint64_t)u * BH_TILE + (uint64_t)tid * BH_PER, f0[u], f1[u]);
  const uint64_t lim2 = lim < hi ? lim : hi;
  auto step = [&](uint64_t p0, const uint4 a, const uint4 b4) {
    if constexpr (REG && NODRAIN && !ALL) {
      if (__all(p0 + BH_PER <= lim2)) {   // (uniform) every lane's 16 positions keyed: the wave's adds
        const uint32_t c0 = pack16_2(a, sl), c1 = pack16_2(b4, sl);   // counted from the keep ballots (SALU)
#pragma unroll
        for (int k = 0; k < BH_PER; ++k) {
          const uint32_t w = win32(c0, c1, k) - sl.wb;
          const bool keep = w <= sl.wn1;
          kcw += (uint32_t)__popcll(__ballot(keep));
          if (keep) add(w >> dsh, true);
        }
        return;
      }
    }
    if (p0 < lim2) {
      const bool full = p0 + BH_PER <= lim2;
      if constexpr (REG) {
        const uint32_t c0 = pack16_2(a, sl), c1 = pack16_2(b4, sl);
        if (full) {   // (split so the full body carries no per-position 64-bit bound test)
#pragma unroll
          for (int k = 0; k < BH_PER; ++k) {
            if constexpr (ALL) {
              add(win32(c0, c1, k) >> dsh);
            } else {
              const uint32_t w = win32(c0, c1, k) - sl.wb;
              if (w <= sl.wn1) add(w >> dsh);
            }
          }
          if constexpr (ALL && NODRAIN) kc += BH_PER;
        } else {
#pragma unroll
          for (int k = 0; k < BH_PER; ++k) {
            const uint32_t w = win32(c0, c1, k) - sl.wb;
            if (w <= sl.wn1 && p0 + k < lim2) {
              add(w >> dsh);
              if constexpr (ALL && NODRAIN) ++kc;
            }
          }
        }
      } else {
        const uint32_t wd[8] = {a.x, a.y, a.z, a.w, b4.x, b4.y, b4.z, b4.w};
        uint32_t b = 0;
#pragma unroll
        for (int i = 0; i < NI; ++i) {
          b = ((b << lb) | (L[(wd[i >> 2] >> (8 * (i & 3))) & 255u] & 255u)) & bmask;
          const int j = i - (hq - 1);
          if (j >= 0 && j < BH_PER && (full || p0 + j < lim2)) {
            const uint32_t bin = (b >> wdrop) - sl.base;
            if (bin < sl.nb) add(bin);
          }
        }
      }
    }
    for (uint64_t p = p0 > lim ? p0 : lim; p < p0 + BH_PER && p < hi; ++p) {
      const uint32_t bin = (uint32_t)(SK[p - g.s_start] >> sl.bsh) - sl.base;
      if (bin < sl.nb) {
        add(bin);
        if constexpr (ALL && NODRAIN) ++kc;
      }
    }
  };
  for (uint64_t base = lo; base < hi; base += PF * BH_TILE) {
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint64_t bu = base + (uint64_t)u * BH_TILE;
      if (bu >= hi) break;   // uniform
      const uint64_t p0 = bu + (uint64_t)tid * BH_PER;
      step(p0, f0[u], f1[u]);
      fetch(p0 + PF * BH_TILE, f0[u], f1[u]);
    }
  }
  if (CB == 8 && bad) atomicOr(ovf, 1ull);
  if (NODRAIN) {
    const uint32_t wk = wave_incl_sum<uint32_t>(kc) + (uint32_t)__builtin_amdgcn_readfirstlane(kcw);
    if ((tid & 63) == 63 && wk) atomicAdd(&KT[0], wk);
  }
  __syncthreads();
  const uint32_t nbl = hb >= 0 ? 65536u : 1u << D;
  hist_spans_flush<CB>(H, M, nbl, boff, 1u << D, sA, part, spanc, NODRAIN ? &KT[1] : nullptr);
  if (NODRAIN) {
    __syncthreads();
    if (tid == 0 && KT[0] != KT[1]) atomicOr(ovf, 1ull);
  }
}

// Pass A of a slice: workgroup = one unit (g sub-tiles of CP_TILE positions of one span).  Round 1
// counts the unit's kept suffixes per pass A digit (LDS atomics, nothing staged); when they fit one
// tile (<= CP_TILE, iid text: g is ~0.9 of the text / slice ratio) the runs are reserved at once and
// round 2 keys the unit again, staging every kept suffix straight at its final slot; a denser unit
// (non-iid text) takes each sub-tile as a tile of its own (rank, reserve, stage, write).  PK: packed
// records ((sym - (base << bsh)) & the bits below the pass A digit, prev code, position), one u64
// each; else keys (sym - (base << bsh)) << pbe | prev << hb | position >> 32 and u32 values.
// REG (radix 2^2, packed records): keys in registers from the thread's 16 consecutive positions
// (three 16-B loads and the word before; prev codes from the stream).  Else CONSEC (radix 2^2, packed):
// text_keys_consec2 over the LDS-staged sub-tile; else lane-strided text_keys.
template <bool CONSEC>
struct SlText {   // one sub-tile's text staging (text_keys: packed codes + raw bytes)
  uint32_t pk[(CP_TILE + 64) / 4 + 4];
  uint8_t raw[CP_TILE + 64];
};
template <>
struct SlText<true> {   // radix 2^2, consecutive items (text_keys_consec2): packed codes only
  uint32_t pk[(CP_TILE + 64) / 16 + 4];
};

template <int LB, bool PK, bool REG>
struct SlShared {
  uint64_t keys[CP_TILE];           // records / keys by final slot
  uint32_t vals[PK ? 1 : CP_TILE];  // key planes: low position bits by final slot
  uint8_t sd[CP_TILE];              // low 8 bits of each staged slot's digit
  SlText<LB == 2 && PK> tx[REG ? 0 : 1];
  uint32_t tg[CP_NAM];   // tile-local exclusive digit starts, then the runs' destinations minus them
  uint32_t cnt[CP_NAM];
  uint32_t wsum[CP_NAM / 64];
  uint32_t prev0;
  uint16_t L[256], LP[256];
  uint64_t SK[72];
};

template <int LB, bool PK, bool REG = false>
__global__ __launch_bounds__(CP_T, 2) void k_slice_cpart(uint64_t* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         uint64_t n, unsigned long long* __restrict__ cur,
                                                         uint64_t span, TextKeySrc src, SliceSel sl,
                                                         const unsigned long long* __restrict__ skip,
                                                         uint64_t mcap) {
  constexpr int T = CP_T;
  static_assert(!REG || (LB == 2 && PK), "register keys: radix 2^2 packed records");
  // consecutive items take their prev codes from the keyed code stream: packed records only (a key
  // plane's prev field is the dense code)
  constexpr bool CONSEC = LB == 2 && PK;
  __shared__ SlShared<LB, PK, REG> sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (skip && *skip) return;   // the pre-pass counters overflowed: recounted, then relaunched
  const uint64_t U = (uint64_t)SL_SUB * sl.g;
  // XCD groups as k_cpart: workgroups b, b + 8, ... take consecutive units of one span
  const uint32_t per = (uint32_t)(span / U), gx = blockIdx.x & 7u, k8 = blockIdx.x >> 3;
  const uint64_t unit = (uint64_t)(gx + 8u * (k8 / per)) * per + k8 % per;
  const uint64_t ubase = unit * U;
  if (ubase >= n) return;   // past the last span (whole workgroup, before any barrier)
  unsigned long long* const row = cur + (ubase / span) * CP_NAM;
  if (tid < 256) {
    sh.L[tid] = src.lutk[tid];
    sh.LP[tid] = src.lutp[tid];
  }
  if (tid < 72) sh.SK[tid] = src.skey[tid];
  sh.cnt[tid] = 0;
  __syncthreads();
  const uint64_t lim = n < src.g.s_start ? n : src.g.s_start;
  const uint64_t kmask_lo = (1ull << (sl.bsh + sl.sA)) - 1;   // record: the bits below the pass A digit
  const uint64_t sbase = (uint64_t)sl.base << sl.bsh;
  const int kpb = src.g.pb;                                    // prev bits of the keys
  const uint64_t pmk = (1ull << kpb) - 1;
  const int hbk = PK ? 0 : sl.pbe - kpb;                       // key planes: position-high bits
  const int dsh = 32 - sl.DB, kbits = 2 * src.g.q;
  const uint32_t nsub = (uint32_t)((n - ubase < U ? n - ubase : U) + SL_SUB - 1) / SL_SUB;
  uint64_t key[CP_I];
  uint32_t rk[CP_I];
  auto keys_of = [&](uint64_t tb) {
    __syncthreads();   // the previous sub-tile's staging has been read
    if constexpr (REG) {
      // no staging: this thread's 16 consecutive positions from three 16-B loads (T' has 64 pad bytes)
      const uint64_t p0 = tb + 16ull * tid;
      if (p0 >= n) {
#pragma unroll
        for (int k = 0; k < CP_I; ++k) key[k] = ~0ull;
        return;
      }
      const uint4* q4 = reinterpret_cast<const uint4*>(src.text + p0);
      const uint32_t c0 = pack16_2(q4[0], sl), c1 = pack16_2(q4[1], sl), c2 = pack16_2(q4[2], sl);
      uint32_t pc;   // prev code of position p0: the records' code of T'[p0 - 1] (T'[n - 1] for p0 = 0)
      if (p0) {
        const uint32_t pw = reinterpret_cast<const uint32_t*>(src.text + p0)[-1] >> 24;
        pc = __builtin_amdgcn_perm(sl.th, sl.tl, (pw >> sl.ps) & 7u) & 3u;
      } else {
        pc = sh.LP[src.text[n - 1]];
      }
#pragma unroll
      for (int k = 0; k < CP_I; ++k) {
        const uint64_t j = p0 + k;
        const uint64_t win = ((uint64_t)win32(c0, c1, k) << 32) | win32(c1, c2, k);
        uint64_t sym = kbits >= 64 ? win : win >> (64 - kbits);
        if (j >= src.g.s_start) sym = j < n ? sh.SK[j - src.g.s_start] : 0;
        const uint32_t prv = k ? (c0 >> (32 - 2 * k)) & 3u : pc;
        key[k] = j < n ? (sym << kpb) | prv : ~0ull;
      }
    } else if constexpr (CONSEC) {
      text_keys_consec2<T>(key, src, n, tb, sh.tx[0].pk, &sh.prev0, sh.L, sh.LP, sh.SK);
    } else {
      text_keys<T, CP_I, LB>(key, src, n, tb, tb + (uint64_t)wv * (CP_I * 64), lane, nullptr, sh.tx[0].pk,
                             sh.tx[0].raw, &sh.prev0, sh.L, sh.LP, sh.SK);
    }
  };
  auto pos_of = [&](uint64_t tb, int k) -> uint64_t {
    return (REG || CONSEC) ? tb + 16ull * tid + (uint64_t)k : tb + (uint64_t)wv * (CP_I * 64) + 64ull * k + lane;
  };
  // the kept suffix's record / key and its pass A digit (~0u: not in the slice)
  auto record = [&](uint64_t j, uint64_t kk, uint64_t& out) -> uint32_t {
    if (j >= n) return ~0u;
    const uint64_t sym = kk >> kpb;
    const uint32_t bin = (uint32_t)(sym >> sl.bsh) - sl.base;
    if (bin >= sl.nb) return ~0u;
    const uint64_t x = sym - sbase;
    if (PK) out = ((((x & kmask_lo) << sl.pb2) | (kk & pmk)) << sl.pbits) | j;
    else out = (x << sl.pbe) | ((kk & pmk) << hbk) | (hbk ? j >> 32 : 0ull);
    return bin >> sl.sA;
  };
  auto write_out = [&](uint32_t cnt_tile, uint32_t hi256) {
    for (int i = 0; i < CP_I; ++i) {
      const uint32_t s = (uint32_t)i * T + tid;
      if (s < cnt_tile) {
        const uint32_t d = (uint32_t)sh.sd[s] | (s >= hi256 ? 256u : 0u);
        const uint32_t o = sh.tg[d] + s;   // u32 arithmetic: tg = destination - tile start (mod 2^32)
        if (o < mcap) {   // guard: counts that disagree with the pre-pass fail the host's check, not memory
          kout[o] = sh.keys[s];
          if constexpr (!PK) vout[o] = sh.vals[s];
        }
      }
    }
  };
  // ---- round 1: the unit's kept suffixes per digit
  for (uint32_t st = 0; st < nsub; ++st) {
    const uint64_t tb = ubase + (uint64_t)st * SL_SUB;
    if constexpr (REG) {   // bins only, from two 16-B loads
      const uint64_t p0 = tb + 16ull * tid;
      if (p0 < n) {
        const uint4* q4 = reinterpret_cast<const uint4*>(src.text + p0);
        const uint32_t c0 = pack16_2(q4[0], sl), c1 = pack16_2(q4[1], sl);
        const bool full = p0 + 16 <= lim;
#pragma unroll
        for (int k = 0; k < CP_I; ++k) {
          const uint32_t bin = (win32(c0, c1, k) >> dsh) - sl.base;
          if (bin < sl.nb && (full || p0 + k < lim)) atomicAdd(&sh.cnt[bin >> sl.sA], 1u);
        }
        for (uint64_t j = p0 > lim ? p0 : lim; j < p0 + 16 && j < n; ++j) {   // short suffixes
          const uint32_t bin = (uint32_t)(sh.SK[j - src.g.s_start] >> sl.bsh) - sl.base;
          if (bin < sl.nb) atomicAdd(&sh.cnt[bin >> sl.sA], 1u);
        }
      }
    } else {
      keys_of(tb);
#pragma unroll
      for (int k = 0; k < CP_I; ++k) {
        uint64_t rec = 0;
        const uint32_t d = record(pos_of(tb, k), key[k], rec);
        if (d != ~0u) atomicAdd(&sh.cnt[d], 1u);
      }
    }
  }
  __syncthreads();
  const uint32_t cu = sh.cnt[tid];
  uint32_t total = 0;
  {
    const uint32_t inc = wave_incl_sum<uint32_t>(cu);
    if (lane == 63) sh.wsum[wv] = inc;
    __syncthreads();
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; ++w) {
      carry += w < wv ? sh.wsum[w] : 0u;
      total += sh.wsum[w];
    }
    sh.tg[tid] = carry + inc - cu;
    sh.cnt[tid] = 0;   // every thread read its own count above
  }
  const bool fast = total <= (uint32_t)CP_TILE;
  if (fast) {
    // the unit's runs reserved now (the result is first needed at the write-out)
    const unsigned long long resv = cu ? atomicAdd(&row[tid], (unsigned long long)cu) : 0ull;
    __syncthreads();
    for (uint32_t st = 0; st < nsub; ++st) {
      const uint64_t tb = ubase + (uint64_t)st * SL_SUB;
      keys_of(tb);
#pragma unroll
      for (int k = 0; k < CP_I; ++k) {
        const uint64_t j = pos_of(tb, k);
        uint64_t rec = 0;
        const uint32_t d = record(j, key[k], rec);
        if (d != ~0u) {
          uint32_t f = sh.tg[d] + atomicAdd(&sh.cnt[d], 1u);
          f = f < (uint32_t)CP_TILE ? f : (uint32_t)CP_TILE - 1;   // (only a count mismatch overruns)
          sh.keys[f] = rec;
          sh.sd[f] = (uint8_t)d;
          if constexpr (!PK) sh.vals[f] = (uint32_t)j;
        }
      }
    }
    __syncthreads();
    const uint32_t hi256 = sh.tg[256];   // staged slots >= hi256 hold digits >= 256
    const uint32_t gbv = (uint32_t)(resv - sh.tg[tid]);
    __syncthreads();
    sh.tg[tid] = gbv;
    __syncthreads();
    write_out(total, hi256);
    return;
  }
  // dense unit: every sub-tile is a tile of its own
  for (uint32_t st = 0; st < nsub; ++st) {
    const uint64_t tb = ubase + (uint64_t)st * SL_SUB;
    keys_of(tb);   // (barrier first: the previous tile's write-out has read sh)
    sh.cnt[tid] = 0;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CP_I; ++k) {
      const uint64_t j = pos_of(tb, k);
      uint64_t rec = 0;
      const uint32_t d = record(j, key[k], rec);
      key[k] = rec;
      rk[k] = d == ~0u ? ~0u : (atomicAdd(&sh.cnt[d], 1u) | (d << 16));
    }
    __syncthreads();
    const uint32_t c = sh.cnt[tid];
    const unsigned long long g = c ? atomicAdd(&row[tid], (unsigned long long)c) : 0ull;
    const uint32_t inc = wave_incl_sum<uint32_t>(c);
    if (lane == 63) sh.wsum[wv] = inc;
    __syncthreads();
    uint32_t carry = 0, tot = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; ++w) {
      carry += w < wv ? sh.wsum[w] : 0u;
      tot += sh.wsum[w];
    }
    sh.tg[tid] = carry + inc - c;
    __syncthreads();
#pragma unroll
    for (int k = 0; k < CP_I; ++k)
      if (rk[k] != ~0u) {
        const uint32_t d = rk[k] >> 16;
        const uint32_t f = sh.tg[d] + (rk[k] & 0xFFFFu);
        sh.keys[f] = key[k];
        sh.sd[f] = (uint8_t)d;
        if constexpr (!PK) sh.vals[f] = (uint32_t)pos_of(tb, k);
      }
    __syncthreads();
    const uint32_t hi256 = sh.tg[256];
    const uint32_t gbv = (uint32_t)(g - sh.tg[tid]);
    __syncthreads();
    sh.tg[tid] = gbv;
    __syncthreads();
    write_out(tot, hi256);
  }
}

// (stamp(), the TRACE phase stamps: hk_bucket.hpp)

// Pass A of a slice, radix 2^2 packed records (g <= SL_G sub-tiles per unit): the unit's text is copied
// into LDS up front by DMA (every load in flight together, no VGPRs held), the packed codes and the
// kept-position masks stay in registers between round 1 (bins -> digit counts) and round 2, which keys
// only the kept positions (a bit loop: ~1/N of the 16 per sub-tile) and stages them at their final slots.  Each sub-tile of a unit denser than one tile is
// ranked, reserved and written on its own (non-iid text), as in k_slice_cpart.
constexpr int SL_G = 8;
// quarter staging: units of <= 3 sub-tiles keeping <= 3584 records (slices of <= 1/7.5 of T', N >= 8), 37 KiB
// of LDS, four workgroups per CU; a dense sub-tile is staged in quarters
constexpr int SL_CAPQ = 3584;

// G: sub-tiles per unit held in registers; CAP: staging capacity (records of one write-out).  CAP =
// CP_TILE / 2 (N >= 4: units of <= 4 sub-tiles keep ~1/N of their positions) halves the LDS to ~41 KiB,
// so three workgroups share a CU instead of two (the kernel waits between its DMA, ranking and write
// phases); a dense sub-tile is then staged in two halves (its positions k < 8, then k >= 8).
template <bool TRACE = false, int G = SL_G, int CAP = CP_TILE>
__global__ __launch_bounds__(CP_T, CAP == CP_TILE ? 4 : CAP == CP_TILE / 2 ? 6 : 8) void k_slice_cpart_reg(uint64_t* __restrict__ kout, uint64_t n,
                                                             unsigned long long* __restrict__ cur, uint64_t span,
                                                             TextKeySrc src, SliceSel sl,
                                                             const unsigned long long* __restrict__ skip,
                                                             uint64_t mcap, uint64_t* __restrict__ trace = nullptr) {
  constexpr int T = CP_T;
  static_assert((uint64_t)G * SL_SUB + 64 <= (uint64_t)(CAP + 8) * 8, "the unit's text image fits the staging");
  static_assert(CAP == CP_TILE || CAP == CP_TILE / 2 || CAP == SL_CAPQ, "full, half or quarter staging");
  __shared__ uint64_t keys[CAP + 8];   // round 1: the unit's text image (<= G sub-tiles + 64 B)
  __shared__ uint8_t sdg[CAP];
  __shared__ uint32_t tg[CP_NAM], cnt[CP_NAM], wsum[CP_NAM / 64];
  __shared__ uint16_t LP[256];
  __shared__ uint64_t SK[72];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = __builtin_amdgcn_readfirstlane(tid >> 6);   // (wv in an SGPR)
  if (skip && *skip) return;   // the pre-pass counters overflowed: recounted, then relaunched
  const uint64_t U = (uint64_t)SL_SUB * sl.g;
  const uint32_t per = (uint32_t)(span / U), gx = blockIdx.x & 7u, k8 = blockIdx.x >> 3;
  const uint64_t unit = (uint64_t)(gx + 8u * (k8 / per)) * per + k8 % per;
  const uint64_t ubase = unit * U;
  if (ubase >= n) return;   // past the last span (whole workgroup, before any barrier)
  uint64_t ts[5] = {0, 0, 0, 0, 0};
  if (TRACE) ts[0] = stamp();
  auto trace_out = [&]() {
    if (TRACE && tid == 0) {
      ts[4] = stamp();
      for (int i = 0; i < 5; ++i) trace[(uint64_t)blockIdx.x * 8 + i] = ts[i];
      trace[(uint64_t)blockIdx.x * 8 + 5] = 1;
    }
  };
  unsigned long long* const row = cur + (ubase / span) * CP_NAM;
  const uint32_t nsub = (uint32_t)((n - ubase < U ? n - ubase : U) + SL_SUB - 1) / SL_SUB;
  // the unit's text bytes [ubase - 16, ubase + U + 48) land in LDS by DMA (global_load_lds, 1 KiB per
  // wave-instruction, all in flight together, no VGPRs held); bytes outside [0, n + 64) are not read
  // (T' has 64 readable pad bytes; positions past n only feed short suffixes, keyed from SK)
  uint8_t* const img = reinterpret_cast<uint8_t*>(keys);
  __shared__ uint32_t last_byte;   // position 0's prev byte (every global load done before the copies)
  if (tid == 0) last_byte = src.text[n - 1];
  if (tid < 256) LP[tid] = src.lutp[tid];
  if (tid < 72) SK[tid] = src.skey[tid];
  cnt[tid] = 0;
  // the unit's text bytes [ubase - 16, ubase + U + 48) land in LDS by DMA (1 KiB per wave-instruction,
  // all in flight together, no VGPRs held); bytes outside [0, n + 64) are not read (T' has 64 readable
  // pad bytes; positions past n only feed short suffixes, keyed from SK).  Issued after every other
  // global load, waited for once.  (Per-wave copies of each sub-tile with counted waits instead were
  // slower: 8.5 vs 7.8 ms per emulated N = 8 rank.)
  {
    const uint32_t nins = (uint32_t)((U + 64 + 1023) / 1024);
    for (uint32_t i = wv; i < nins; i += T / 64) {
      const uint64_t off = (uint64_t)i * 1024 + lane * 16u;   // image byte of this lane
      if (ubase + off >= 16 && ubase + off <= n + 64)
        __builtin_amdgcn_global_load_lds(src.text + (ubase + off - 16), img + (uint64_t)i * 1024, 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t lim = n < src.g.s_start ? n : src.g.s_start;
  const uint64_t sbase = (uint64_t)sl.base << sl.bsh;
  const int kbits = 2 * src.g.q, dsh = 32 - sl.DB;
  // ---- round 1: packed codes (from the LDS image), kept-position masks, digit counts
  uint32_t c[G][3], msk[G], pcs = 0;
#pragma unroll
  for (int st = 0; st < G; ++st) {
    msk[st] = 0;
    c[st][0] = c[st][1] = c[st][2] = 0;
    const uint64_t p0 = ubase + (uint64_t)st * SL_SUB + 16ull * tid;
    if ((uint32_t)st >= nsub || p0 >= n) continue;
    const uint32_t ib = 16u + (uint32_t)st * SL_SUB + 16u * tid;
    const uint4* q4 = reinterpret_cast<const uint4*>(img + ib);
    c[st][0] = pack16_2(q4[0], sl);
    c[st][1] = pack16_2(q4[1], sl);
    c[st][2] = pack16_2(q4[2], sl);
    // prev code of p0: the records' code of T'[p0 - 1] (T'[n - 1] for p0 = 0)
    const uint32_t pb = reinterpret_cast<const uint32_t*>(img + ib)[-1] >> 24;
    const uint32_t pc = p0 ? __builtin_amdgcn_perm(sl.th, sl.tl, (pb >> sl.ps) & 7u) & 3u : (uint32_t)LP[last_byte];
    pcs |= pc << (2 * st);
    const bool full = p0 + 16 <= lim;
    uint32_t m = 0;
    const int dA = dsh + sl.sA;
    if (full) {
#pragma unroll
      for (int k = 0; k < CP_I; ++k) {
        const uint32_t w = win32(c[st][0], c[st][1], k) - sl.wb;
        if (w <= sl.wn1) {
          m |= 1u << k;
          atomicAdd(&cnt[w >> dA], 1u);
        }
      }
    } else {
#pragma unroll
      for (int k = 0; k < CP_I; ++k) {
        const uint32_t w = win32(c[st][0], c[st][1], k) - sl.wb;
        if (w <= sl.wn1 && p0 + k < lim) {
          m |= 1u << k;
          atomicAdd(&cnt[w >> dA], 1u);
        }
      }
    }
    for (uint64_t j = p0 > lim ? p0 : lim; j < p0 + 16 && j < n; ++j) {   // short suffixes: boundary keys
      const uint32_t bin = (uint32_t)(SK[j - src.g.s_start] >> sl.bsh) - sl.base;
      if (bin < sl.nb) {
        m |= 1u << (uint32_t)(j - p0);
        atomicAdd(&cnt[bin >> sl.sA], 1u);
      }
    }
    msk[st] = m;
  }
  // the record of kept position k of sub-tile st (runtime k) and its pass A digit
  // (the 64-bit window minus the slice base at its sym field: its top kbits are sym - sbase, whose
  // low Z bits go to the record and whose bits above them are the pass A digit)
  const int Z = sl.bsh + sl.sA, pz = sl.pb2 + sl.pbits;
  const uint64_t wS = sbase << (64 - kbits);
  auto record_at = [&](int st, int k, uint64_t& rec) -> uint32_t {
    const uint64_t j = ubase + (uint64_t)st * SL_SUB + 16ull * tid + (uint64_t)k;
    const int sh = 32 - 2 * k;   // 2..32
    const uint64_t s01 = ((uint64_t)c[st][0] << 32) | c[st][1], s12 = ((uint64_t)c[st][1] << 32) | c[st][2];
    uint64_t wr = (((uint64_t)(uint32_t)(s01 >> sh) << 32) | (uint32_t)(s12 >> sh)) - wS;
    if (j >= src.g.s_start) wr = (SK[j - src.g.s_start] - sbase) << (64 - kbits);
    const uint32_t prv = (uint32_t)(((((uint64_t)((pcs >> (2 * st)) & 3u)) << 32) | c[st][0]) >> sh) & 3u;
    rec = (((wr << (kbits - Z)) >> (64 - Z)) << pz) | ((uint64_t)prv << sl.pbits) | j;
    return (uint32_t)(wr >> (64 - kbits + Z));
  };
  if (TRACE) ts[1] = stamp();
  __syncthreads();
  const uint32_t cu = cnt[tid];
  uint32_t total = 0;
  {
    const uint32_t inc = wave_incl_sum<uint32_t>(cu);
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    uint32_t carry = 0;
#pragma unroll
    for (uint32_t w = 0; w < T / 64; ++w) {
      carry += w < wv ? wsum[w] : 0u;
      total += wsum[w];
    }
    tg[tid] = carry + inc - cu;
    cnt[tid] = 0;
  }
  auto write_out = [&](uint32_t cnt_tile, uint32_t hi256) {
    for (int i = 0; i < CAP / T; ++i) {
      const uint32_t s = (uint32_t)i * T + tid;
      if (s < cnt_tile) {
        const uint32_t d = (uint32_t)sdg[s] | (s >= hi256 ? 256u : 0u);
        const uint32_t o = tg[d] + s;   // u32: tg = destination - tile start (mod 2^32)
        if (o < mcap) kout[o] = keys[s];
      }
    }
  };
  if (total <= (uint32_t)CAP) {
    const unsigned long long resv = cu ? atomicAdd(&row[tid], (unsigned long long)cu) : 0ull;
    __syncthreads();
    if (TRACE) ts[2] = stamp();
    // ---- round 2: key and stage the kept positions only
#pragma unroll
    for (int st = 0; st < G; ++st) {
      uint32_t m = msk[st];
      while (m) {   // two kept positions a trip: their slot atomics in flight together
        const int k = __builtin_ctz(m);
        m &= m - 1;
        const bool two = m != 0;
        const int k2 = two ? __builtin_ctz(m) : k;
        m &= m - 1;
        uint64_t rec, rec2;
        const uint32_t d = record_at(st, k, rec);
        const uint32_t d2 = record_at(st, k2, rec2);
        uint32_t f = tg[d] + atomicAdd(&cnt[d], 1u);
        uint32_t f2 = two ? tg[d2] + atomicAdd(&cnt[d2], 1u) : 0u;
        f = f < (uint32_t)CAP ? f : (uint32_t)CAP - 1;   // (only a count mismatch overruns)
        keys[f] = rec;
        sdg[f] = (uint8_t)d;
        if (two) {
          f2 = f2 < (uint32_t)CAP ? f2 : (uint32_t)CAP - 1;
          keys[f2] = rec2;
          sdg[f2] = (uint8_t)d2;
        }
      }
    }
    __syncthreads();
    if (TRACE) ts[3] = stamp();
    const uint32_t hi256 = tg[256];
    const uint32_t gbv = (uint32_t)(resv - tg[tid]);
    __syncthreads();
    tg[tid] = gbv;
    __syncthreads();
    write_out(total, hi256);
    trace_out();
    return;
  }
  // dense unit: each sub-tile (half staging: each half of a sub-tile) counted, reserved, staged and written on
  // its own (ranks by a second round of atomics, as the fast path: no per-position rank registers)
  constexpr int PARTS = CAP == CP_TILE ? 1 : CAP >= CP_TILE / 2 ? 2 : 4;
#pragma unroll
  for (int st = 0; st < G; ++st) {   // (unrolled: c[st] / msk[st] stay register-resident)
    if ((uint32_t)st >= nsub) break;   // uniform
#pragma unroll
    for (int part = 0; part < PARTS; ++part) {
      const uint32_t pm = msk[st] & (((1u << (16 / PARTS)) - 1u) << (16 / PARTS * part));
      __syncthreads();   // the previous write-out has read keys / tg; counters free
      cnt[tid] = 0;
      __syncthreads();
      for (uint32_t m = pm; m; m &= m - 1) {
        uint64_t rec;
        atomicAdd(&cnt[record_at(st, __builtin_ctz(m), rec)], 1u);
      }
      __syncthreads();
      const uint32_t cc = cnt[tid];
      unsigned long long* rowp = row;
      asm volatile("" : "+s"(rowp));   // (re-derived per sub-tile: a hoisted row + tid pair spilled at 80 VGPRs)
      const unsigned long long g = cc ? atomicAdd(&rowp[tid], (unsigned long long)cc) : 0ull;
      const uint32_t inc = wave_incl_sum<uint32_t>(cc);
      if (lane == 63) wsum[wv] = inc;
      __syncthreads();
      uint32_t carry = 0, tot = 0;
#pragma unroll
      for (uint32_t w = 0; w < T / 64; ++w) {
        carry += w < wv ? wsum[w] : 0u;
        tot += wsum[w];
      }
      tg[tid] = carry + inc - cc;
      cnt[tid] = 0;
      __syncthreads();
      for (uint32_t m = pm; m; m &= m - 1) {
        uint64_t rec;
        const uint32_t d = record_at(st, __builtin_ctz(m), rec);
        const uint32_t f = tg[d] + atomicAdd(&cnt[d], 1u);
        keys[f] = rec;
        sdg[f] = (uint8_t)d;
      }
      __syncthreads();
      const uint32_t hi256 = tg[256];
      const uint32_t gbv = (uint32_t)(g - tg[tid]);
      __syncthreads();
      tg[tid] = gbv;
      __syncthreads();
      write_out(tot, hi256);
    }
  }
}

// Fused pass A of up to FS_N slices of one single-GPU build (n >= 2^32 - 1): one scan of T' keys every
// position once for the whole group, instead of one scan per slice (each of which keyed all of T' to keep
// a quarter of it).  The group's slices are contiguous and each starts at a pass A digit boundary (its
// first bin a multiple of 2^sA), so a window's group digit (w >> dA) - gd0 indexes one count array for all
// of them (u16 pairs: a unit has < 2^16 positions) and its slice follows from the digit bounds; round 1
// keeps each kept position's slice (2 bits) next to the packed codes.  Then, slice by slice, the reserve /
// round 2 / write-out of k_slice_cpart_reg, into the slice's own cursor rows and output.
constexpr int FS_N = 4;
// staging of one slice's records of a unit: ~1/4 of <= 3 sub-tiles (6144 for iid text) + margin; 67 KiB of
// LDS in all, two workgroups per CU (a full tile's 81 KiB allowed one); a dense unit is staged by half sub-tiles
constexpr int FS_CAP = 6656;
struct FusedSel {
  uint64_t* kout[FS_N];
  unsigned long long* cur[FS_N];   // [span][CP_NAM] cursor rows of each slice's pre-pass
  uint64_t mcap[FS_N];
  uint32_t base[FS_N];             // the slice's first bin
  uint32_t gd[FS_N + 1];           // group digits of slice s: [gd[s], gd[s + 1]), gd[0] = 0; ~0u past ns
  uint32_t gd0;                    // the group's first absolute digit (base[0] >> sA)
  int ns;
};

// G: sub-tiles per unit held in registers (g <= G; groups of <= 4 of every slice of the text have g <= 3)
template <int G>
__global__ __launch_bounds__(CP_T, 4) void k_slice_cpart_fused(uint64_t n, uint64_t span, TextKeySrc src, SliceSel sl,
                                                               FusedSel fs, const unsigned long long* __restrict__ skip) {
  constexpr int T = CP_T;
  static_assert((uint64_t)G * SL_SUB + 64 <= (uint64_t)(FS_CAP + 8) * 8, "the unit's text image fits the staging");
  __shared__ uint64_t keys[FS_CAP + 8];   // round 1: the unit's text image; then the staged records
  __shared__ uint8_t sdg[FS_CAP];
  __shared__ uint32_t cnt[FS_N * CP_NAM / 2];   // u16 digit counters, two per word
  __shared__ uint32_t tg[CP_NAM], wsum[CP_NAM / 64];
  __shared__ uint16_t LP[256];
  __shared__ uint64_t SK[72];
  __shared__ uint32_t last_byte;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (skip && *skip) return;   // a pre-pass overflowed: the slices run one by one instead
  const uint64_t U = (uint64_t)SL_SUB * sl.g;
  const uint32_t per = (uint32_t)(span / U), gx = blockIdx.x & 7u, k8 = blockIdx.x >> 3;
  const uint64_t unit = (uint64_t)(gx + 8u * (k8 / per)) * per + k8 % per;
  const uint64_t ubase = unit * U;
  if (ubase >= n) return;   // past the last span (whole workgroup, before any barrier)
  const uint64_t rowoff = (ubase / span) * CP_NAM;
  const uint32_t nsub = (uint32_t)((n - ubase < U ? n - ubase : U) + SL_SUB - 1) / SL_SUB;
  uint8_t* const img = reinterpret_cast<uint8_t*>(keys);
  if (tid == 0) last_byte = src.text[n - 1];
  if (tid < 256) LP[tid] = src.lutp[tid];
  if (tid < 72) SK[tid] = src.skey[tid];
  for (uint32_t i = tid; i < FS_N * CP_NAM / 2; i += T) cnt[i] = 0;
  {   // the unit's text bytes [ubase - 16, ubase + U + 48) by DMA, as k_slice_cpart_reg
    const uint32_t nins = (uint32_t)((U + 64 + 1023) / 1024);
    for (uint32_t i = wv; i < nins; i += T / 64) {
      const uint64_t off = (uint64_t)i * 1024 + lane * 16u;
      if (ubase + off >= 16 && ubase + off <= n + 64)
        __builtin_amdgcn_global_load_lds(src.text + (ubase + off - 16), img + (uint64_t)i * 1024, 16, 0, 0);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const uint64_t lim = n < src.g.s_start ? n : src.g.s_start;
  const int kbits = 2 * src.g.q, dsh = 32 - sl.DB, dA = dsh + sl.sA;
  const uint32_t gdn = fs.gd[fs.ns];
  // the group digit's slice (gd[j] = ~0u past ns)
  auto slice_of = [&](uint32_t d) -> uint32_t {
    return (d >= fs.gd[1] ? 1u : 0u) + (d >= fs.gd[2] ? 1u : 0u) + (d >= fs.gd[3] ? 1u : 0u);
  };
  auto count = [&](uint32_t d) { atomicAdd(&cnt[d >> 1], 1u << (16 * (d & 1u))); };
  // ---- round 1: packed codes, kept positions (bit 2k) and their slices (bits 2k..2k+1), digit counts
  uint32_t c[G][3], mv[G], sid[G], pcs = 0;
#pragma unroll
  for (int st = 0; st < G; ++st) {
    mv[st] = sid[st] = 0;
    c[st][0] = c[st][1] = c[st][2] = 0;
    const uint64_t p0 = ubase + (uint64_t)st * SL_SUB + 16ull * tid;
    if ((uint32_t)st >= nsub || p0 >= n) continue;
    const uint32_t ib = 16u + (uint32_t)st * SL_SUB + 16u * tid;
    const uint4* q4 = reinterpret_cast<const uint4*>(img + ib);
    c[st][0] = pack16_2(q4[0], sl);
    c[st][1] = pack16_2(q4[1], sl);
    c[st][2] = pack16_2(q4[2], sl);
    const uint32_t pb = reinterpret_cast<const uint32_t*>(img + ib)[-1] >> 24;
    const uint32_t pc = p0 ? __builtin_amdgcn_perm(sl.th, sl.tl, (pb >> sl.ps) & 7u) & 3u : (uint32_t)LP[last_byte];
    pcs |= pc << (2 * st);
    const bool full = p0 + 16 <= lim;
    uint32_t m = 0, sd = 0;
#pragma unroll
    for (int k = 0; k < CP_I; ++k) {
      const uint32_t d = (win32(c[st][0], c[st][1], k) >> dA) - fs.gd0;
      if (d < gdn && (full || p0 + k < lim)) {
        m |= 1u << (2 * k);
        sd |= slice_of(d) << (2 * k);
        count(d);
      }
    }
    for (uint64_t j = p0 > lim ? p0 : lim; j < p0 + 16 && j < n; ++j) {   // short suffixes: boundary keys
      const uint32_t d = ((uint32_t)(SK[j - src.g.s_start] >> sl.bsh) >> sl.sA) - fs.gd0;
      if (d < gdn) {
        m |= 1u << (2 * (uint32_t)(j - p0));
        sd |= slice_of(d) << (2 * (uint32_t)(j - p0));
        count(d);
      }
    }
    mv[st] = m;
    sid[st] = sd;
  }
  const int Z = sl.bsh + sl.sA, pz = sl.pb2 + sl.pbits;
  // ---- per slice: scan, reserve, stage, write (k_slice_cpart_reg's fast and dense paths)
  for (int s = 0; s < fs.ns; ++s) {   // uniform
    const uint32_t db = fs.gd[s], nd = fs.gd[s + 1] - db;
    const uint64_t sbase = (uint64_t)fs.base[s] << sl.bsh;
    const uint64_t wS = sbase << (64 - kbits);
    const uint32_t spat = (uint32_t)s * 0x55555555u;
    unsigned long long* const row = fs.cur[s] + rowoff;
    uint64_t* const kout = fs.kout[s];
    const uint64_t mcap = fs.mcap[s];
    auto kept = [&](int st) -> uint32_t {   // bit 2k: position k of sub-tile st is in slice s
      const uint32_t x = sid[st] ^ spat;
      return ~(x | (x >> 1)) & mv[st] & 0x55555555u;
    };
    auto record_at = [&](int st, int k, uint64_t& rec) -> uint32_t {
      const uint64_t j = ubase + (uint64_t)st * SL_SUB + 16ull * tid + (uint64_t)k;
      const int sh = 32 - 2 * k;
      const uint64_t s01 = ((uint64_t)c[st][0] << 32) | c[st][1], s12 = ((uint64_t)c[st][1] << 32) | c[st][2];
      uint64_t wr = (((uint64_t)(uint32_t)(s01 >> sh) << 32) | (uint32_t)(s12 >> sh)) - wS;
      if (j >= src.g.s_start) wr = (SK[j - src.g.s_start] - sbase) << (64 - kbits);
      const uint32_t prv = (uint32_t)(((((uint64_t)((pcs >> (2 * st)) & 3u)) << 32) | c[st][0]) >> sh) & 3u;
      rec = (((wr << (kbits - Z)) >> (64 - Z)) << pz) | ((uint64_t)prv << sl.pbits) | j;
      return (uint32_t)(wr >> (64 - kbits + Z));
    };
    auto rank = [&](uint32_t d) -> uint32_t {   // d: the slice's digit
      const uint32_t x = db + d, sh16 = 16u * (x & 1u);
      return (atomicAdd(&cnt[x >> 1], 1u << sh16) >> sh16) & 0xFFFFu;
    };
    auto clear_mine = [&]() {   // the slice's counters to zero (the other half of a pair is another slice's)
      if (tid < nd) atomicAnd(&cnt[(db + tid) >> 1], ~(0xFFFFu << (16u * ((db + tid) & 1u))));
    };
    auto scan = [&](uint32_t cu, uint32_t& total) {   // tg = exclusive digit starts; total
      const uint32_t inc = wave_incl_sum<uint32_t>(cu);
      if (lane == 63) wsum[wv] = inc;
      __syncthreads();
      uint32_t carry = 0;
      total = 0;
#pragma unroll
      for (uint32_t w = 0; w < T / 64; ++w) {
        carry += w < wv ? wsum[w] : 0u;
        total += wsum[w];
      }
      tg[tid] = carry + inc - cu;
    };
    auto write_out = [&](uint32_t cnt_tile, uint32_t hi256) {
      for (int i = 0; i < FS_CAP / T; ++i) {
        const uint32_t q = (uint32_t)i * T + tid;
        if (q < cnt_tile) {
          const uint32_t d = (uint32_t)sdg[q] | (q >= hi256 ? 256u : 0u);
          const uint32_t o = tg[d] + q;   // u32: tg = destination - tile start (mod 2^32)
          if (o < mcap) kout[o] = keys[q];
        }
      }
    };
    __syncthreads();   // the previous slice's write-out has read keys / sdg / tg
    const uint32_t cu = tid < nd ? (cnt[(db + tid) >> 1] >> (16u * ((db + tid) & 1u))) & 0xFFFFu : 0u;
    uint32_t total;
    scan(cu, total);
    __syncthreads();   // every count read
    clear_mine();
    if (total <= (uint32_t)FS_CAP) {
      const unsigned long long resv = cu ? atomicAdd(&row[tid], (unsigned long long)cu) : 0ull;
      __syncthreads();
#pragma unroll
      for (int st = 0; st < G; ++st) {
        uint32_t m = kept(st);
        while (m) {   // two kept positions a trip: their slot atomics in flight together
          const int k = __builtin_ctz(m) >> 1;
          m &= m - 1;
          const bool two = m != 0;
          const int k2 = two ? __builtin_ctz(m) >> 1 : k;
          m &= m - 1;
          uint64_t rec, rec2;
          const uint32_t d = record_at(st, k, rec);
          const uint32_t d2 = record_at(st, k2, rec2);
          uint32_t f = tg[d] + rank(d);
          uint32_t f2 = two ? tg[d2] + rank(d2) : 0u;
          f = f < (uint32_t)FS_CAP ? f : (uint32_t)FS_CAP - 1;   // (only a count mismatch overruns)
          keys[f] = rec;
          sdg[f] = (uint8_t)d;
          if (two) {
            f2 = f2 < (uint32_t)FS_CAP ? f2 : (uint32_t)FS_CAP - 1;
            keys[f2] = rec2;
            sdg[f2] = (uint8_t)d2;
          }
        }
      }
      __syncthreads();
      const uint32_t hi256 = tg[256];
      const uint32_t gbv = (uint32_t)(resv - tg[tid]);
      __syncthreads();
      tg[tid] = gbv;
      __syncthreads();
      write_out(total, hi256);
      continue;
    }
    // dense unit for this slice: each half sub-tile counted, reserved, staged and written on its own
#pragma unroll
    for (int st = 0; st < G; ++st) {
      if ((uint32_t)st >= nsub) break;   // uniform
#pragma unroll
     for (int part = 0; part < 2; ++part) {
      const uint32_t pm = kept(st) & (part ? 0xFFFF0000u : 0x0000FFFFu);   // positions k >= 8 / k < 8
      __syncthreads();   // the previous write-out has read keys / tg; counters clear
      for (uint32_t m = pm; m; m &= m - 1) {
        uint64_t rec;
        const uint32_t d = record_at(st, __builtin_ctz(m) >> 1, rec);
        atomicAdd(&cnt[(db + d) >> 1], 1u << (16u * ((db + d) & 1u)));
      }
      __syncthreads();
      const uint32_t cc = tid < nd ? (cnt[(db + tid) >> 1] >> (16u * ((db + tid) & 1u))) & 0xFFFFu : 0u;
      const unsigned long long g = cc ? atomicAdd(&row[tid], (unsigned long long)cc) : 0ull;
      uint32_t tot;
      scan(cc, tot);
      __syncthreads();
      clear_mine();
      __syncthreads();
      for (uint32_t m = pm; m; m &= m - 1) {
        uint64_t rec;
        const uint32_t d = record_at(st, __builtin_ctz(m) >> 1, rec);
        const uint32_t f = tg[d] + rank(d);
        keys[f] = rec;
        sdg[f] = (uint8_t)d;
      }
      __syncthreads();
      const uint32_t hi256 = tg[256];
      const uint32_t gbv = (uint32_t)(g - tg[tid]);
      __syncthreads();
      tg[tid] = gbv;
      __syncthreads();
      write_out(tot, hi256);
      __syncthreads();
      clear_mine();
     }
    }
  }
}

// ------------------------------------------------------------ 2. keys
constexpr int PKK_TILE = 4096;
__global__ __launch_bounds__(256) void k_pack_keyed(const uint8_t* __restrict__ t, uint64_t n,
                                                    const uint16_t* __restrict__ lutk,
                                                    const uint16_t* __restrict__ lutp,
                                                    const uint64_t* __restrict__ skey, KeyedArgs g,
                                                    uint64_t* __restrict__ keys) {
  __shared__ uint16_t c[PKK_TILE + kCodePad];
  __shared__ uint16_t L[256], LP[256];
  __shared__ uint64_t SK[72];
  L[threadIdx.x] = lutk[threadIdx.x];
  LP[threadIdx.x] = lutp[threadIdx.x];
  if (threadIdx.x < 72) SK[threadIdx.x] = skey[threadIdx.x];
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * PKK_TILE;
  TextWords<PKK_TILE, 256> tw;
  if ((uint64_t)blockIdx.x * PKK_TILE < n) load_text_words(tw, t, n, (uint64_t)blockIdx.x * PKK_TILE);
  for (uint64_t base = (uint64_t)blockIdx.x * PKK_TILE; base < n; base += stride) {
    store_text_codes(c, L, tw, n, base);
    __syncthreads();
    if (base + stride < n) load_text_words(tw, t, n, base + stride);
#pragma unroll 4
    for (int k = 0; k < PKK_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      const uint64_t p = base + off;
      if (p < n) keys[p] = (keyed_sym(c, off, p, g, SK) << g.pb) | LP[c[off] >> 8];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------ 4. LDS bucket sorts: hk_bsort.hip

// ------------------------------------------------------------ 5. big buckets
// compacted copy of the big buckets: key top D bits replaced by the big-bucket ordinal, J = slot;
// pbits > 0: packed records (key bits << pbits | position, section 1b), no value plane
__global__ __launch_bounds__(256) void k_big_gather(const uint64_t* __restrict__ keys,
                                                    const uint32_t* __restrict__ vals,
                                                    const uint64_t* __restrict__ bstart,
                                                    const uint64_t* __restrict__ cstart, uint32_t nbig,
                                                    uint64_t total, int lowbits, uint64_t* __restrict__ ok,
                                                    uint32_t* __restrict__ ov, uint32_t* __restrict__ oj,
                                                    PkGeom pg) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < total; a += (uint64_t)gridDim.x * 256) {
    uint32_t lo = 0, hi = nbig;   // last g with cstart[g] <= a
    while (hi - lo > 1) {
      const uint32_t mid = (lo + hi) >> 1;
      if (cstart[mid] <= a) lo = mid; else hi = mid;
    }
    const uint64_t src = bstart[lo] + (a - cstart[lo]);
    const uint64_t r = keys[src], k = pg.pbits ? pk_full_low(r, pg) : r;
    ok[a] = ((uint64_t)lo << lowbits) | (lowbits ? (k & ((1ull << lowbits) - 1)) : 0);
    ov[a] = pg.pbits ? (uint32_t)(r & ((1ull << pg.pbits) - 1)) : vals[src];
    oj[a] = (uint32_t)src;
  }
}

// packed records back to (key, position) planes for the paths that take full keys (the LSD item
// sorts, the global path): items[i] = {start, count}; the region (pass A digit) of index j is the last
// r with startA[r] <= j, and the key is region << klw | the record's key bits in the full layout
// uhb > 0 (u64 positions): the position's bits above 32 go below the key (the hb layout of the key
// planes), the low 32 to vout
__global__ __launch_bounds__(256) void k_unpack_items(const uint64_t* __restrict__ rec, const uint2* __restrict__ items,
                                                      uint32_t nitems, const uint64_t* __restrict__ startA,
                                                      uint32_t ndA, PkGeom pg, int klw, uint64_t* __restrict__ kout,
                                                      uint32_t* __restrict__ vout, int uhb = 0) {
  __shared__ uint64_t S[CP_NAM + 1];
  for (uint32_t i = threadIdx.x; i <= ndA; i += 256) S[i] = startA[i];
  __syncthreads();
  const uint64_t pmask = (1ull << pg.pbits) - 1;
  for (uint32_t i = blockIdx.x; i < nitems; i += gridDim.x) {
    const uint2 it = items[i];
    for (uint32_t a = threadIdx.x; a < it.y; a += 256) {
      const uint64_t j = (uint64_t)it.x + a;
      uint32_t lo = 0, hi = ndA;   // S[lo] <= j < S[hi]
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (S[mid] <= j) lo = mid; else hi = mid;
      }
      const uint64_t r = rec[j];
      const uint64_t k = ((uint64_t)lo << klw) | pk_full_low(r, pg);
      kout[j] = uhb ? (k << uhb) | ((r & pmask) >> 32) : k;
      vout[j] = (uint32_t)(r & pmask);
    }
  }
}

// key planes with hb position bits below the key -> u64 SA entries (high bits | low 32) and bare keys
__global__ __launch_bounds__(256) void k_split_join_keys(uint64_t* __restrict__ keys, const uint32_t* __restrict__ lo32,
                                                         uint64_t m, int hb, uint64_t* __restrict__ sa) {
  const uint64_t mask = (1ull << hb) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = keys[i];
    sa[i] = ((k & mask) << 32) | lo32[i];
    keys[i] = k >> hb;
  }
}

// ------------------------------------------------------------ 6. ties
// refine_step's (P, J, G) output of the big path appended to the tie list
__global__ __launch_bounds__(256) void k_tie_append(const uint32_t* __restrict__ P, const uint32_t* __restrict__ J,
                                                    const uint32_t* __restrict__ G, uint64_t A, uint64_t at,
                                                    uint64_t* __restrict__ tie_k, uint32_t* __restrict__ tie_v) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const bool head = a == 0 || G[a] != G[a - 1];
    tie_k[at + a] = ((uint64_t)J[a] << 1) | (head ? 1u : 0u);
    tie_v[at + a] = P[a];
  }
}

template <typename V>
__global__ __launch_bounds__(256) void k_tie_split(const uint64_t* __restrict__ tk, const V* __restrict__ tv,
                                                   uint64_t A, V* __restrict__ P, uint32_t* __restrict__ J,
                                                   uint32_t* __restrict__ H) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint64_t k = tk[a];
    P[a] = tv[a];
    J[a] = (uint32_t)(k >> 1);
    H[a] = (uint32_t)(k & 1u);
  }
}

// G = inclusive head count - 1 (in place over H); head_slot[G] = J of the head
__global__ __launch_bounds__(256) void k_tie_groups(const uint64_t* __restrict__ hx, const uint32_t* __restrict__ J,
                                                    uint64_t A, uint32_t* __restrict__ GH,
                                                    uint32_t* __restrict__ head_slot) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint32_t h = GH[a];
    const uint32_t g = (uint32_t)(hx[a] + h - 1);
    GH[a] = g;
    if (h) head_slot[g] = J[a];
  }
}

inline unsigned grid_of(uint64_t n, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, 256);
  return (unsigned)(g < cap ? g : cap);
}

// bucket = sym >> bsh for m suffixes whose sym fields span `span` values: the largest shift that keeps
// the uniform-model mean bucket at <= 16.5k suffixes (one LDS sort holds 18432), with D = sb - bsh in
// [1, maxD] (bsh = sb, i.e. one bucket, when one sort holds all).  maxD = 16 keeps the LSD passes over
// the bucket bits at two; sharded slices of more than ~1.2G suffixes use up to 18 (a third pass).
int bucket_shift(uint64_t m, int sb, unsigned __int128 span, int maxD = 16) {
  if (m <= (uint64_t)BS_CAP) return sb;
  const double l = std::log2(16500.0 * (double)span / (double)m);
  int b = (int)std::floor(l);
  b = std::min(b, sb - 1);
  b = std::max(b, sb - maxD);
  return std::max(b, 0);
}

int bits_of(unsigned __int128 v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}


// Work items of the LDS bucket sort: consecutive whole buckets packed up to one workgroup's capacity
// (kept narrow — local keys within 32 bits — when the geometry allows), and the buckets too large for
// one workgroup.  hist[b] = suffixes in bucket b, buckets in sorted order.
// (BucketPlan: hk_bucket.hpp)

// split_sh < 32: no item spans two values of bucket >> split_sh (packed records: pass A regions)
BucketPlan plan_buckets(const std::vector<uint64_t>& hist, int bsh, uint64_t cap, int split_sh = 32) {
  BucketPlan pl;
  pl.cap = cap;
  const bool wide_geom = bsh > 32;
  uint64_t off = 0, istart = 0, icnt = 0;
  uint32_t ib0 = 0;
  auto flush = [&](uint32_t last_b) {
    if (!icnt) return;
    const int wb = bsh + (last_b != ib0 ? 32 - __builtin_clz(last_b ^ ib0) : 0);
    (wb > 32 ? pl.items_w : pl.items_n).push_back(make_uint2((uint32_t)istart, (uint32_t)icnt));
    icnt = 0;
  };
  uint32_t prev_b = 0;
  for (uint32_t b = 0; b < (uint32_t)hist.size(); ++b) {
    const uint64_t c = hist[b];
    if (!c) continue;
    if (c > cap) {
      flush(prev_b);
      pl.big_cstart.push_back(pl.big_total);
      pl.big_start.push_back(off);
      pl.big_total += c;
    } else {
      const bool keep_narrow = !wide_geom && icnt && bsh + (32 - __builtin_clz(b ^ ib0)) > 32;
      const bool region = split_sh < 32 && (b >> split_sh) != (ib0 >> split_sh);
      if (icnt && (icnt + c > cap || keep_narrow || region)) flush(prev_b);
      if (!icnt) {
        istart = off;
        ib0 = b;
      }
      icnt += c;
      prev_b = b;
    }
    off += c;
  }
  flush(prev_b);
  return pl;
}

// (PackedRecs: hk_bucket.hpp)

}  // namespace

// (declared in hk_bucket.hpp: the item sorts unpack their fallback items with it)
void unpack_items(Index& ix, const PackedRecs& pk, const uint64_t* rec, const uint2* d_items, uint32_t nitems) {
  if (!nitems) return;
  k_unpack_items<<<std::min<uint32_t>(nitems, 4096), 256, 0, ix.stream>>>(rec, d_items, nitems, pk.startA, pk.ndA,
                                                                         pk.g, pk.klw, pk.kfull, pk.vfull, pk.uhb);
  HK_HIP(hipGetLastError());
}

namespace {

// (sort_bucket_items, the LDS sorts of a plan's work items: hk_bsort.hip)


// starts[b] = first index of bin b in keys sorted by bin = ((key - kbias) >> shift) & (nbins - 1)
// (one lower-bound search per bin); starts[nbins] = m
__global__ __launch_bounds__(256) void k_bin_starts(const uint64_t* __restrict__ keys, uint64_t m, uint64_t kbias,
                                                    int shift, uint32_t nbins, uint64_t* __restrict__ starts) {
  const uint32_t b = blockIdx.x * 256 + threadIdx.x;
  if (b > nbins) return;
  uint64_t lo = 0, hi = m;
  if (b == nbins) lo = m;
  while (lo < hi) {
    const uint64_t mid = lo + (hi - lo) / 2;
    if ((((keys[mid] - kbias) >> shift) & (nbins - 1)) < b) lo = mid + 1;
    else hi = mid;
  }
  starts[b] = lo;
}

}  // namespace

// ---------------------------------------------------------------- geometry
KeyGeom key_geometry_keyed(Index& ix, int reserve, int min_q, int max_sb) {
  compute_alphabet(ix);
  const uint64_t n = ix.n;
  KeyGeom g{};
  g.keyed = true;
  g.R = (uint64_t)ix.sigma + 1;
  // prev field = dense code (no end code in the keyed layout): bits(sigma - 1), at least 1
  int pbits = 1;
  while ((1 << pbits) < ix.sigma) ++pbits;
  g.pb = pbits;
  for (int c = 0; c < 256; ++c) {
    g.lut[c] = ix.code_of[c] < 0 ? 0 : (uint16_t)(ix.code_of[c] + 1);   // refinement: 0 = end of text
    g.lutp[c] = ix.code_of[c] < 0 ? 0 : (uint16_t)ix.code_of[c];
  }
  memset(g.inv, 0, sizeof(g.inv));
  for (int k = 0; k < ix.sigma; ++k) g.inv[k] = ix.syms[k];

  // the last bytes of T' (short suffixes)
  const uint64_t nt = std::min<uint64_t>(n, 70);
  if (!ix.tail_valid) {   // alphabet set without compute_alphabet (sharded all-reduce): read it here
    HK_HIP(hipMemcpyAsync(ix.tail, ix.text.as<uint8_t>() + (n - nt), nt, hipMemcpyDeviceToHost, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));
    ix.tail_valid = true;
  }
  const uint8_t* tail = ix.tail;
  const uint8_t term = tail[nt - 1];
  const bool unkeyed = ix.byte_hist[term] == 1 && ix.sigma >= 2;
  int codek[256];
  int Rk = 0, m_term = 0;
  for (int b = 0; b < 256; ++b) {
    codek[b] = 0;
    if (!ix.byte_hist[b] || (unkeyed && b == term)) continue;
    if (b < term) ++m_term;
    codek[b] = Rk++;
  }
  if (!unkeyed) m_term = 0;
  g.tcode = unkeyed ? (int)g.lutp[term] : -1;
  g.Rk = (uint64_t)std::max(Rk, 2);
  for (int b = 0; b < 256; ++b) g.lutk[b] = (uint16_t)(codek[b] | (b << 8));
  {
    int below = 0;
    for (int b = 0; b < 256; ++b) {
      const bool k = ix.byte_hist[b] && !(unkeyed && b == term);
      g.kdig[b] = (uint16_t)below;
      g.kflag[b] = k ? 1 : 0;
      below += k ? 1 : 0;
    }
    memset(g.k2d, 0, sizeof(g.k2d));
    for (int b = 0; b < 256; ++b)
      if (g.kflag[b]) g.k2d[codek[b]] = g.lutp[b];
  }
  double p2 = 0;
  for (int b = 0; b < 256; ++b)
    if (ix.byte_hist[b] && !(unkeyed && b == term)) {
      const double f = (double)ix.byte_hist[b] / (double)n;
      p2 += f * f;
    }
  // short-suffix keys for a given q; returns the sym bits (or 99 when they do not fit)
  auto shorts = [&](int q, uint64_t* skey, uint64_t& s_start, unsigned __int128* span) -> int {
    unsigned __int128 Rq = 1;
    for (int i = 0; i < q; ++i) {
      Rq *= g.Rk;
      if (Rq > ((unsigned __int128)1 << 64)) return 99;
    }
    const uint64_t back = unkeyed ? (uint64_t)q : (uint64_t)q - 1;
    s_start = n > back ? n - back : 0;
    unsigned __int128 mx = Rq - 1;
    for (uint64_t p = s_start; p < n; ++p) {
      const uint64_t ul = unkeyed ? n - 1 - p : n - p;
      unsigned __int128 v = 0;
      for (uint64_t i = 0; i < ul; ++i) v = v * g.Rk + (unsigned)codek[tail[p + i - (n - nt)]];
      v = v * g.Rk + (unsigned)(unkeyed ? m_term : 0);
      for (uint64_t i = ul + 1; i < (uint64_t)q; ++i) v *= g.Rk;
      if (skey) skey[p - s_start] = (uint64_t)v;
      if (v > mx) mx = v;
    }
    if (span) *span = mx + 1;
    return std::max(1, bits_of(mx));
  };
  auto shift_for = [&](int sb, unsigned __int128 span) { return bucket_shift(n, sb, span); };
  // Symbols per key by cost, in units of one LDS radix pass over all suffixes: the passes over the
  // local (below-bucket) bits, 30% more when they need the wide (two-plane) kernel, plus ~13 per
  // expected tied suffix (refinement: text gathers, a 64-bit sort and a regrouping pass), from the
  // iid collision rate sum(p_c^2)^q of the keyed symbols.
  auto ties = [&](int q) { return std::min((double)n, (double)n * (double)n * std::pow(p2, (double)q)); };
  double best = 1e300;
  for (int q = std::max(1, min_q); q <= 64; ++q) {
    uint64_t ss;
    unsigned __int128 span = 0;
    const int sb = shorts(q, nullptr, ss, &span);
    if (sb == 99 || g.pb + sb + reserve > 64 || sb > max_sb) break;
    const int bs = shift_for(sb, span);
    const double passes = (double)((bs + 7) / 8) * (bs > 32 ? 1.3 : 1.0);
    const double cost = passes + 13.0 * ties(q) / (double)n;
    if (cost <= best) {
      best = cost;
      g.q = q;
      g.sym_bits = sb;
      g.bucket_bits = sb - bs;
    }
  }
  if (g.q == 0) throw ApiError{-6, "keyed geometry: no symbol count fits a 64-bit key"};
  if (ix.flags & kFlagMaxBuckets) g.bucket_bits = std::min(16, g.sym_bits);   // the 1 GiB pipeline at any n
  shorts(g.q, g.skey, g.s_start, nullptr);
  g.nS = (uint32_t)(n - g.s_start);
  // exact order of the short suffixes (bytes compare like Python str over latin-1 code points)
  std::vector<uint64_t> ord(g.nS);
  for (uint32_t i = 0; i < g.nS; ++i) ord[i] = g.s_start + i;
  std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
    const uint8_t* pa = tail + (a - (n - nt));
    const uint8_t* pb2 = tail + (b - (n - nt));
    const uint64_t la = n - a, lb = n - b;
    const int c = memcmp(pa, pb2, std::min(la, lb));
    return c < 0 || (c == 0 && la < lb);
  });
  for (uint32_t r = 0; r < g.nS; ++r) g.srank[ord[r] - g.s_start] = r;
  g.key_bits = g.pb + g.sym_bits;
  return g;
}

// ---------------------------------------------------------------- ties -> refinement
template <typename V>
void refine_from_ties(Index& ix, const KeyGeom& kg, uint64_t A, bool allow_doubling) {
  if (A == 0) return;
  hipStream_t s = ix.stream;
  for (int i = 0; i < 2; ++i) {
    ix.act[i][0].ensure(A * sizeof(V) + 16);
    ix.act[i][1].ensure(A * 4 + 16);
    ix.act[i][2].ensure(A * 4 + 16);
  }
  ix.head_slot.ensure(A * 4 + 16);
  // The list needs no sort by slot: every producer writes runs of whole groups, each group's records
  // consecutive with its head first (the bucket sorts append one item's ties in slot order, the
  // big-bucket path refine_step's grouped output); the groups' order in the list is free.
  uint64_t* const tk = ix.ties_k.as<uint64_t>();
  const V* const tv = ix.ties_v.as<V>();
  V* P = ix.act[0][0].as<V>();
  uint32_t* J = ix.act[0][1].as<uint32_t>();
  uint32_t* GH = ix.act[0][2].as<uint32_t>();
  k_tie_split<V><<<grid_of(A), 256, 0, s>>>(tk, tv, A, P, J, GH);
  HK_HIP(hipGetLastError());
  uint64_t* hx = tk;   // u64 scratch (A + 1): the list is consumed
  scan_exclusive_u32_to_u64(ix.sw, GH, hx, A, true, s);
  k_tie_groups<<<grid_of(A), 256, 0, s>>>(hx, J, A, GH, ix.head_slot.as<uint32_t>());
  HK_HIP(hipGetLastError());
  uint64_t* const hg = ix.rb();
  HK_HIP(hipMemcpyAsync(hg, hx + A, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  const uint64_t groups = hg[0];
  refine_loop<V>(ix, kg, 0, A, groups, allow_doubling);
}

template void refine_from_ties<uint32_t>(Index&, const KeyGeom&, uint64_t, bool);
template void refine_from_ties<uint64_t>(Index&, const KeyGeom&, uint64_t, bool);

// ---------------------------------------------------------------- one sharded slice
SliceBins slice_bins(uint64_t m, const KeyGeom& kg, int hb, uint64_t kmin, uint64_t kmax, bool force_mul) {
  SliceBins b;
  b.kmin = kmin;
  b.kmax = kmax;
  b.binpos = kg.pb + hb + kg.sym_bits;
  const unsigned __int128 span = (unsigned __int128)(kmax - kmin) + 1;
  const int sbl = std::max(1, bits_of((unsigned __int128)(kmax - kmin)));   // bits of the slice's sym range
  b.bsh = bucket_shift(m, sbl, span, 18);
  b.D = sbl - b.bsh;
  if (b.D <= 0) {
    b.D = 0;
    return b;
  }
  // Shift bins cover [kmin, kmin + 2^(bsh+D)): a range just past a power of two wastes half of the
  // 2^16 bins and leaves every bucket over one sort's capacity.  Multiplicative bins (exactly 2^16
  // over the range) need 16 free key bits above the sym field.
  const double mean = (double)m / (double)(((kmax - kmin) >> b.bsh) + 1);
  // multiplicative bins: 2^Dm over the range, Dm = 16 .. 18 (the fewest that keep the mean <= 16.5k)
  int Dm = 16;
  while (Dm < 18 && (double)m / (double)(1u << Dm) > 16500.0) ++Dm;
  // also when the shift bins need more 8-bit passes than Dm multiplicative bins (a 17-bit shift bin
  // over a range just past a power of two costs a whole third pass for one bit)
  const bool fewer_passes = (b.D + 7) / 8 > (Dm + 7) / 8;
  if ((mean > 16500.0 || force_mul || fewer_passes) && b.binpos + Dm <= 64 && span > ((unsigned __int128)1 << Dm)) {
    b.mul = (uint64_t)((((unsigned __int128)1) << (64 + Dm)) / span);   // hi64(x * mul) < 2^Dm for x < span
    b.D = Dm;
    b.bsh = bits_of(span >> Dm) + 1;
  }
  return b;
}

int cursor_partition(Index& ix, uint64_t n, int D, int bitlo, uint64_t kbias, const TextKeySrc* tks, uint64_t* kp[2],
                     uint32_t* vp[2], std::vector<uint64_t>& hist, PackedRecs* pk = nullptr);

// the cursor partition groups buckets wherever D <= 16 (lookback-free; the stable onesweep passes
// remain for texts without whole-symbol buckets)
template <typename V>
bool bucket_sort_slice(Index& ix, const KeyGeom& kg, uint64_t m, int hb, const SliceBins& bins, const uint64_t* d_h0) {
  hipStream_t s = ix.stream;
  const int pb = kg.pb, sb = kg.sym_bits, pbe = pb + hb;
  const int D = bins.D;
  const uint32_t nbins = 1u << D;
  std::vector<uint64_t> hist(nbins, 0);
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  uint32_t* vp[2] = {reinterpret_cast<uint32_t*>(ix.vals[0].p), reinterpret_cast<uint32_t*>(ix.vals[1].p)};
  int slot = 0;
  if (D > 0) {
    // LSD passes over the bin: the bin field above the sym field (mul), or the D bits of
    // (key - kmin << pbe) above bsh
    const uint64_t kbias = bins.mul ? 0 : bins.kmin << pbe;
    const int shift = bins.mul ? bins.binpos : pbe + bins.bsh;
    if (D <= 16) {
      // bin counts from the packed keys, then the two lookback-free cursor passes
      slot = cursor_partition(ix, m, D, shift, kbias, nullptr, kp, vp, hist);
    } else {
      slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, m, shift, shift + D, false, s, d_h0, nullptr,
                                        kbias);
      ix.info[0] += ix.sw.passes_run;
      ix.info[1] += ix.sw.passes_skipped;
      ix.bk_hist.ensure((uint64_t)(nbins + 1) * 8);
      {
        TimedLaunch t(ix.timer, "sa_bin_starts", (double)(nbins + 1) * 8);
        k_bin_starts<<<(nbins + 1 + 255) / 256, 256, 0, s>>>(kp[slot], m, kbias, shift, nbins,
                                                            ix.bk_hist.as<uint64_t>());
        HK_HIP(hipGetLastError());
      }
      std::vector<uint64_t> st(nbins + 1);
      HK_HIP(hipMemcpyAsync(st.data(), ix.bk_hist.p, (uint64_t)(nbins + 1) * 8, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
      for (uint32_t b = 0; b < nbins; ++b) hist[b] = st[b + 1] - st[b];
    }
  } else {
    hist[0] = m;
  }
  const BucketPlan plan = plan_buckets(hist, bins.bsh, BS_CAP);
  ix.info[4] = plan.items_n.size() + plan.items_w.size();
  ix.info[5] = plan.big_start.size();
  ix.info[6] = plan.big_total;
  static const bool dbg = getenv("HKCSA_SHARD_DEBUG") != nullptr;   // diagnostic: slice plan
  if (dbg) {
    uint64_t hmax = 0, nz = 0;
    for (uint64_t c : hist) {
      hmax = std::max(hmax, c);
      nz += c != 0;
    }
    fprintf(stderr, "[slice] m=%llu bsh=%d D=%d mul=%d nonempty=%llu max=%llu narrow=%zu wide=%zu big=%zu\n",
            (unsigned long long)m, bins.bsh, D, bins.mul ? 1 : 0, (unsigned long long)nz,
            (unsigned long long)hmax, plan.items_n.size(), plan.items_w.size(), plan.big_start.size());
  }
  if (plan.big_total) {
    if (slot != 0) {   // the global path starts from keys[0] / vals[0]
      std::swap(ix.keys[0], ix.keys[1]);
      std::swap(ix.vals[0], ix.vals[1]);
    }
    return false;
  }
  ix.bwt.ensure(m + 64);
  const uint64_t ntie = sort_bucket_items<V>(ix, plan, kp[slot], vp[slot], m, pb, sb, hb, bins.kmin,
                                             ix.sa.as<V>(), ix.bwt.as<uint8_t>());
  ix.info.push_back(ntie);
  refine_from_ties<V>(ix, kg, ntie, false);
  return true;
}

template bool bucket_sort_slice<uint32_t>(Index&, const KeyGeom&, uint64_t, int, const SliceBins&,
                                          const uint64_t*);
template bool bucket_sort_slice<uint64_t>(Index&, const KeyGeom&, uint64_t, int, const SliceBins&,
                                          const uint64_t*);

// ---------------------------------------------------------------- cursor partition (host)
// Pass B's region table: the top-digit regions dealt to 8 XCD groups (largest first, to the group with
// the fewest tiles); group g's tiles go to workgroups g, g + 8, ... so that one XCD works through one
// region's cursor row at a time and its L2 merges the runs the row hands out back to back (blocks are
// dealt round-robin over the XCDs: a speed assumption only).  Returns the most tiles of any group.
static uint64_t deal_regions(Index& ix, const uint64_t* totA, uint32_t ndA, uint64_t btile, uint32_t* h_gtab,
                             uint32_t* d_gtab) {
  std::vector<uint32_t> order;
  for (uint32_t d = 0; d < ndA; ++d)
    if (totA[d]) order.push_back(d);
  std::stable_sort(order.begin(), order.end(), [&](uint32_t a, uint32_t b) { return totA[a] > totA[b]; });
  std::vector<std::vector<uint32_t>> grp(8);
  uint64_t load[8] = {0};
  for (uint32_t d : order) {
    const int g = (int)(std::min_element(load, load + 8) - load);
    grp[g].push_back(d);
    load[g] += ceil_div(totA[d], (uint64_t)CP_TILE);
  }
  uint32_t e = 0;
  uint64_t maxl = 0;
  for (int g = 0; g < 8; ++g) {
    h_gtab[g] = e;
    uint32_t k0 = 0;
    for (uint32_t d : grp[g]) {
      h_gtab[9 + 2 * e] = d;
      h_gtab[9 + 2 * e + 1] = k0;
      k0 += (uint32_t)ceil_div(totA[d], btile);
      ++e;
    }
    maxl = std::max<uint64_t>(maxl, k0);
  }
  h_gtab[8] = e;
  HK_HIP(hipMemcpyAsync(d_gtab, h_gtab, (9 + 2 * e) * 4, hipMemcpyHostToDevice, ix.stream));
  return maxl;
}

// Groups n suffixes by bucket (section 1b): pre-pass counts and cursors on the device, pass A
// launched at once; the bucket counts and digit totals come back behind an event while pass A
// runs (the host deals the pass-B regions to XCD groups and the caller plans the bucket items
// meanwhile), then pass B (D > 8).  bucket = ((key - kbias) >> bitlo) & (2^D - 1).  With `tks` the
// keys are built from the text (single GPU); without, they are the packed keys in kp[0] / vp[0]
// (a sharded slice).  Leaves the bucket counts in `hist`; returns the slot holding the grouped pairs.
// pk (pk->pbits > 0, text keys, D = 17): packed records, pass A over the top 9 bucket bits with
// 1024-thread tiles, pass B over the low 8 (k_cpart PK); the records land in kp[0] and pk gets the
// region starts for unpacking.
int cursor_partition(Index& ix, uint64_t n, int D, int bitlo, uint64_t kbias, const TextKeySrc* tks, uint64_t* kp[2],
                     uint32_t* vp[2], std::vector<uint64_t>& hist, PackedRecs* pk) {
  hipStream_t s = ix.stream;
  if (D > 17 || (!tks && D > 16)) throw ApiError{-1, "cursor partition: too many bucket bits"};
  const bool packed = pk && pk->g.pbits > 0;
  // packed: pass A builds the keys with the records' prev field (pb2 bits), so below the bucket
  // there are bitlo2 = bitlo - pb + pb2 bits
  const int bitlo2 = packed ? bitlo - pk->g.pb + pk->g.pb2 : bitlo;
  if (packed && (!tks || D != 17 || kbias || bitlo2 + 8 + pk->g.pbits > 64 || tks->g.pb != pk->g.pb))
    throw ApiError{-1, "cursor partition: packed records need 17 text bucket bits"};
  // pass A digit = bucket >> sA (its top 8 bits, all of it for D <= 8; 9 bits for packed records);
  // pass B digit = the low sA bits
  const int sA = packed ? D - 9 : (D > 16 ? D - 8 : (D > 8 ? 8 : 0));
  const uint32_t nb = 1u << D, ndA = 1u << (D - sA);
  const uint64_t span = ceil_div(ceil_div(n, (uint64_t)BH_TILE), 256) * BH_TILE;   // one workgroup per CU
  const uint32_t nspan = (uint32_t)ceil_div(n, span);
  const uint32_t stride = nb;
  ix.cp_part.ensure((uint64_t)nspan * stride * 4 + (uint64_t)nspan * CP_NAM * 4 + 16);
  ix.bk_hist.ensure((uint64_t)nb * 16 + 16);
  ix.cp_cur.ensure(((uint64_t)nspan * CP_NAM + nb + 2 * (CP_NAM + 1) + 16 + (uint64_t)CP_NG * CP_NAM) * 8);
  constexpr uint64_t kLp2Off = (9 + 2 * CP_NAM + 16) * 4;   // packed: the records' prev-code table
  ix.cp_tiles.ensure(kLp2Off + 512);
  ix.cp_host.ensure((uint64_t)nb * 8 + 2 * (CP_NAM + 1) * 8 + (9 + 2 * CP_NAM) * 4 + 64);
  uint32_t* d_part = ix.cp_part.as<uint32_t>();
  uint32_t* d_spanc = d_part + (uint64_t)nspan * stride;
  unsigned long long* d_drain = ix.bk_hist.as<unsigned long long>();
  uint64_t* d_hist = ix.bk_hist.as<uint64_t>() + nb;
  unsigned long long* d_curA = ix.cp_cur.as<unsigned long long>();
  unsigned long long* d_curB = d_curA + (uint64_t)nspan * CP_NAM;
  uint64_t* d_totA = reinterpret_cast<uint64_t*>(d_curB + nb);
  uint64_t* d_startA = d_totA + (CP_NAM + 1);
  uint32_t* d_gtab = ix.cp_tiles.as<uint32_t>();
  uint64_t* h_hist = ix.cp_host.as<uint64_t>();
  uint64_t* h_totA = h_hist + nb;   // totA[CP_NAM + 1] then startA[CP_NAM + 1]
  uint32_t* h_gtab = reinterpret_cast<uint32_t*>(h_totA + 2 * (CP_NAM + 1) + 1);   // after the overflow flag
  unsigned long long* d_ovf = reinterpret_cast<unsigned long long*>(d_totA + 2 * (CP_NAM + 1));
  uint64_t* d_gpre = d_totA + 2 * (CP_NAM + 1) + 16;   // [CP_NG][CP_NAM] span-group prefixes
  const uint64_t* h_ovf = h_totA + 2 * (CP_NAM + 1);
  TextKeySrc tks2{};
  if (packed) {
    pk->startA = d_startA;
    pk->ndA = ndA;
    pk->klw = bitlo + sA;
    uint16_t* d_lp2 = reinterpret_cast<uint16_t*>(ix.cp_tiles.as<uint8_t>() + kLp2Off);
    HK_HIP(hipMemcpyAsync(d_lp2, pk->lutp2, 512, hipMemcpyHostToDevice, s));   // pk outlives the stream's use
    tks2 = *tks;
    tks2.lutp = d_lp2;
    tks2.g.pb = pk->g.pb2;
  }
  // pre-pass (exact: 2^17 buckets as two u16 runs over the bucket halves, after a u8 overflow)
  // pre-pass with the code width and window fixed at compile time where they are 2 bits x 9 / 8 bits x 3
  auto prepass = [&](bool exact) {
    HK_HIP(hipMemsetAsync(d_drain, 0, (uint64_t)nb * 16, s));   // drain, then hist (bucket_reduce adds)
    HK_HIP(hipMemsetAsync(d_ovf, 0, 8, s));
    TimedLaunch t(ix.timer, "sa_bucket_hist", (double)n * (tks ? (exact ? 2 : 1) : 8));
    if (tks && D > 16 && !exact) {   // 2^17 buckets: u8 counters (drained at 128)
      const int lbk = 31 - __builtin_clz((uint32_t)tks->g.Rk);
      if (packed && pk->reg) {   // register scan, undrained u8 counters (checked; exact recount on a wrap)
        k_slice_hist_spans<8, -1, 2, 0, true, true><<<nspan, BH_T, 0, s>>>(tks->text, n, tks->lutk, tks->skey, tks->g,
                                                                     pk->rsl, D, d_part, d_drain, d_spanc, span,
                                                                     d_ovf);
      } else {
        auto kern = k_bucket_hist_spans<8>;
        if (lbk == 2 && tks->g.hq == 9) kern = k_bucket_hist_spans<8, -1, 2, 9>;
        else if (lbk == 8 && tks->g.hq == 3) kern = k_bucket_hist_spans<8, -1, 8, 3>;
        kern<<<nspan, BH_T, 0, s>>>(tks->text, n, tks->lutk, tks->skey, tks->g, bitlo - tks->g.pb, D, sA, d_part,
                                    d_drain, d_spanc, span, d_ovf);
      }
    } else if (tks) {
      if (D > 16) {
        k_bucket_hist_spans<16, 0><<<nspan, BH_T, 0, s>>>(tks->text, n, tks->lutk, tks->skey, tks->g,
                                                          bitlo - tks->g.pb, D, sA, d_part, d_drain, d_spanc, span,
                                                          d_ovf);
        k_bucket_hist_spans<16, 1><<<nspan, BH_T, 0, s>>>(tks->text, n, tks->lutk, tks->skey, tks->g,
                                                          bitlo - tks->g.pb, D, sA, d_part, d_drain, d_spanc, span,
                                                          d_ovf);
      } else {
        k_bucket_hist_spans<16><<<nspan, BH_T, 0, s>>>(tks->text, n, tks->lutk, tks->skey, tks->g, bitlo - tks->g.pb,
                                                       D, sA, d_part, d_drain, d_spanc, span, d_ovf);
      }
    } else {
      k_key_hist_spans<<<nspan, BH_T, 0, s>>>(kp[0], n, bitlo, kbias, D, sA, d_part, d_drain, d_spanc, span);
    }
    HK_HIP(hipGetLastError());
    bucket_reduce(d_part, d_drain, nspan, stride, nb, d_hist, s);
    HK_HIP(hipGetLastError());
    const uint32_t nblkA = (ndA + CP_DB - 1) / CP_DB;
    k_cp_colsum<<<nblkA, 1024, 0, s>>>(d_spanc, nspan, ndA, d_gpre, d_totA);
    HK_HIP(hipGetLastError());
    k_cp_cursors<<<nblkA, 1024, 0, s>>>(d_hist, d_spanc, d_gpre, nspan, nb, ndA, d_curA,
                                                          D > 8 ? d_curB : nullptr, d_totA, d_startA);
    HK_HIP(hipGetLastError());
  };
  // pass A: text -> slot D > 8 ? 1 : 0; packed keys: slot 0 -> 1.  A text pass skips itself when the
  // pre-pass flagged an overflow
  const int outA = tks ? (D > 8 ? 1 : 0) : 1;
  auto passA = [&]() {
    TimedLaunch t(ix.timer, tks ? "radix_part_text" : "radix_part_keys",
                  (double)n * (packed ? 1 + 8 : tks ? 1 + 8 + 4 : 2 * (8 + 4)));
    const unsigned grid = (unsigned)(8 * ceil_div(nspan, 8u) * (span / CP_TILE));
    // packed: 512-thread tiles, two workgroups per CU; radix 2^2: 16 consecutive positions per thread
    if (packed && tks->g.lb == 2)
      k_cpart<0, 2, 512, CP_T, true><<<grid, CP_T, 0, s>>>(nullptr, nullptr, kp[outA], nullptr, n, bitlo2 + sA, 0,
                                                          d_curA, nullptr, nullptr, span, tks2, pk->g.pbits, d_ovf);
    else if (packed)
      k_cpart<0, 0, 512, CP_T, true><<<grid, CP_T, 0, s>>>(nullptr, nullptr, kp[outA], nullptr, n, bitlo2 + sA, 0,
                                                          d_curA, nullptr, nullptr, span, tks2, pk->g.pbits, d_ovf);
    else if (!tks)
      k_cpart<1, 0><<<grid, CP_T, 0, s>>>(kp[0], vp[0], kp[1], vp[1], n, bitlo + sA, kbias, d_curA, nullptr, nullptr,
                                          span, TextKeySrc{});
    else if (tks->g.lb == 2)
      k_cpart<0, 2><<<grid, CP_T, 0, s>>>(nullptr, nullptr, kp[outA], vp[outA], n, bitlo + sA, 0, d_curA, nullptr,
                                          nullptr, span, *tks, 0, d_ovf);
    else
      k_cpart<0, 0><<<grid, CP_T, 0, s>>>(nullptr, nullptr, kp[outA], vp[outA], n, bitlo + sA, 0, d_curA, nullptr,
                                          nullptr, span, *tks, 0, d_ovf);
    HK_HIP(hipGetLastError());
    ix.info[0] += 1;
  };
  // the counts come back on the auxiliary stream while pass A runs (pass A does not wait for the
  // copies; the host waits for them alone)
  if (!ix.aux_stream) HK_HIP(hipStreamCreateWithFlags(&ix.aux_stream, hipStreamNonBlocking));
  auto counts_then_passA = [&]() {
    ScopedEvent ev_pre, ev_cnt;
    HK_HIP(hipEventRecord(ev_pre, s));
    HK_HIP(hipStreamWaitEvent(ix.aux_stream, ev_pre, 0));
    HK_HIP(hipMemcpyAsync(h_hist, d_hist, (uint64_t)nb * 8, hipMemcpyDeviceToHost, ix.aux_stream));
    HK_HIP(hipMemcpyAsync(h_totA, d_totA, (2 * (CP_NAM + 1) + 1) * 8, hipMemcpyDeviceToHost, ix.aux_stream));
    HK_HIP(hipEventRecord(ev_cnt, ix.aux_stream));
    passA();
    const hipError_t we = hipEventSynchronize(ev_cnt);   // the counts, not pass A
    HK_HIP(we);
  };
  prepass(false);
  counts_then_passA();
  if (*h_ovf) {   // u8 counters overflowed (long runs of one bucket): exact recount, pass A again
    ix.info[0] -= 1;
    prepass(true);
    counts_then_passA();
    if (*h_ovf) throw ApiError{-7, "cursor partition: exact recount flagged an overflow"};
  }
  hist.assign(h_hist, h_hist + nb);
  const uint64_t* totA = h_totA;
  uint64_t tsum = 0, hsum = 0;
  for (uint32_t d = 0; d < ndA; ++d) tsum += totA[d];
  for (uint32_t b = 0; b < nb; ++b) hsum += hist[b];
  if (tsum != n || hsum != n) throw ApiError{-7, "cursor partition: bucket counts do not cover the text"};
  if (D > 8) {
    // 9-bit digits: 1024-thread tiles (twice the run length per digit)
    const uint64_t btile = sA > 8 ? 1024 * CP_I : CP_TILE;
    const uint64_t maxl = deal_regions(ix, totA, ndA, btile, h_gtab, d_gtab);
    TimedLaunch t(ix.timer, "radix_part", (double)n * 2 * (packed ? 8 : 8 + 4));
    if (packed)
      k_cpart<2, 0, 256, CP_T, true, true, true><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(
          kp[1], nullptr, kp[0], nullptr, n, bitlo2 + pk->g.pbits, 0, d_curB, d_gtab, d_startA, 0, TextKeySrc{},
          pk->g.pbits);
    else if (sA > 8 && btile > CP_TILE)
      k_cpart<2, 0, 512, 1024><<<(unsigned)(8 * maxl), 1024, 0, s>>>(kp[1], vp[1], kp[0], vp[0], n, bitlo, kbias,
                                                                      d_curB, d_gtab, d_startA, 0, TextKeySrc{});
    else if (sA > 8)
      k_cpart<2, 0, 512><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(kp[1], vp[1], kp[0], vp[0], n, bitlo, kbias, d_curB,
                                                              d_gtab, d_startA, 0, TextKeySrc{});
    else
      k_cpart<2, 0><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(kp[1], vp[1], kp[0], vp[0], n, bitlo, kbias, d_curB, d_gtab,
                                                         d_startA, 0, TextKeySrc{});
    HK_HIP(hipGetLastError());
    ix.info[0] += 1;
    return 0;
  }
  return outA;
}

// ---------------------------------------------------------------- sharded slices, keyed scheme (host)
namespace {

// Exact histogram of the coarse keyed bucket (the top 16 bits of the sym field: the first 16 / lb
// symbols, radix 2^lb) of the positions [lo, hi) (lo a multiple of 16): one span per workgroup, u16
// counter pairs drained at 2^15 (bh_add), per-span partials reduced by k_bucket_reduce.
__global__ __launch_bounds__(BH_T, 1) void k_coarse_hist(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                         uint64_t hi, const uint16_t* __restrict__ lutk,
                                                         const uint64_t* __restrict__ skey, KeyedArgs g, int hq,
                                                         int bsh16, uint64_t span, uint32_t* __restrict__ part,
                                                         unsigned long long* __restrict__ drain,
                                                         const unsigned long long* __restrict__ only_if = nullptr) {
  __shared__ uint32_t H[32768];
  __shared__ uint16_t L[256];
  __shared__ uint64_t SK[72];
  const uint32_t tid = threadIdx.x;
  if (only_if && !*only_if) return;   // the register count did not wrap: nothing to recount
  for (uint32_t i = tid; i < 32768; i += BH_T) H[i] = 0;
  if (tid < 256) L[tid] = lutk[tid];
  if (tid < 72) SK[tid] = skey[tid];
  __syncthreads();
  const uint64_t a = lo + (uint64_t)blockIdx.x * span;
  const uint64_t b = a + span < hi ? a + span : hi;
  const uint64_t lim = n < g.s_start ? n : g.s_start;
  const int lb = 31 - __clz((uint32_t)g.Rk);
  for (uint64_t base = a; base < b; base += BH_TILE) {
    const uint64_t p0 = base + (uint64_t)tid * BH_PER;
    if (p0 >= b) continue;
    const uint4* src = reinterpret_cast<const uint4*>(t + p0);   // T' has 64 readable pad bytes
    const uint4 w0 = src[0], w1 = src[1];
    const uint32_t wd[8] = {w0.x, w0.y, w0.z, w0.w, w1.x, w1.y, w1.z, w1.w};
    const uint64_t lim2 = lim < b ? lim : b;
    if (p0 < lim2) {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 2 * BH_PER - 1; ++i) {
        w = (w << lb) | (L[(wd[i >> 2] >> (8 * (i & 3))) & 255u] & 255u);
        const int j = i - (hq - 1);
        if (j >= 0 && j < BH_PER && p0 + j < lim2) bh_add(H, w & 0xFFFFu, drain);
      }
    }
    for (uint64_t p = p0 > lim ? p0 : lim; p < p0 + BH_PER && p < b; ++p)
      bh_add(H, (uint32_t)(SK[p - g.s_start] >> bsh16), drain);
  }
  __syncthreads();
  uint2* const pw = reinterpret_cast<uint2*>(part + (uint64_t)blockIdx.x * 65536);
  for (uint32_t i = tid; i < 32768; i += BH_T) {
    const uint32_t v = H[i];
    pw[i] = make_uint2(v & 0xFFFFu, v >> 16);
  }
}

int coarse_lb(const KeyGeom& kg) {
  const uint64_t R = kg.Rk;
  if (R != 2 && R != 4 && R != 16 && R != 256) return 0;
  return __builtin_ctzll(R);
}

}  // namespace

// lb of the keyed coarse scheme (whole-symbol keyed radix 2^lb, lb in {1, 2, 4, 8}), 0 when it does not apply
int shard_keyed_lb(Index& ix) {
  const KeyGeom kg = key_geometry_keyed(ix);
  return coarse_lb(kg);
}

static bool reg_tables(const KeyGeom& kk, SliceSel& sl);

void shard_coarse_hist(Index& ix, uint64_t lo, uint64_t hi, uint64_t* d_hist) {
  hipStream_t s = ix.stream;
  const KeyGeom kg0 = key_geometry_keyed(ix);
  const int lb = coarse_lb(kg0);
  if (!lb) throw ApiError{-1, "keyed coarse histogram: alphabet without a whole-symbol keyed radix"};
  const KeyGeom kg = key_geometry_keyed(ix, 0, 16 / lb);   // q >= 16 / lb: the coarse bucket is q-independent
  upload_geometry(ix, kg);
  const uint8_t* small = ix.small.as<uint8_t>();
  const KeyChunks kch = key_chunks(kg.Rk, kg.q);
  const KeyedArgs ka{kg.Rk, kch.Rck, kch.Rlast, kg.s_start, kg.q, kch.ck, kg.pb, 0, lb};
  HK_HIP(hipMemsetAsync(d_hist, 0, 65536 * 8, s));
  if (hi <= lo) return;
  if (lo % 16) throw ApiError{-1, "coarse histogram: block start not 16-aligned"};
  ix.bk_hist.ensure(65536 * 8 + 16);
  unsigned long long* d_drain = ix.bk_hist.as<unsigned long long>();
  HK_HIP(hipMemsetAsync(d_drain, 0, 65536 * 8, s));
  TimedLaunch t(ix.timer, "shard_hist", (double)(hi - lo));
  // radix 2^2 with a 3-bit byte field separating the keyed bytes: the register pre-pass of the slices
  // (k_slice_hist_spans REG, the whole sym space as one slice of 2^16 bins: the 16-bit window's top
  // bits) over 4 MiB spans of the block with undrained u8 counters; a wrap raises the flag and the
  // exact u16 count below runs in its place (device-side: it returns at once when the flag is clear).
  SliceSel rs;
  const unsigned long long* only_if = nullptr;
  if (lb == 2 && lo <= kg.s_start && reg_tables(kg, rs)) {
    rs.base = 0;
    rs.nb = 65536;
    rs.DB = 16;
    rs.bsh = kg.sym_bits - 16;
    rs.sA = 7;
    rs.wb = 0;
    rs.wn1 = ~0u;
    KeyedArgs kr = ka;
    kr.s_start = kg.s_start - lo;   // positions relative to the block (the windows read on past its end)
    const uint64_t rspan = (uint64_t)1 << 22;
    const uint32_t rn = (uint32_t)ceil_div(hi - lo, rspan);
    // (one allocation for both counts: the exact count's partials follow the flag word)
    const uint64_t span = ceil_div(ceil_div(hi - lo, (uint64_t)BH_TILE), 256) * BH_TILE;
    ix.cp_part.ensure(((uint64_t)rn * (65536 + CP_NAM) + 16 + ceil_div(hi - lo, span) * 65536) * 4 + 16);
    uint32_t* d_part = ix.cp_part.as<uint32_t>();
    unsigned long long* d_ovf = reinterpret_cast<unsigned long long*>(d_part + (uint64_t)rn * (65536 + CP_NAM));
    HK_HIP(hipMemsetAsync(d_ovf, 0, 8, s));
    k_slice_hist_spans<8, -1, 2, 0, true, true><<<rn, BH_T, 0, s>>>(
        ix.text.as<uint8_t>() + lo, hi - lo, reinterpret_cast<const uint16_t*>(small + 2560),
        reinterpret_cast<const uint64_t*>(small + 3584), kr, rs, 16, d_part, d_drain, d_part + (uint64_t)rn * 65536,
        rspan, d_ovf);
    HK_HIP(hipGetLastError());
    k_bucket_reduce<<<65536 / 256, 256, 0, s>>>(d_part, d_drain, rn, 65536, 65536, d_hist);
    HK_HIP(hipGetLastError());
    HK_HIP(hipMemsetAsync(d_drain, 0, 65536 * 8, s));
    only_if = d_ovf;
  }
  const uint64_t span = ceil_div(ceil_div(hi - lo, (uint64_t)BH_TILE), 256) * BH_TILE;
  const uint32_t nspan = (uint32_t)ceil_div(hi - lo, span);
  // (the exact count's partials after the register count's flag word)
  const uint64_t poff = only_if ? (uint64_t)ceil_div(hi - lo, (uint64_t)1 << 22) * (65536 + CP_NAM) + 16 : 0;
  ix.cp_part.ensure((poff + (uint64_t)nspan * 65536) * 4 + 16);
  uint32_t* const xpart = ix.cp_part.as<uint32_t>() + poff;
  k_coarse_hist<<<nspan, BH_T, 0, s>>>(ix.text.as<uint8_t>(), ix.n, lo, hi,
                                       reinterpret_cast<const uint16_t*>(small + 2560),
                                       reinterpret_cast<const uint64_t*>(small + 3584), ka, 16 / lb, kg.sym_bits - 16,
                                       span, xpart, d_drain, only_if);
  HK_HIP(hipGetLastError());
  k_bucket_reduce<<<65536 / 256, 256, 0, s>>>(xpart, d_drain, nspan, 65536, 65536, d_hist, only_if);
  HK_HIP(hipGetLastError());
}

namespace {

struct SlicePlan {
  KeyGeom kk;
  SliceSel sl;
  int D = 0, lb = 0, pb = 0, hb = 0;   // hb: key planes' position-high bits (u64 SA)
  bool packed = false;
  bool reg = false;   // radix 2^2 packed records with a perm-table byte field: the register kernels
  bool half = false;  // register pass A with half staging (three workgroups per CU; slices of <= 1/6 of T')
  bool quarter = false;   // ... quarter staging (four per CU; slices of <= 1/7.5 of T')
  PkGeom pg;
  int uhb = 0;
};

}  // namespace

// Register-scan tables (radix 2^2 keyed codes): the 3-bit field (b >> ps) & 7 of a byte that separates
// the keyed bytes indexes an 8-entry table of their codes; false when no field separates them
static bool reg_tables(const KeyGeom& kk, SliceSel& sl) {
  for (int ps = 0; ps <= 5; ++ps) {
    uint8_t tab[8] = {0};
    bool used[8] = {false}, ok = true;
    for (int b = 0; b < 256 && ok; ++b) {
      if (!kk.kflag[b]) continue;
      const int idx = (b >> ps) & 7;
      ok = !used[idx];
      used[idx] = true;
      tab[idx] = (uint8_t)kk.kdig[b];
    }
    if (!ok) continue;
    sl.ps = ps;
    sl.tl = (uint32_t)tab[0] | (uint32_t)tab[1] << 8 | (uint32_t)tab[2] << 16 | (uint32_t)tab[3] << 24;
    sl.th = (uint32_t)tab[4] | (uint32_t)tab[5] << 8 | (uint32_t)tab[6] << 16 | (uint32_t)tab[7] << 24;
    return true;
  }
  return false;
}

namespace {

// Geometry of the slice of coarse buckets [c_lo, c_hi): f = the most extra bin bits with at most 2^17
// bins (k << f) and a pre-pass window of <= 16 symbols; packed records when the bits below the pass A
// digit, the prev code and the position fit one u64 (q capped for that), else key / value planes.
SlicePlan plan_slice(Index& ix, uint32_t c_lo, uint32_t c_hi, bool u64pos) {
  SlicePlan P;
  const KeyGeom kg0 = key_geometry_keyed(ix);
  P.lb = coarse_lb(kg0);
  if (!P.lb) throw ApiError{-1, "slice plan: no whole-symbol keyed radix"};
  const int lb = P.lb;
  const uint64_t n = ix.n;
  const int pbits = n > 1 ? 64 - __builtin_clzll(n - 1) : 1;
  P.hb = 0;
  if (u64pos) {
    P.hb = 1;
    while (((n - 1) >> 32) >> P.hb) ++P.hb;
  }
  const uint32_t k = c_hi - c_lo;
  auto geom_f = [&](int sb, int& f) {   // the pre-pass window: <= 16 symbols of <= 32 bits
    f = 0;
    while ((uint64_t)k << (f + 1) <= (1u << 17) && 16 + f + 1 <= sb) {
      const int hq = (16 + f + 1 + lb - 1) / lb;
      if (hq > 16 || hq * lb > 32) break;
      ++f;
    }
  };
  int pb2 = kg0.pb;
  if (kg0.tcode >= 0) {
    pb2 = 1;
    while ((1ull << pb2) < kg0.Rk) ++pb2;
    pb2 = std::min(pb2, kg0.pb);
  }
  // the fallback key planes of packed records keep >= 1 position bit below the key for a u64 SA
  const int uhb = u64pos ? std::max(1, pbits - 32) : 0;
  bool packed = true;
  KeyGeom kk;
  int f = 0;
  if (packed) {
    // bsh + 8 + pb2 + pbits <= 64 with bsh = sb - (16 + f): sb <= 56 - pb2 - pbits + 16 + f
    kk = key_geometry_keyed(ix, uhb, 16 / lb);
    for (int it = 0; it < 4 && packed; ++it) {
      geom_f(kk.sym_bits, f);
      const int bound = 56 - pb2 - pbits + 16 + f;
      if (kk.sym_bits <= bound) break;
      if (bound < 16 + f || bound < lb * (16 / lb)) {
        packed = false;
        break;
      }
      kk = key_geometry_keyed(ix, uhb, 16 / lb, bound);
    }
    if (packed) {
      geom_f(kk.sym_bits, f);
      if (kk.sym_bits - (16 + f) + 8 + pb2 + pbits > 64) packed = false;
    }
  }
  if (!packed) {
    kk = key_geometry_keyed(ix, P.hb, 16 / lb);
    geom_f(kk.sym_bits, f);
  }
  P.kk = kk;
  P.packed = packed;
  P.pb = kk.pb;
  SliceSel& sl = P.sl;
  sl.DB = 16 + f;
  sl.bsh = kk.sym_bits - sl.DB;
  sl.base = c_lo << f;
  sl.nb = k << f;
  sl.hq = (sl.DB + lb - 1) / lb;
  sl.wdrop = sl.hq * lb - sl.DB;
  sl.wb = sl.base << (32 - sl.DB);
  sl.wn1 = (uint32_t)(((uint64_t)sl.nb << (32 - sl.DB)) - 1);
  P.D = 1;
  while ((1u << P.D) < sl.nb) ++P.D;
  sl.sA = P.D > 8 ? 8 : 0;
  if (packed) {
    sl.pbits = pbits;
    sl.pb2 = pb2;
    P.pg.pbits = pbits;
    P.pg.pb = kk.pb;
    P.pg.pb2 = pb2;
    P.pg.tcode = pb2 < kk.pb ? kk.tcode : -1;
    P.pg.phb = std::max(0, pbits - 32);
    P.uhb = uhb;
  } else {
    sl.pbe = kk.pb + P.hb;
  }
  // register kernels (radix 2^2, packed): a 3-bit field of the byte that separates the keyed bytes
  // indexes an 8-entry table of their codes (every byte the scans key is keyed: the unkeyed terminal
  // only ends short suffixes, which take their boundary keys)
  if (packed && lb == 2) P.reg = reg_tables(kk, sl);
  return P;
}

}  // namespace

// one slice's pre-pass outputs (drain and hist contiguous: one memset clears both)
struct SliceCur {
  unsigned long long* drain;
  uint64_t* hist;
  unsigned long long* curA;
  unsigned long long* curB;   // nullptr: no pass B (sA = 0)
  uint64_t* totA;
  uint64_t* startA;
  unsigned long long* ovf;
  uint64_t* gpre;
};

// The slice's pre-pass over the whole text: its bin counts and per-span pass A digit counts (the span
// counters and digit sums in d_part / d_spanc, consumed here), then both passes' cursors.  A u8
// counter wrap raises *c.ovf (the caller clears it): the exact recount runs with `exact`.
static void slice_prepass(Index& ix, const SlicePlan& P, const TextKeySrc& tks, uint64_t span, uint32_t nspan,
                          uint32_t* d_part, uint32_t* d_spanc, const SliceCur& c, bool exact) {
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  const SliceSel& sl = P.sl;
  const int D = P.D, sA = sl.sA;
  const uint32_t nb2 = 1u << D, ndA = 1u << (D - sA);
  HK_HIP(hipMemsetAsync(c.drain, 0, (uint64_t)nb2 * 16, s));   // drain, then hist (bucket_reduce adds)
  TimedLaunch t(ix.timer, "shard_slice_hist", (double)n * (exact ? 2 : 1));
  const KeyedArgs& g = tks.g;
  const bool reg = P.reg;
  if (D > 16 && !exact) {
    auto kern = k_slice_hist_spans<8>;
    if (reg) kern = k_slice_hist_spans<8, -1, 2, 0, true>;
    else if (P.lb == 2 && sl.hq == 9) kern = k_slice_hist_spans<8, -1, 2, 9>;
    else if (P.lb == 2 && sl.hq == 10) kern = k_slice_hist_spans<8, -1, 2, 10>;
    kern<<<nspan, BH_T, 0, s>>>(tks.text, n, tks.lutk, tks.skey, g, sl, D, d_part, c.drain, d_spanc, span, c.ovf);
  } else if (D > 16) {
    auto k0 = reg ? k_slice_hist_spans<16, 0, 2, 0, true> : k_slice_hist_spans<16, 0>;
    auto k1 = reg ? k_slice_hist_spans<16, 1, 2, 0, true> : k_slice_hist_spans<16, 1>;
    k0<<<nspan, BH_T, 0, s>>>(tks.text, n, tks.lutk, tks.skey, g, sl, D, d_part, c.drain, d_spanc, span, c.ovf);
    k1<<<nspan, BH_T, 0, s>>>(tks.text, n, tks.lutk, tks.skey, g, sl, D, d_part, c.drain, d_spanc, span, c.ovf);
  } else {
    auto kern = k_slice_hist_spans<16>;
    if (reg) kern = k_slice_hist_spans<16, -1, 2, 0, true>;
    else if (P.lb == 2 && sl.hq == 9) kern = k_slice_hist_spans<16, -1, 2, 9>;
    else if (P.lb == 2 && sl.hq == 10) kern = k_slice_hist_spans<16, -1, 2, 10>;
    kern<<<nspan, BH_T, 0, s>>>(tks.text, n, tks.lutk, tks.skey, g, sl, D, d_part, c.drain, d_spanc, span, c.ovf);
  }
  HK_HIP(hipGetLastError());
  bucket_reduce(d_part, c.drain, nspan, nb2, nb2, c.hist, s);
  const uint32_t nblkA = (ndA + CP_DB - 1) / CP_DB;
  k_cp_colsum<<<nblkA, 1024, 0, s>>>(d_spanc, nspan, ndA, c.gpre, c.totA);
  HK_HIP(hipGetLastError());
  k_cp_cursors<<<nblkA, 1024, 0, s>>>(c.hist, d_spanc, c.gpre, nspan, nb2, ndA, c.curA, c.curB, c.totA, c.startA);
  HK_HIP(hipGetLastError());
}

// The slice's cursor partition (section 1c): pre-pass over the whole text counting the slice's bins
// (and its units' pass A digits), cursors, fused pass A from the text, pass B.  Records / key planes
// end in slot 0 (D > 8) or 1; hist gets the bin counts.
static int cursor_partition_slice(Index& ix, const SlicePlan& P, const TextKeySrc& tks, uint64_t m, uint64_t* kp[2],
                                  uint32_t* vp[2], std::vector<uint64_t>& hist, PackedRecs& pkr) {
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  const SliceSel& sl = P.sl;
  const int D = P.D, sA = sl.sA;
  const uint32_t nb2 = 1u << D, ndA = 1u << (D - sA);
  const uint64_t U = (uint64_t)SL_SUB * sl.g;
  const uint64_t Lq = sl.g % 2 ? 2 * U : U;   // lcm(BH_TILE, U)
  const uint64_t span = ceil_div(ceil_div(n, Lq), 256) * Lq;
  const uint32_t nspan = (uint32_t)ceil_div(n, span);
  ix.cp_part.ensure((uint64_t)nspan * nb2 * 4 + (uint64_t)nspan * CP_NAM * 4 + 16);
  ix.bk_hist.ensure((uint64_t)nb2 * 16 + 16);
  ix.cp_cur.ensure(((uint64_t)nspan * CP_NAM + nb2 + 2 * (CP_NAM + 1) + 16 + (uint64_t)CP_NG * CP_NAM) * 8);
  constexpr uint64_t kLp2Off = (9 + 2 * CP_NAM + 16) * 4;
  ix.cp_tiles.ensure(kLp2Off + 512);
  ix.cp_host.ensure((uint64_t)nb2 * 8 + 2 * (CP_NAM + 1) * 8 + (9 + 2 * CP_NAM) * 4 + 64);
  uint32_t* d_part = ix.cp_part.as<uint32_t>();
  uint32_t* d_spanc = d_part + (uint64_t)nspan * nb2;
  unsigned long long* d_drain = ix.bk_hist.as<unsigned long long>();
  uint64_t* d_hist = ix.bk_hist.as<uint64_t>() + nb2;
  unsigned long long* d_curA = ix.cp_cur.as<unsigned long long>();
  unsigned long long* d_curB = d_curA + (uint64_t)nspan * CP_NAM;
  uint64_t* d_totA = reinterpret_cast<uint64_t*>(d_curB + nb2);
  uint64_t* d_startA = d_totA + (CP_NAM + 1);
  unsigned long long* d_ovf = reinterpret_cast<unsigned long long*>(d_totA + 2 * (CP_NAM + 1));
  uint64_t* d_gpre = d_totA + 2 * (CP_NAM + 1) + 16;
  uint32_t* d_gtab = ix.cp_tiles.as<uint32_t>();
  uint64_t* h_hist = ix.cp_host.as<uint64_t>();
  uint64_t* h_totA = h_hist + nb2;
  uint32_t* h_gtab = reinterpret_cast<uint32_t*>(h_totA + 2 * (CP_NAM + 1) + 1);
  const uint64_t* h_ovf = h_totA + 2 * (CP_NAM + 1);
  TextKeySrc tks2 = tks;
  if (P.packed) {
    uint16_t* d_lp2 = reinterpret_cast<uint16_t*>(ix.cp_tiles.as<uint8_t>() + kLp2Off);
    HK_HIP(hipMemcpyAsync(d_lp2, pkr.lutp2, 512, hipMemcpyHostToDevice, s));
    tks2.lutp = d_lp2;
    tks2.g.pb = P.pg.pb2;
    pkr.startA = d_startA;
    pkr.ndA = ndA;
    pkr.klw = P.pb + sl.bsh + sA;
  }
  const SliceCur cur{d_drain, d_hist, d_curA, sA ? d_curB : nullptr, d_totA, d_startA, d_ovf, d_gpre};
  auto prepass = [&](bool exact) {
    HK_HIP(hipMemsetAsync(d_ovf, 0, 8, s));
    slice_prepass(ix, P, tks, span, nspan, d_part, d_spanc, cur, exact);
  };
  const int outA = sA ? 1 : 0;
  auto passA = [&]() {
    TimedLaunch t(ix.timer, "shard_slice_part", (double)n + (double)m * (P.packed ? 8 : 8 + 4));
    const unsigned grid = (unsigned)(8 * ceil_div(nspan, 8u) * (span / U));
    void* vo = P.packed ? nullptr : (void*)vp[outA];
    const unsigned long long* skip = D > 16 ? d_ovf : nullptr;
    const bool trace = getenv("HKCSA_SL_TRACE") != nullptr;   // diagnostic phase stamps (identical results, tested)
    if (P.reg) {
      if (trace) {
        DevBuf tb;
        tb.ensure((uint64_t)grid * 64 + 64);
        HK_HIP(hipMemsetAsync(tb.p, 0, (uint64_t)grid * 64, s));
        if (P.quarter)
          k_slice_cpart_reg<true, 3, SL_CAPQ><<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m,
                                                                   tb.as<uint64_t>());
        else if (P.half)
          k_slice_cpart_reg<true, 4, CP_TILE / 2><<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m,
                                                                       tb.as<uint64_t>());
        else
          k_slice_cpart_reg<true><<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m, tb.as<uint64_t>());
        std::vector<uint64_t> h((uint64_t)grid * 8);
        HK_HIP(hipMemcpyAsync(h.data(), tb.p, h.size() * 8, hipMemcpyDeviceToHost, s));
        HK_HIP(hipStreamSynchronize(s));
        double acc[4] = {0, 0, 0, 0};
        uint64_t nw = 0;
        for (uint64_t w = 0; w < grid; ++w)
          if (h[w * 8 + 5]) {
            ++nw;
            for (int i = 0; i < 4; ++i) acc[i] += (double)(h[w * 8 + i + 1] - h[w * 8 + i]);
          }
        if (nw)
          fprintf(stderr, "[slice_cpart_reg trace] %llu units, mean cycles: round 1 %.0f, count+reserve %.0f, "
                  "round 2 %.0f, write %.0f\n", (unsigned long long)nw, acc[0] / nw, acc[1] / nw, acc[2] / nw, acc[3] / nw);
      } else {
        if (P.quarter)
          k_slice_cpart_reg<false, 3, SL_CAPQ><<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m);
        else if (P.half)
          k_slice_cpart_reg<false, 4, CP_TILE / 2><<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m);
        else
          k_slice_cpart_reg<<<grid, CP_T, 0, s>>>(kp[outA], n, d_curA, span, tks2, sl, skip, m);
      }
    }
    else if (P.packed && P.lb == 2)
      k_slice_cpart<2, true><<<grid, CP_T, 0, s>>>(kp[outA], nullptr, n, d_curA, span, tks2, sl, skip, m);
    else if (P.packed && P.lb == 1)
      k_slice_cpart<1, true><<<grid, CP_T, 0, s>>>(kp[outA], nullptr, n, d_curA, span, tks2, sl, skip, m);
    else if (P.packed && P.lb == 4)
      k_slice_cpart<4, true><<<grid, CP_T, 0, s>>>(kp[outA], nullptr, n, d_curA, span, tks2, sl, skip, m);
    else if (P.packed)
      k_slice_cpart<8, true><<<grid, CP_T, 0, s>>>(kp[outA], nullptr, n, d_curA, span, tks2, sl, skip, m);
    else if (P.lb == 1)
      k_slice_cpart<1, false><<<grid, CP_T, 0, s>>>(kp[outA], (uint32_t*)vo, n, d_curA, span, tks2, sl, skip, m);
    else if (P.lb == 2)
      k_slice_cpart<2, false><<<grid, CP_T, 0, s>>>(kp[outA], (uint32_t*)vo, n, d_curA, span, tks2, sl, skip, m);
    else if (P.lb == 4)
      k_slice_cpart<4, false><<<grid, CP_T, 0, s>>>(kp[outA], (uint32_t*)vo, n, d_curA, span, tks2, sl, skip, m);
    else
      k_slice_cpart<8, false><<<grid, CP_T, 0, s>>>(kp[outA], (uint32_t*)vo, n, d_curA, span, tks2, sl, skip, m);
    HK_HIP(hipGetLastError());
    ix.info[0] += 1;
  };
  if (!ix.aux_stream) HK_HIP(hipStreamCreateWithFlags(&ix.aux_stream, hipStreamNonBlocking));
  auto counts_then_passA = [&]() {
    ScopedEvent ev_pre, ev_cnt;
    HK_HIP(hipEventRecord(ev_pre, s));
    HK_HIP(hipStreamWaitEvent(ix.aux_stream, ev_pre, 0));
    HK_HIP(hipMemcpyAsync(h_hist, d_hist, (uint64_t)nb2 * 8, hipMemcpyDeviceToHost, ix.aux_stream));
    HK_HIP(hipMemcpyAsync(h_totA, d_totA, (2 * (CP_NAM + 1) + 1) * 8, hipMemcpyDeviceToHost, ix.aux_stream));
    HK_HIP(hipEventRecord(ev_cnt, ix.aux_stream));
    passA();
    const hipError_t we = hipEventSynchronize(ev_cnt);
    HK_HIP(we);
  };
  prepass(false);
  counts_then_passA();
  if (D > 16 && *h_ovf) {   // u8 counters overflowed: exact recount, pass A again
    ix.info[0] -= 1;
    if (ix.info.size() > 7) ix.info[7] |= 8;
    prepass(true);
    counts_then_passA();
  }
  hist.assign(h_hist, h_hist + nb2);
  uint64_t tsum = 0, hsum = 0;
  for (uint32_t d = 0; d < ndA; ++d) tsum += h_totA[d];
  for (uint32_t b = 0; b < nb2; ++b) hsum += hist[b];
  if (tsum != m || hsum != m) throw ApiError{-7, "slice partition: bin counts do not match the slice size"};
  if (!sA) return outA;
  const uint64_t maxl = deal_regions(ix, h_totA, ndA, CP_TILE, h_gtab, d_gtab);
  TimedLaunch t(ix.timer, "radix_part", (double)m * 2 * (P.packed ? 8 : 8 + 4));
  if (P.packed)
    k_cpart<2, 0, 256, CP_T, true, true, true><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(
        kp[1], nullptr, kp[0], nullptr, m, P.pg.pbits + P.pg.pb2 + sl.bsh, 0, d_curB, d_gtab, d_startA, 0,
        TextKeySrc{}, P.pg.pbits);
  else
    k_cpart<2, 0><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(kp[1], vp[1], kp[0], vp[0], m, sl.pbe + sl.bsh, 0, d_curB,
                                                       d_gtab, d_startA, 0, TextKeySrc{});
  HK_HIP(hipGetLastError());
  ix.info[0] += 1;
  return 0;
}

// ---------------------------------------------------------------- fused pass A of single-GPU slices
// build_sa_slices runs the slices of a text one after another; each slice's pass A (k_slice_cpart_reg)
// keys all of T' to keep ~1/k of it.  For up to FS_N slices with one geometry (same bin width, radix
// 2^2 packed records, first bins on pass A digit boundaries) the pre-passes run first, each into its
// own cursor set, then k_slice_cpart_fused keys T' once and scatters every suffix into its slice's
// records; each slice later takes its pass B from them (fused_pass_b).
struct FusedSlice {
  uint32_t c_lo = 0, c_hi = 0;
  uint64_t m = 0;
  SlicePlan P;
  uint64_t* kA = nullptr;                // pass A records, grouped by the slice's digit
  unsigned long long* curB = nullptr;    // pass B cursors (bucket starts)
  uint64_t* startA = nullptr;            // digit starts (pass B regions)
  std::vector<uint64_t> hist, totA;      // bin counts, digit totals
};
struct FusedState {   // (its buffers are the handle's fused_recs / fused_ws / fused_host)
  std::vector<FusedSlice> sl;
};

static TextKeySrc slice_tks(Index& ix, const KeyGeom& kk, int lb) {
  const uint8_t* small = ix.small.as<uint8_t>();
  const KeyChunks kch = key_chunks(kk.Rk, kk.q);
  KeyedArgs ka{kk.Rk, kch.Rck, kch.Rlast, kk.s_start, kk.q, kch.ck, kk.pb, 0, lb};
  return TextKeySrc{ix.text.as<uint8_t>(), ix.n, reinterpret_cast<const uint16_t*>(small + 2560),
                    reinterpret_cast<const uint16_t*>(small + 4608), reinterpret_cast<const uint64_t*>(small + 3584),
                    ka};
}

static void prev_code_table(const KeyGeom& kk, const PkGeom& pg, uint16_t* lutp2) {
  for (int b = 0; b < 256; ++b) lutp2[b] = pg.tcode < 0 ? kk.lutp[b] : (kk.kflag[b] ? kk.kdig[b] : 0);
}

static FusedSlice* fused_slice(Index& ix, uint32_t c_lo, uint32_t c_hi) {
  if (!ix.fused) return nullptr;
  for (FusedSlice& f : static_cast<FusedState*>(ix.fused.get())->sl)
    if (f.c_lo == c_lo && f.c_hi == c_hi) return &f;
  return nullptr;
}

bool slices_fuse(Index& ix, const std::vector<uint32_t>& B, const std::vector<uint64_t>& below, int r0, int r1,
                 bool u64pos) {
  ix.fused.reset();   // (the previous group's records)
  const int ns = r1 - r0;
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  if (ns < 2 || ns > FS_N || getenv("HKCSA_SL_TRACE")) return false;   // (the trace stamps the per-slice kernel)
  auto st = std::make_shared<FusedState>();
  st->sl.resize(ns);
  uint64_t mmax = 0, msum = 0;
  for (int i = 0; i < ns; ++i) {
    FusedSlice& f = st->sl[i];
    f.c_lo = B[r0 + i];
    f.c_hi = B[r0 + i + 1];
    f.m = below[r0 + i + 1] - below[r0 + i];
    if (!f.m) return false;
    f.P = plan_slice(ix, f.c_lo, f.c_hi, u64pos);
    const SlicePlan& P = f.P;
    if (!P.packed || !P.reg || P.lb != 2 || P.sl.sA != 8 || P.D <= 8 || P.sl.base % 256 || P.sl.nb % 256) return false;
    if (i) {
      const SlicePlan& Q = st->sl[0].P;
      const SliceSel &a = P.sl, &b = Q.sl;
      if (P.kk.q != Q.kk.q || P.kk.sym_bits != Q.kk.sym_bits || P.kk.pb != Q.kk.pb || P.kk.s_start != Q.kk.s_start ||
          P.kk.tcode != Q.kk.tcode || P.pb != Q.pb || P.uhb != Q.uhb || a.DB != b.DB || a.bsh != b.bsh ||
          a.hq != b.hq || a.wdrop != b.wdrop || a.pbits != b.pbits || a.pb2 != b.pb2 || a.tl != b.tl ||
          a.th != b.th || a.ps != b.ps || P.pg.pbits != Q.pg.pbits || P.pg.pb2 != Q.pg.pb2 ||
          P.pg.tcode != Q.pg.tcode || P.pg.phb != Q.pg.phb)
        return false;
      if (a.base != st->sl[i - 1].P.sl.base + st->sl[i - 1].P.sl.nb) return false;   // contiguous
    }
    mmax = std::max(mmax, f.m);
    msum += f.m;
  }
  // one unit size for the group (the spans, hence the cursor rows, are shared)
  uint32_t g = (uint32_t)std::floor(0.9 * (double)n / (double)mmax);
  // at most 4 sub-tiles per unit: the 8-sub-tile form holds 8 x 3 code words and masks and spilled 24 B/lane
  // at 128 VGPRs (only texts of 6+ slices reach g > 4)
  g = std::max<uint32_t>(1, std::min<uint32_t>(g, 4u));
  for (FusedSlice& f : st->sl) f.P.sl.g = g;
  const uint64_t U = (uint64_t)SL_SUB * g;
  const uint64_t Lq = g % 2 ? 2 * U : U;
  const uint64_t span = ceil_div(ceil_div(n, Lq), 256) * Lq;
  const uint32_t nspan = (uint32_t)ceil_div(n, span);
  // cursor sets: drain, hist [nb2 each], curA [nspan][CP_NAM], curB [nb2], totA, startA [CP_NAM + 1], gpre
  auto set_words = [&](const SlicePlan& P) -> uint64_t {
    const uint64_t nb2 = 1ull << P.D;
    return 3 * nb2 + (uint64_t)nspan * CP_NAM + 2 * (CP_NAM + 1) + (uint64_t)CP_NG * CP_NAM + 16;
  };
  uint64_t wsw = 16, hw = 16;
  for (const FusedSlice& f : st->sl) {
    wsw += set_words(f.P);
    hw += (1ull << f.P.D) + 2 * (CP_NAM + 1);
  }
  // memory: the group's records next to one slice's workspace (keys / values planes, bucket items)
  {
    size_t fr = 0, tot = 0;
    HK_HIP(hipMemGetInfo(&fr, &tot));
    const uint64_t held = ix.fused_recs.bytes + ix.fused_ws.bytes;   // (reused, or freed by a regrowth)
    const uint64_t need = msum * 8 + wsw * 8 + mmax * 40 + (1ull << 30);
    if ((double)need > 0.9 * (double)(fr + held)) return false;
  }
  const SlicePlan& P0 = st->sl[0].P;
  upload_geometry(ix, P0.kk);
  TextKeySrc tks = slice_tks(ix, P0.kk, P0.lb);
  uint32_t maxnb2 = 0;
  for (const FusedSlice& f : st->sl) maxnb2 = std::max(maxnb2, 1u << f.P.D);
  ix.cp_part.ensure((uint64_t)nspan * maxnb2 * 4 + (uint64_t)nspan * CP_NAM * 4 + 16);
  uint32_t* d_part = ix.cp_part.as<uint32_t>();
  uint32_t* d_spanc = d_part + (uint64_t)nspan * maxnb2;
  ix.fused_ws.ensure(wsw * 8);
  ix.fused_host.ensure(hw * 8 + 64);
  uint64_t* w = ix.fused_ws.as<uint64_t>();
  unsigned long long* d_ovf = reinterpret_cast<unsigned long long*>(w);
  HK_HIP(hipMemsetAsync(d_ovf, 0, 8, s));
  w += 16;
  std::vector<SliceCur> cur(ns);
  for (int i = 0; i < ns; ++i) {
    const SlicePlan& P = st->sl[i].P;
    const uint64_t nb2 = 1ull << P.D;
    SliceCur& c = cur[i];
    c.drain = reinterpret_cast<unsigned long long*>(w);
    c.hist = w + nb2;
    c.curA = reinterpret_cast<unsigned long long*>(w + 2 * nb2);
    c.curB = c.curA + (uint64_t)nspan * CP_NAM;
    c.totA = reinterpret_cast<uint64_t*>(c.curB + nb2);
    c.startA = c.totA + (CP_NAM + 1);
    c.gpre = c.startA + (CP_NAM + 1);
    c.ovf = d_ovf;
    w += set_words(P);
    st->sl[i].curB = c.curB;
    st->sl[i].startA = c.startA;
    slice_prepass(ix, P, tks, span, nspan, d_part, d_spanc, c, false);
  }
  // counts back behind an event while pass A runs
  uint64_t* h = ix.fused_host.as<uint64_t>();
  std::vector<uint64_t*> h_hist(ns), h_tot(ns);
  ScopedEvent ev_pre, ev_cnt;
  if (!ix.aux_stream) HK_HIP(hipStreamCreateWithFlags(&ix.aux_stream, hipStreamNonBlocking));
  HK_HIP(hipEventRecord(ev_pre, s));
  HK_HIP(hipStreamWaitEvent(ix.aux_stream, ev_pre, 0));
  for (int i = 0; i < ns; ++i) {
    const uint64_t nb2 = 1ull << st->sl[i].P.D;
    h_hist[i] = h;
    h_tot[i] = h + nb2;
    h += nb2 + 2 * (CP_NAM + 1);
    HK_HIP(hipMemcpyAsync(h_hist[i], cur[i].hist, nb2 * 8, hipMemcpyDeviceToHost, ix.aux_stream));
    HK_HIP(hipMemcpyAsync(h_tot[i], cur[i].totA, (CP_NAM + 1) * 8, hipMemcpyDeviceToHost, ix.aux_stream));
  }
  uint64_t* h_ovf = h;
  HK_HIP(hipMemcpyAsync(h_ovf, d_ovf, 8, hipMemcpyDeviceToHost, ix.aux_stream));
  HK_HIP(hipEventRecord(ev_cnt, ix.aux_stream));
  // pass A of the group
  ix.fused_recs.ensure(msum * 8 + 16);
  FusedSel fs{};
  fs.ns = ns;
  fs.gd0 = P0.sl.base >> 8;
  uint64_t off = 0;
  for (int i = 0; i < ns; ++i) {
    FusedSlice& f = st->sl[i];
    f.kA = ix.fused_recs.as<uint64_t>() + off;
    off += f.m;
    fs.kout[i] = f.kA;
    fs.cur[i] = cur[i].curA;
    fs.mcap[i] = f.m;
    fs.base[i] = f.P.sl.base;
    fs.gd[i] = (f.P.sl.base >> 8) - fs.gd0;
  }
  fs.gd[ns] = ((st->sl[ns - 1].P.sl.base + st->sl[ns - 1].P.sl.nb) >> 8) - fs.gd0;
  for (int i = ns + 1; i <= FS_N; ++i) fs.gd[i] = ~0u;
  for (int i = ns; i < FS_N; ++i) {
    fs.kout[i] = nullptr;
    fs.cur[i] = nullptr;
  }
  constexpr uint64_t kLp2Off = (9 + 2 * CP_NAM + 16) * 4;   // (cursor_partition_slice's table slot)
  ix.cp_tiles.ensure(kLp2Off + 512);
  ix.cp_host.ensure(512 + 64);
  uint16_t* h_lp2 = ix.cp_host.as<uint16_t>();
  prev_code_table(P0.kk, P0.pg, h_lp2);
  uint16_t* d_lp2 = reinterpret_cast<uint16_t*>(ix.cp_tiles.as<uint8_t>() + kLp2Off);
  HK_HIP(hipMemcpyAsync(d_lp2, h_lp2, 512, hipMemcpyHostToDevice, s));
  TextKeySrc tks2 = tks;
  tks2.lutp = d_lp2;
  tks2.g.pb = P0.pg.pb2;
  {
    TimedLaunch t(ix.timer, "shard_slice_part", (double)n + (double)msum * 8);
    const unsigned grid = (unsigned)(8 * ceil_div(nspan, 8u) * (span / U));
    k_slice_cpart_fused<4><<<grid, CP_T, 0, s>>>(n, span, tks2, P0.sl, fs, d_ovf);
    HK_HIP(hipGetLastError());
  }
  const hipError_t we = hipEventSynchronize(ev_cnt);
  HK_HIP(we);
  HK_HIP(hipStreamSynchronize(s));   // (h_lp2 lives in cp_host, which the slices reuse)
  if (*h_ovf) return false;   // a u8 counter wrapped: the slices run one by one (exact recounts)
  for (int i = 0; i < ns; ++i) {
    FusedSlice& f = st->sl[i];
    const uint32_t nb2 = 1u << f.P.D, ndA = 1u << (f.P.D - 8);
    f.hist.assign(h_hist[i], h_hist[i] + nb2);
    f.totA.assign(h_tot[i], h_tot[i] + ndA);
    uint64_t tsum = 0, hsum = 0;
    for (uint64_t x : f.totA) tsum += x;
    for (uint64_t x : f.hist) hsum += x;
    if (tsum != f.m || hsum != f.m) throw ApiError{-7, "fused slices: bin counts do not match the slice size"};
  }
  ix.fused = st;
  return true;
}

// pass B of a fused slice (its pass A ran in slices_fuse): records land in kp[0]
static int fused_pass_b(Index& ix, FusedSlice& f, uint64_t m, uint64_t* kp[2], std::vector<uint64_t>& hist,
                        PackedRecs& pkr) {
  hipStream_t s = ix.stream;
  const SlicePlan& P = f.P;
  const SliceSel& sl = P.sl;
  const uint32_t ndA = 1u << (P.D - sl.sA);
  pkr.startA = f.startA;
  pkr.ndA = ndA;
  pkr.klw = P.pb + sl.bsh + sl.sA;
  hist = f.hist;
  ix.info[0] += 1;
  ix.cp_tiles.ensure((9 + 2 * CP_NAM + 16) * 4 + 512);
  ix.cp_host.ensure((9 + 2 * CP_NAM) * 4 + 64);
  uint32_t* d_gtab = ix.cp_tiles.as<uint32_t>();
  uint32_t* h_gtab = ix.cp_host.as<uint32_t>();
  const uint64_t maxl = deal_regions(ix, f.totA.data(), ndA, CP_TILE, h_gtab, d_gtab);
  TimedLaunch t(ix.timer, "radix_part", (double)m * 2 * 8);
  k_cpart<2, 0, 256, CP_T, true, true, true><<<(unsigned)(8 * maxl), CP_T, 0, s>>>(
      f.kA, nullptr, kp[0], nullptr, m, P.pg.pbits + P.pg.pb2 + sl.bsh, 0, f.curB, d_gtab, f.startA, 0,
      TextKeySrc{}, P.pg.pbits);
  HK_HIP(hipGetLastError());
  ix.info[0] += 1;
  return 0;
}

// One sharded slice under the keyed coarse scheme: the coarse buckets [c_lo, c_hi), m suffixes.
template <typename V>
void build_slice_keyed(Index& ix, uint32_t c_lo, uint32_t c_hi, uint64_t m) {
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  FusedSlice* const fz = fused_slice(ix, c_lo, c_hi);
  if (fz && fz->m != m) throw ApiError{-7, "fused slice: size mismatch"};
  SlicePlan P = fz ? fz->P : plan_slice(ix, c_lo, c_hi, sizeof(V) == 8);
  const KeyGeom& kk = P.kk;
  upload_geometry(ix, kk);
  ix.info[3] = (uint64_t)kk.q;
  ix.info[7] |= 4 | (P.packed ? 2 : 0);
  // units: ~0.9 of the slice density per sub-tile keeps the kept suffixes of a unit within one tile
  {
    const double ratio = m ? (double)n / (double)m : 1.0;
    uint32_t g = (uint32_t)std::floor(0.9 * ratio);
    if (g < 1) g = 1;
    if (g > (P.reg ? (uint32_t)SL_G : 64u)) g = P.reg ? (uint32_t)SL_G : 64u;   // register kernel: <= SL_G
    // a slice of <= 1/6 of the text (N >= 6 ranks): half staging, units of <= 4 sub-tiles keeping ~0.45 of
    // a full tile, so three workgroups share a CU
    if (P.reg && ratio >= 7.5) {
      P.quarter = true;
      g = std::min<uint32_t>(3, (uint32_t)std::floor(0.42 * ratio));   // ~3072 of 3584 records at N = 8
    } else if (P.reg && ratio >= 6.0) {
      P.half = true;
      g = std::min<uint32_t>(4, (uint32_t)std::floor(0.45 * ratio));
    }
    P.sl.g = g;
  }
  const TextKeySrc tks = slice_tks(ix, kk, P.lb);
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(m * 8 + 16);
    ix.vals[i].ensure(m * sizeof(V) + 16);   // u32 here; the tie refinement sorts V values in them
  }
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  uint32_t* vp[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
  PackedRecs pkr;
  if (P.packed) {
    pkr.g = P.pg;
    prev_code_table(kk, pkr.g, pkr.lutp2);
    pkr.kfull = kp[1];
    pkr.vfull = vp[1];
    pkr.uhb = P.uhb;
  }
  std::vector<uint64_t> hist;
  const int slot = fz ? fused_pass_b(ix, *fz, m, kp, hist, pkr) : cursor_partition_slice(ix, P, tks, m, kp, vp, hist, pkr);
  const int sbx = P.sl.bsh + P.D;   // bits of the slice-relative sym field
  const int lhb = P.packed ? P.uhb : P.hb;
  uint64_t hmax = 0;
  for (uint64_t c : hist) hmax = std::max(hmax, c);
  const uint64_t cap = hmax <= (uint64_t)BR_CAP ? (uint64_t)BR_CAP : (uint64_t)BS_CAP;
  const BucketPlan plan = plan_buckets(hist, P.sl.bsh, cap, P.packed ? P.sl.sA : 32);
  ix.info[4] = plan.items_n.size() + plan.items_w.size();
  ix.info[5] = plan.big_start.size();
  ix.info[6] = plan.big_total;
  static const bool dbg = getenv("HKCSA_SHARD_DEBUG") != nullptr;
  if (dbg)
    fprintf(stderr, "[slice-k] m=%llu q=%d sb=%d f=%d bsh=%d D=%d nb=%u g=%u packed=%d pbits=%d hmax=%llu items=%zu big=%zu recount=%d\n",
            (unsigned long long)m, kk.q, kk.sym_bits, P.sl.DB - 16, P.sl.bsh, P.D, P.sl.nb, P.sl.g, P.packed ? 1 : 0,
            P.sl.pbits, (unsigned long long)hmax, plan.items_n.size() + plan.items_w.size(), plan.big_start.size(),
            (int)(ix.info[7] >> 3 & 1));
  ix.bwt.ensure(m + 64);
  if (!plan.big_total && !(ix.flags & kFlagGlobalSort)) {
    const uint64_t ntie = sort_bucket_items<V>(ix, plan, kp[slot], vp[slot], m, P.pb, sbx, P.packed ? 0 : P.hb, 0,
                                               ix.sa.as<V>(), ix.bwt.as<uint8_t>(), P.packed ? &pkr : nullptr);
    ix.info.push_back(ntie);
    refine_from_ties<V>(ix, kk, ntie, false);
    return;
  }
  // big buckets (skewed text) or HKCSA_FLAG_GLOBAL_SORT: full LSD sort of the slice's keys
  ix.info[7] |= 1;
  int ks = slot;
  if (P.packed) {   // key planes first (slot 1; each record's region found in the pass A starts)
    std::vector<uint2> ch;
    for (uint64_t a = 0; a < m; a += 65536)
      ch.push_back(make_uint2((uint32_t)a, (uint32_t)std::min<uint64_t>(65536, m - a)));
    if (!ch.empty()) {
      ix.bk_items.ensure(ch.size() * sizeof(uint2) + 16);
      HK_HIP(hipMemcpyAsync(ix.bk_items.p, ch.data(), ch.size() * sizeof(uint2), hipMemcpyHostToDevice, s));
      unpack_items(ix, pkr, kp[slot], ix.bk_items.as<uint2>(), (uint32_t)ch.size());
    }
    HK_HIP(hipStreamSynchronize(s));   // ch is freed at the end of this block
    ks = 1;
  }
  const int pbe = P.pb + lhb;
  if (lhb) {
    const int sl2 = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, ks, m, pbe, pbe + sbx, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    TimedLaunch t(ix.timer, "shard_split_join", (double)m * (8 + 4 + 8 + 8));
    k_split_join_keys<<<grid_of(m), 256, 0, s>>>(kp[sl2], vp[sl2], m, lhb, ix.sa.as<uint64_t>());
    HK_HIP(hipGetLastError());
    refine_after_sort<V>(ix, kk, sl2, m, false);
  } else {
    V* vq[2] = {reinterpret_cast<V*>(vp[0]), reinterpret_cast<V*>(vp[1])};
    if (sizeof(V) == 8) throw ApiError{-1, "slice: u64 positions need split position bits"};
    const int sl2 = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vq, ks, m, P.pb, P.pb + sbx, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    std::swap(ix.sa, ix.vals[sl2]);
    ix.vals[sl2].ensure(m * sizeof(V) + 16);
    refine_after_sort<V>(ix, kk, sl2, m, false);
  }
}

template void build_slice_keyed<uint32_t>(Index&, uint32_t, uint32_t, uint64_t);
template void build_slice_keyed<uint64_t>(Index&, uint32_t, uint32_t, uint64_t);

// ---------------------------------------------------------------- driver
void build_sa_bucketed(Index& ix) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  if (n >= 0xFFFFFFFFull) throw ApiError{-6, "single-GPU build supports n < 2^32 - 1"};
  ix.have_alpha = false;   // every build recomputes the byte histogram / C (utils/utils.py:16-24)
  compute_alphabet(ix);
  ix.info.assign(9, 0);
  ix.dbl = Index::DblState{};
  ix.sharded = false;
  ix.sa_pos64 = false;
  ix.have_sa = ix.have_bwt = ix.have_wt = false;
  ix.sa.ensure(n * 4 + 16);
  ix.bwt.ensure(n + 64);
  if (n <= 1) {
    HK_HIP(hipMemsetAsync(ix.sa.p, 0, 4, s));
    HK_HIP(hipMemcpyAsync(ix.bwt.p, ix.text.p, n, hipMemcpyDeviceToDevice, s));
    HK_HIP(hipStreamSynchronize(s));
    ix.have_sa = ix.have_bwt = true;
    return;
  }
  const KeyGeom kg = key_geometry_keyed(ix);
  upload_geometry(ix, kg);
  ix.info[3] = (uint64_t)kg.q;
  int D = kg.bucket_bits;
  const int sb = kg.sym_bits, pb = kg.pb;
  const uint8_t* small = ix.small.as<uint8_t>();
  const uint16_t* d_lutp = reinterpret_cast<const uint16_t*>(small + 4608);
  const uint16_t* d_lutk = reinterpret_cast<const uint16_t*>(small + 2560);
  const uint64_t* d_skey = reinterpret_cast<const uint64_t*>(small + 3584);
  const KeyChunks kch = key_chunks(kg.Rk, kg.q);
  KeyedArgs ka{kg.Rk, kch.Rck, kch.Rlast, kg.s_start, kg.q, kch.ck, kg.pb, 0};
  // half items: one more bucket bit and 9216-suffix items sorted by 512-thread workgroups, two per
  // CU (the cursor pre-pass takes ceil((D + 1) / lb) symbols and drops the excess low bits)
  int item_T = 1024;
  {
    // first hq symbols are exactly the top D bits when Rk = 2^k, k | D and no short key exceeds Rk^q - 1
    const int lb = (kg.Rk & (kg.Rk - 1)) == 0 ? __builtin_ctzll(kg.Rk) : 0;
    const bool whole = lb && sb == lb * kg.q;
    const int hq1 = lb ? (D + 1 + lb - 1) / lb : 0;
    if (whole && D > 0 && D + 1 <= 17 && D + 1 <= sb && hq1 * lb <= 32 && hq1 <= 16) {
      D += 1;
      ka.hq = hq1;
      item_T = 512;
    } else if (whole && D > 0 && D % lb == 0) {
      ka.hq = D / lb;
    }
    // packed bit windows need whole codes per 32-bit word: lb in {1, 2, 4, 8}
    if (lb && 32 % lb == 0 && whole) ka.lb = lb;
  }
  const int bsh = sb - D;

  // ---- 1. bucket histogram.  Radix 2^k with whole-symbol buckets: only the first LSD pass's digit
  // histogram is taken from the text now; the bucket counts come from the sorted keys after the
  // passes (bin starts by binary search), which saves the 64K-bin histogram pass.
  const uint32_t nbins = 1u << D;
  std::vector<uint64_t> hist(nbins, 0);
  uint64_t* d_h0 = reinterpret_cast<uint64_t*>(ix.small.as<uint8_t>() + 5120);
  // whole-symbol buckets: the lookback-free cursor partition; otherwise the stable onesweep passes with
  // the late bucket histogram
  const bool use_cp = D > 0 && ka.hq > 0 && D <= 17;
  const bool late_hist = D > 0 && ka.hq > 0 && !use_cp;
  bool skip_plan = false;   // a sample of the bucket counts already says: the global path
  if (use_cp) {
    // counted with the partition below
  } else if (late_hist) {
    HK_HIP(hipMemsetAsync(d_h0, 0, 256 * 8, s));
    TimedLaunch t(ix.timer, "sa_digit_hist", (double)n);
    const uint64_t tiles = ceil_div(n, (uint64_t)BH_TILE);
    const uint64_t tpw = ceil_div(tiles, 512);   // two workgroups per CU (small LDS)
    const unsigned grid = (unsigned)ceil_div(tiles, tpw);
    k_bucket_hist<true, true><<<grid, BH_T, 0, s>>>(ix.text.as<uint8_t>(), n, d_lutk, d_skey, ka, bsh, D,
                                                    reinterpret_cast<unsigned long long*>(d_h0), tpw * BH_TILE);
    HK_HIP(hipGetLastError());
  } else if (D > 0) {
    ix.bk_hist.ensure((uint64_t)nbins * 8);
    // skewed texts at scale (natural language, proteins) end on the global path anyway: the bucket counts of a
    // sixteenth of the text - spans spread evenly over it, so a skewed head (a header, a run) does not decide
    // alone - settle that before the whole text is counted (1 GiB protein-like: 4.1 ms)
    if (n >= (1ull << 26)) {
      HK_HIP(hipMemsetAsync(ix.bk_hist.p, 0, (uint64_t)nbins * 8, s));
      {
        TimedLaunch t(ix.timer, "sa_bucket_hist", (double)n / 16);
        const uint64_t tiles = ceil_div(n / 16, (uint64_t)BH_TILE);
        const uint64_t tpw = ceil_div(tiles, 256);
        const unsigned grid = (unsigned)ceil_div(tiles, tpw);
        const uint64_t stride = n / grid / BH_TILE * BH_TILE;   // >= the span: n / grid >= 16 spans
        k_bucket_hist<false><<<grid, BH_T, 0, s>>>(ix.text.as<uint8_t>(), n, d_lutk, d_skey, ka, bsh, D,
                                                   ix.bk_hist.as<unsigned long long>(), tpw * BH_TILE, stride);
        HK_HIP(hipGetLastError());
      }
      HK_HIP(hipMemcpyAsync(hist.data(), ix.bk_hist.p, (uint64_t)nbins * 8, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
      uint64_t tot = 0, big = 0;
      for (uint32_t b = 0; b < nbins; ++b) tot += hist[b];
      const uint64_t cap = item_T == 512 ? (uint64_t)BR_CAP : (uint64_t)BS_CAP;
      for (uint32_t b = 0; b < nbins; ++b)
        if (tot && (double)hist[b] * (double)n / (double)tot > (double)cap) big += hist[b];
      if (tot && big * 4 > tot * 3) skip_plan = true;   // over 3/4 of the suffixes in big buckets
    }
  }
  if (D > 0 && !use_cp && !late_hist && !skip_plan) {
    HK_HIP(hipMemsetAsync(ix.bk_hist.p, 0, (uint64_t)nbins * 8, s));
    {
      TimedLaunch t(ix.timer, "sa_bucket_hist", (double)n);
      const uint64_t tiles = ceil_div(n, (uint64_t)BH_TILE);
      const uint64_t tpw = ceil_div(tiles, 256);   // one workgroup per CU
      const unsigned grid = (unsigned)ceil_div(tiles, tpw);
      k_bucket_hist<false><<<grid, BH_T, 0, s>>>(ix.text.as<uint8_t>(), n, d_lutk, d_skey, ka, bsh, D,
                                                 ix.bk_hist.as<unsigned long long>(), tpw * BH_TILE);
      HK_HIP(hipGetLastError());
    }
    HK_HIP(hipMemcpyAsync(hist.data(), ix.bk_hist.p, (uint64_t)nbins * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
  } else if (D == 0) {
    hist[0] = n;
  }

  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(n * 8 + 16);
    ix.vals[i].ensure(n * 4 + 16);
  }
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  uint32_t* vp[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
  const TextKeySrc tks{ix.text.as<uint8_t>(), n, d_lutk, d_lutp, d_skey, ka};
  int slot = 0;
  bool sorted_by_bucket = false;
  // packed records (section 1b): one u64 per suffix through both passes and the item sorts when the
  // key bits below pass A's 9-bit digit and the position bits fit 64 (1 GiB DNA: 33 + 31)
  PackedRecs pkr;
  {
    const int posb = 64 - __builtin_clzll(n - 1);
    // prev field of the records: the keyed code when the terminal is unkeyed (bits(Rk - 1))
    int pb2 = pb;
    if (kg.tcode >= 0) {
      pb2 = 1;
      while ((1ull << pb2) < kg.Rk) ++pb2;
      pb2 = std::min(pb2, pb);
    }
    if (use_cp && D == 17 && pb2 + bsh + 8 + posb <= 64) {
      pkr.g.pbits = posb;
      pkr.g.pb = pb;
      pkr.g.pb2 = pb2;
      pkr.g.tcode = pb2 < pb ? kg.tcode : -1;
      for (int b = 0; b < 256; ++b)
        pkr.lutp2[b] = pkr.g.tcode < 0 ? kg.lutp[b] : (kg.kflag[b] ? kg.kdig[b] : 0);
      pkr.kfull = kp[1];
      pkr.vfull = vp[1];
      // radix 2^2: the register pre-pass over all 2^17 buckets
      SliceSel& r = pkr.rsl;
      if (tks.g.lb == 2 && reg_tables(kg, r)) {
        r.base = 0;
        r.nb = 1u << 17;
        r.DB = 17;
        r.bsh = bsh;
        r.sA = 8;
        r.wb = 0;
        r.wn1 = ~0u;
        pkr.reg = true;
      }
    }
  }
  const bool packed = pkr.g.pbits > 0;
  if (use_cp) {
    slot = cursor_partition(ix, n, D, pb + bsh, 0, &tks, kp, vp, hist, packed ? &pkr : nullptr);
    sorted_by_bucket = true;
    if (packed) ix.info[7] |= 2;
  } else if (late_hist) {
    // ---- LSD passes over the bucket bits (the first builds the keys from the text), then the
    // bucket counts from the sorted keys
    slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, n, pb + bsh, pb + sb, true, s, d_h0, &tks);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    sorted_by_bucket = true;
    ix.bk_hist.ensure((uint64_t)(nbins + 1) * 8);
    {
      TimedLaunch t(ix.timer, "sa_bin_starts", (double)(nbins + 1) * 8);
      k_bin_starts<<<(nbins + 1 + 255) / 256, 256, 0, s>>>(kp[slot], n, 0, pb + bsh, nbins,
                                                          ix.bk_hist.as<uint64_t>());
      HK_HIP(hipGetLastError());
    }
    std::vector<uint64_t> st(nbins + 1);
    HK_HIP(hipMemcpyAsync(st.data(), ix.bk_hist.p, (uint64_t)(nbins + 1) * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    for (uint32_t b = 0; b < nbins; ++b) hist[b] = st[b + 1] - st[b];
  }

  // ---- 2. work items (whole buckets, packed while they fit) and big buckets
  BucketPlan plan;
  if (skip_plan) plan.big_total = n;   // (the global path: no items)
  else plan = plan_buckets(hist, bsh, item_T == 512 ? (uint64_t)BR_CAP : (uint64_t)BS_CAP, packed ? 8 : 32);
  const std::vector<uint2>& items_n = plan.items_n;
  const std::vector<uint2>& items_w = plan.items_w;
  const std::vector<uint64_t>& big_start = plan.big_start;
  const std::vector<uint64_t>& big_cstart = plan.big_cstart;
  const uint64_t big_total = plan.big_total;
  ix.info[4] = items_n.size() + items_w.size();
  ix.info[5] = big_start.size();
  ix.info[6] = big_total;

  auto pack = [&]() {
    TimedLaunch t(ix.timer, "sa_pack_keys", (double)n * 9);
    const uint64_t g = std::min<uint64_t>(ceil_div(n, PKK_TILE), 4096);
    k_pack_keyed<<<(unsigned)g, 256, 0, s>>>(ix.text.as<uint8_t>(), n, d_lutk, d_lutp, d_skey, ka, kp[0]);
    HK_HIP(hipGetLastError());
  };

  if (big_total > n / 2) {
    // skewed text: the global path (full LSD radix sort + refinement from the keys)
    int gs;
    if (packed) {   // full keys into slot 1 first
      std::vector<uint2> ch;
      for (uint64_t a = 0; a < n; a += 65536) ch.push_back(make_uint2((uint32_t)a, (uint32_t)std::min<uint64_t>(65536, n - a)));
      ix.bk_items.ensure(ch.size() * sizeof(uint2) + 16);
      HK_HIP(hipMemcpyAsync(ix.bk_items.p, ch.data(), ch.size() * sizeof(uint2), hipMemcpyHostToDevice, s));
      unpack_items(ix, pkr, kp[slot], ix.bk_items.as<uint2>(), (uint32_t)ch.size());
      HK_HIP(hipStreamSynchronize(s));   // ch is freed at the end of this block
      gs = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 1, n, pb, pb + sb, false, s);
    } else if (sorted_by_bucket) {
      gs = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, slot, n, pb, pb + sb, false, s);
    } else {
      pack();
      gs = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, n, pb, pb + sb, true, s);
    }
    const int slot = gs;
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    std::swap(ix.sa, ix.vals[slot]);
    ix.vals[slot].ensure(n * 4 + 16);
    ix.info[7] |= 1;
    refine_after_sort<uint32_t>(ix, kg, slot, n, true);
    HK_HIP(hipStreamSynchronize(s));
    ix.have_sa = ix.have_bwt = true;
    return;
  }

  // ---- 3. LSD passes over the top D bits (digit histograms are marginals of the bucket histogram)
  if (sorted_by_bucket) {
    // done above
  } else if (D > 0) {
    // the first pass builds the keys from the text (no key array is written and re-read); both
    // passes are onesweep passes with decoupled lookback (measured faster on MI355X than a
    // reduce-then-scan with per-tile offset tables, which adds table traffic to every tile)
    uint64_t h0[256] = {0};
    const int lowd = std::min(D, 8);
    for (uint32_t b = 0; b < nbins; ++b) h0[b & ((1u << lowd) - 1)] += hist[b];
    HK_HIP(hipMemcpyAsync(d_h0, h0, sizeof(h0), hipMemcpyHostToDevice, s));
    slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, n, pb + bsh, pb + sb, true, s, d_h0, &tks);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
  } else {
    pack();
    fill_iota<uint32_t>(vp[0], n, s);
  }

  // ---- 4. LDS sorts of the buckets
  uint64_t ntie = sort_bucket_items<uint32_t>(ix, plan, kp[slot], vp[slot], n, pb, sb, 0, 0, ix.sa.as<uint32_t>(),
                                              ix.bwt.as<uint8_t>(), packed ? &pkr : nullptr);

  // ---- 5. big buckets on the global path
  if (big_total) {
    const uint32_t nbig = (uint32_t)big_start.size();
    int gbits = 1;
    while ((1ull << gbits) < nbig) ++gbits;
    const int lowbits = pb + bsh;
    for (int i = 0; i < 2; ++i) {
      ix.big_k[i].ensure(big_total * 8 + 16);
      ix.big_v[i].ensure(big_total * 4 + 16);
    }
    ix.big_j.ensure(big_total * 4 + 16);
    ix.tile_a.ensure(nbig * 8 + 16);
    ix.tile_c.ensure(nbig * 8 + 16);
    HK_HIP(hipMemcpyAsync(ix.tile_a.p, big_start.data(), nbig * 8, hipMemcpyHostToDevice, s));
    HK_HIP(hipMemcpyAsync(ix.tile_c.p, big_cstart.data(), nbig * 8, hipMemcpyHostToDevice, s));
    {
      TimedLaunch t(ix.timer, "sa_big_gather", (double)big_total * (12 + 16));
      k_big_gather<<<grid_of(big_total), 256, 0, s>>>(kp[slot], vp[slot], ix.tile_a.as<uint64_t>(),
                                                     ix.tile_c.as<uint64_t>(), nbig, big_total, lowbits,
                                                     ix.big_k[0].as<uint64_t>(), ix.big_v[0].as<uint32_t>(),
                                                     ix.big_j.as<uint32_t>(), pkr.g);
      HK_HIP(hipGetLastError());
    }
    uint64_t* bk[2] = {ix.big_k[0].as<uint64_t>(), ix.big_k[1].as<uint64_t>()};
    uint32_t* bv[2] = {ix.big_v[0].as<uint32_t>(), ix.big_v[1].as<uint32_t>()};
    const int bsl = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, bk, bv, 0, big_total, pb, lowbits + gbits, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    for (int i = 0; i < 3; ++i) ix.act[0][i].ensure(big_total * 4 + 16);
    ix.head_slot.ensure(big_total * 4 + 16);
    const auto r = refine_step_u32(ix, kg, bk[bsl], bv[bsl], ix.big_j.as<uint32_t>(), big_total, pb,
                                   ix.act[0][0].as<uint32_t>(), ix.act[0][1].as<uint32_t>(),
                                   ix.act[0][2].as<uint32_t>());
    if (r.first) {
      k_tie_append<<<grid_of(r.first), 256, 0, s>>>(ix.act[0][0].as<uint32_t>(), ix.act[0][1].as<uint32_t>(),
                                                   ix.act[0][2].as<uint32_t>(), r.first, ntie,
                                                   ix.ties_k.as<uint64_t>(), ix.ties_v.as<uint32_t>());
      HK_HIP(hipGetLastError());
      ntie += r.first;
    }
  }
  ix.info.push_back(ntie);

  // ---- 6. refinement of the ties
  refine_from_ties<uint32_t>(ix, kg, ntie, true);
  HK_HIP(hipStreamSynchronize(s));
  ix.have_sa = true;
  ix.have_bwt = true;
}

}  // namespace hk
