// hk_sa.hip — suffix array + BWT construction (single GPU), the refinement loop shared with the
// sharded build, alphabet/C array and the synthetic-text generator.
//
// Semantics follow the reference exactly (SURVEY.md §8 "Exact semantics"):
//   * SA of T' in Python str order (csa/suffix_array.py:131-134): symbols compare by byte
//     value, end-of-text is smaller than every symbol ('$' is an ordinary byte).
//   * BWT[j] = T'[SA[j]-1], wrapping to T'[n-1] (csa/bwt.py:3-13).
//   * C[c] = #{symbols < c} (utils/utils.py:16-24).
//
// Algorithm (MI355X-first):
//   1. every suffix p gets a u64 key = [its first q dense codes, b bits each, code 0 past the
//      end] [code of T'[p-1]] — the low field is not sorted on; it rides along so that the BWT
//      symbol of every sorted suffix is read straight out of the sorted keys (no random
//      gather over the text for the BWT);
//   2. one onesweep LSD radix sort orders the suffixes by q symbols (HBM-bound passes);
//   3. tied groups (equal q-prefix) are refined without any rank array: each round sorts the
//      tied suffixes by (dense group ordinal, next symbols of the suffix read from T');
//   4. if ties persist for several rounds (long repeats), the build switches to prefix
//      doubling: it materialises ISA once and sorts the tied suffixes by (group start,
//      ISA[p+h]), doubling h until no ties remain.
// High-entropy texts (the sigma=4 bench configs) finish after step 3's first round.

#include <cmath>

#include <algorithm>

#include "hk_index.hpp"
#include "hk_keys.hpp"
#include "hk_seground.hpp"

namespace hk {
namespace {

constexpr int GR_T = 256;
constexpr int GR_I = 16;
constexpr int GR_TILE = GR_T * GR_I;
constexpr int kChunkRounds = 4;   // refinement rounds before switching to prefix doubling

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

// ------------------------------------------------------------- alphabet
// One counter copy per lane index (64 per workgroup, shared by the 4 waves' lanes of that index), u16
// pairs with rows 129 words apart, so the lanes adding the same byte hit 64 different banks: no
// contention at all (8 copies per wave left 77 % of the LDS cycles in conflicts for DNA,
// profiles/r2c_sq_counters.json).  The grid keeps every copy below 2^16 (byte_hist_range).
constexpr int BH_ROW = 129;
__global__ __launch_bounds__(256) void k_byte_hist(const uint8_t* __restrict__ t, uint64_t n,
                                                   unsigned long long* __restrict__ hist) {
  __shared__ uint32_t h[64 * BH_ROW];
  for (int i = threadIdx.x; i < 64 * BH_ROW; i += 256) h[i] = 0;
  __syncthreads();
  uint32_t* mine = h + (threadIdx.x & 63) * BH_ROW;
  auto add4 = [&](uint32_t w) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const uint32_t x = (w >> (8 * b)) & 255u;
      atomicAdd(&mine[x >> 1], 1u << (16 * (x & 1u)));
    }
  };
  const uint64_t nv = n / 16;
  const uint4* t4 = reinterpret_cast<const uint4*>(t);
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
  for (; i + stride < nv; i += 2 * stride) {   // two 16-byte loads in flight per lane
    const uint4 v0 = t4[i], v1 = t4[i + stride];
    add4(v0.x); add4(v0.y); add4(v0.z); add4(v0.w);
    add4(v1.x); add4(v1.y); add4(v1.z); add4(v1.w);
  }
  for (; i < nv; i += stride) {
    const uint4 v = t4[i];
    add4(v.x); add4(v.y); add4(v.z); add4(v.w);
  }
  if (blockIdx.x == 0)
    for (uint64_t j = nv * 16 + threadIdx.x; j < n; j += 256) {
      const uint32_t x = t[j];
      atomicAdd(&mine[x >> 1], 1u << (16 * (x & 1u)));
    }
  __syncthreads();
  const uint32_t b = threadIdx.x, sh = 16u * (b & 1u);
  uint32_t c = 0;
#pragma unroll 8
  for (int r = 0; r < 64; ++r) c += (h[r * BH_ROW + (b >> 1)] >> sh) & 0xFFFFu;
  if (c) atomicAdd(&hist[b], (unsigned long long)c);
}

// ------------------------------------------------------------- keys
// key(p) = (code(T[p]) .. code(T[p+q-1]) as a radix-R number) << pb | code(T[p-1]);
// also histograms the first sorted digit (bits [pb, pb+8)) for the radix sort's first pass.
constexpr int PK_TILE = 4096;
__global__ __launch_bounds__(256) void k_pack_keys(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                   uint64_t count, const uint16_t* __restrict__ lut, uint64_t R,
                                                   int q, int pb, int ck, uint64_t Rck, uint64_t Rlast,
                                                   uint64_t* __restrict__ keys, unsigned long long* __restrict__ hist0) {
  __shared__ uint16_t c[PK_TILE + kCodePad];   // q <= 64 symbols of look-ahead
  __shared__ uint16_t L[256];
  __shared__ uint32_t H[256];
  L[threadIdx.x] = lut[threadIdx.x];
  H[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t end = lo + count;
  const uint64_t stride = (uint64_t)gridDim.x * PK_TILE;
  TextWords<PK_TILE, 256> tw;
  if (lo + (uint64_t)blockIdx.x * PK_TILE < end) load_text_words(tw, t, n, lo + (uint64_t)blockIdx.x * PK_TILE);
  for (uint64_t base = lo + (uint64_t)blockIdx.x * PK_TILE; base < end; base += stride) {
    store_text_codes(c, L, tw, n, base);
    __syncthreads();
    if (base + stride < end) load_text_words(tw, t, n, base + stride);   // next tile's text in flight
#pragma unroll 4
    for (int k = 0; k < PK_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      const uint64_t p = base + off;
      if (p < end) {
        const uint64_t key = key_chunked(c, off, R, q, pb, ck, Rck, Rlast);
        keys[p - lo] = key;
        if (hist0) atomicAdd(&H[(uint32_t)(key >> pb) & 255u], 1u);
      }
    }
    __syncthreads();
  }
  if (hist0 && H[threadIdx.x]) atomicAdd(&hist0[threadIdx.x], (unsigned long long)H[threadIdx.x]);
}

// ------------------------------------------------------------- refinement
// (the grouping kernels of a refinement / doubling round are the row-major forms below)

// chunk refinement key: (group ordinal << (64-gbits)) | next qn codes of the suffix from offset h (radix R).
// Keyed layout: short suffixes (p >= s_start) tied with others in the first round take their exact
// rank among the short suffixes (srank < nS); every other chunk is offset by nS, so a short
// suffix sorts before the equal-key long suffixes (its boundary key B(s) is the smallest window
// value that sorts after it).
template <typename V>
__global__ __launch_bounds__(256) void k_refine_keys(const V* __restrict__ P, const uint32_t* __restrict__ G,
                                                     uint64_t A, const uint8_t* __restrict__ t, uint64_t n,
                                                     const uint16_t* __restrict__ lut, uint64_t R, int qn, int gbits,
                                                     uint64_t h, uint64_t* __restrict__ keys, V* __restrict__ vals,
                                                     uint64_t s_start, uint32_t nS,
                                                     const uint32_t* __restrict__ srank) {
  __shared__ uint16_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const V p = P[a];
    uint64_t chunk = 0;
    const uint64_t s = (uint64_t)p + h;
    if ((uint64_t)p >= s_start) {
      chunk = srank[(uint64_t)p - s_start];
    } else if (qn <= 16 && s + (uint64_t)qn <= n) {
      // the usual case: both aligned 16-byte loads issued at once (one line fetch, not one per dependent word
      // load — with 10^8 random positions in flight the line is gone from L2 before a dependent second load),
      // then a 16-byte window from s by 64-bit funnel shifts
      // The second chunk only when the qn symbols run past the first (English-like: qn ~ 5, so about a quarter of
      // the suffixes; a second chunk across a line boundary is a second line fetch)
      const uint64_t a16 = s & ~15ull;
      const uint32_t off = (uint32_t)(s & 15), r8 = (off & 7) * 8;
      const uint4 v0 = *reinterpret_cast<const uint4*>(t + a16);
      uint4 v1 = make_uint4(0, 0, 0, 0);
      if (off + (uint32_t)qn > 16) v1 = *reinterpret_cast<const uint4*>(t + a16 + 16);
      const uint64_t w0 = (uint64_t)v0.x | ((uint64_t)v0.y << 32), w1 = (uint64_t)v0.z | ((uint64_t)v0.w << 32);
      const uint64_t w2 = (uint64_t)v1.x | ((uint64_t)v1.y << 32), w3 = (uint64_t)v1.z | ((uint64_t)v1.w << 32);
      const uint64_t A0 = off >= 8 ? w1 : w0, B0 = off >= 8 ? w2 : w1, C0 = off >= 8 ? w3 : w2;
      const uint64_t W0 = r8 ? (A0 >> r8) | (B0 << (64 - r8)) : A0;
      const uint64_t W1 = r8 ? (B0 >> r8) | (C0 << (64 - r8)) : B0;
      for (int j = 0; j < qn; ++j) {
        const uint32_t b = (uint32_t)((j < 8 ? W0 >> (8 * j) : W1 >> (8 * (j - 8))) & 255u);
        chunk = chunk * R + L[b];
      }
      chunk += nS;
    } else {
      // the qn symbols from s, read as aligned 32-bit words (the text buffer has >= 64 bytes of pad)
      const uint64_t w0 = s & ~3ull;
      uint32_t word = s < n ? *reinterpret_cast<const uint32_t*>(t + w0) : 0u;
      uint64_t wpos = w0;
      for (int j = 0; j < qn; ++j) {
        const uint64_t x = s + j;
        if ((x & ~3ull) != wpos) {
          wpos = x & ~3ull;
          word = wpos < n ? *reinterpret_cast<const uint32_t*>(t + wpos) : 0u;
        }
        chunk = chunk * R + (x < n ? L[(word >> (8 * (x & 3))) & 255u] : 0u);
      }
      chunk += nS;
    }
    keys[a] = gbits ? (((uint64_t)G[a] << (64 - gbits)) | chunk) : chunk;
    vals[a] = p;
  }
}

// Segmented sort of a refinement round's keys: the tied suffixes are listed group by group (G
// ascending, each group contiguous) and only the order inside a group matters, so the thread of a
// group's head sorts a group of <= SEG_MAX members in registers (bitonic network over 16, padded with
// ~0 keys) in place; a larger group raises *big and the round takes the global radix sort instead.
// Equal keys may swap (they stay tied, and their slots are reassigned by the next round).
constexpr int SEG_MAX = 16;

// bitonic network over N registers (the group's sz <= N members, padded with ~0 keys), sorted in place
template <int N, typename V>
__device__ __forceinline__ void seg_sort_net(uint64_t* __restrict__ keys, V* __restrict__ vals, uint32_t sz) {
  uint64_t k[N];
  V v[N];
#pragma unroll
  for (int i = 0; i < N; ++i) {
    k[i] = (uint32_t)i < sz ? keys[i] : ~0ull;
    v[i] = (uint32_t)i < sz ? vals[i] : (V)0;
  }
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int j = i ^ stride;
        if (j > i) {
          const bool up = (i & size) == 0;
          const bool sw = up ? k[i] > k[j] : k[i] < k[j];
          const uint64_t ki = k[i], kj = k[j];
          const V vi = v[i], vj = v[j];
          k[i] = sw ? kj : ki;
          k[j] = sw ? ki : kj;
          v[i] = sw ? vj : vi;
          v[j] = sw ? vi : vj;
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < N; ++i)
    if ((uint32_t)i < sz) {
      keys[i] = k[i];
      vals[i] = v[i];
    }
}

template <typename V>
__global__ __launch_bounds__(256) void k_seg_sort16(uint64_t* __restrict__ keys, V* __restrict__ vals,
                                                    const uint32_t* __restrict__ G, uint64_t A,
                                                    unsigned int* __restrict__ big, uint8_t* __restrict__ gbig) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint32_t g = G[a];
    if (a > 0 && G[a - 1] == g) continue;   // not a head
    uint32_t sz = 1;
    while (sz <= SEG_MAX && a + sz < A && G[a + sz] == g) ++sz;
    if (sz > SEG_MAX) {   // left for sort_big_groups (its members gathered by the group's flag)
      atomicOr(big, 1u);
      gbig[g] = 1;
      continue;
    }
    if (sz == 1) continue;
    if (sz == 2) {   // (pairs: most groups of a doubling round over long repeats)
      const uint64_t k0 = keys[a], k1 = keys[a + 1];
      if (k1 < k0) {
        const V v0 = vals[a], v1 = vals[a + 1];
        keys[a] = k1;
        keys[a + 1] = k0;
        vals[a] = v1;
        vals[a + 1] = v0;
      }
      continue;
    }
    if (sz <= 4) seg_sort_net<4>(keys + a, vals + a, sz);
    else seg_sort_net<SEG_MAX>(keys + a, vals + a, sz);
  }
}

// Members of the groups k_seg_sort16 left (over SEG_MAX members, gbig[G] = 1): per-tile counts, then
// gathered in list order (row-major tiles, one block scan per row) with their list positions, radix-sorted
// (the key carries the group in its top bits, so groups stay apart and in order) and scattered back.
__global__ __launch_bounds__(GR_T) void k_big_count_rows(const uint32_t* __restrict__ G,
                                                         const uint8_t* __restrict__ gbig, uint64_t A,
                                                         uint32_t* __restrict__ tcnt) {
  __shared__ uint32_t ra[GR_T / 64];
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  uint32_t c = 0;
#pragma unroll 4
  for (int k = 0; k < GR_I; ++k) {
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    if (j >= A) break;
    c += gbig[G[j]];
  }
  c = wave_sum<uint32_t>(c);
  if ((threadIdx.x & 63) == 0) ra[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < GR_T / 64; ++i) t += ra[i];
    tcnt[blockIdx.x] = t;
  }
}

// oj: the member's list position, or with J its SA slot (a round's big groups regrouped as their own list)
template <typename V>
__global__ __launch_bounds__(GR_T) void k_big_compact_rows(const uint64_t* __restrict__ keys, const V* __restrict__ vals,
                                                           const uint32_t* __restrict__ G,
                                                           const uint8_t* __restrict__ gbig, uint64_t A,
                                                           const uint64_t* __restrict__ toff, uint64_t* __restrict__ ok,
                                                           V* __restrict__ ov, uint32_t* __restrict__ oj,
                                                           const uint32_t* __restrict__ J = nullptr) {
  __shared__ uint32_t wc[2][GR_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  uint64_t run = toff[blockIdx.x];
  for (int k = 0; k < GR_I; ++k) {   // (uniform)
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    const uint32_t f = j < A ? gbig[G[j]] : 0u;
    const uint32_t ci = dpp_incl_sum(f);
    if (lane == 63) wc[k & 1][w] = ci;
    __syncthreads();
    uint32_t pre = 0, row = 0;
#pragma unroll
    for (int i = 0; i < GR_T / 64; ++i) {
      const uint32_t x = wc[k & 1][i];
      pre += i < w ? x : 0u;
      row += x;
    }
    if (f) {
      const uint64_t o = run + pre + ci - 1;
      ok[o] = keys[j];
      ov[o] = vals[j];
      oj[o] = J ? J[j] : (uint32_t)j;
    }
    run += row;
  }
}

template <typename V>
__global__ __launch_bounds__(256) void k_big_scatter(const uint64_t* __restrict__ k, const V* __restrict__ v,
                                                     const uint32_t* __restrict__ pos, uint64_t B,
                                                     uint64_t* __restrict__ keys, V* __restrict__ vals) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < B; i += (uint64_t)gridDim.x * 256) {
    const uint32_t j = pos[i];
    keys[j] = k[i];
    vals[j] = v[i];
  }
}

// ------------------------------------------------------------- prefix doubling
// ISA values are global SA slots (slice offset lo + slot in the slice).  Every member of a tied
// group carries the slot of the group's head, so ISA is an order-consistent K-order rank:
// isa[x] < isa[y] => suffix x < suffix y, and isa[x] == isa[y] => x and y share their first K
// symbols, K = the smallest common-prefix length of any group still tied (on any rank).  A round
// sorts each tied group (members sharing h >= K symbols) by ISA[p + h]: the new groups share h + K.
template <typename V>
__global__ __launch_bounds__(256) void k_isa_from_sa(const V* __restrict__ sa, uint64_t m, uint64_t lo,
                                                     V* __restrict__ isa) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < m; j += (uint64_t)gridDim.x * 256)
    isa[sa[j]] = (V)(lo + j);
}

// tied suffixes: ISA = slot of their group head; into isa directly, or as (position, ISA) pairs
template <typename V>
__global__ __launch_bounds__(256) void k_dbl_emit(const V* __restrict__ P, const uint32_t* __restrict__ G, uint64_t A,
                                                  const uint32_t* __restrict__ head_slot, uint64_t lo,
                                                  V* __restrict__ isa, uint64_t* __restrict__ pairs) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint64_t p = P[a], v = lo + head_slot[G[a]];
    if (pairs) {
      pairs[2 * a] = p;
      pairs[2 * a + 1] = v;
    } else {
      isa[p] = (V)v;
    }
  }
}

template <typename V>
__global__ __launch_bounds__(256) void k_dbl_apply_pairs(const uint64_t* __restrict__ pairs, uint64_t cnt,
                                                         V* __restrict__ isa) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < cnt; i += (uint64_t)gridDim.x * 256)
    isa[pairs[2 * i]] = (V)pairs[2 * i + 1];
}

// ---- ISA of every position at the switch to prefix doubling (single GPU, u32 positions).  ISA[p] = its SA slot,
// or for a tied suffix its group head's slot.  A straight scatter isa[SA[j]] = v writes 4 B at a random
// position per suffix, and each such write costs a whole line at the memory side (7.2 ms and 6.7 GB of writes
// for a 200 MiB text).  Instead: hs[j] = the value of slot j (iota, then the tied slots' head slots, near-
// coalesced along the tie list); the (SA[j], hs[j]) pairs are partitioned twice by position — into 256
// level-1 buckets of 2^S1 positions, then inside each into 2^(S1 - S2) sub-buckets of 2^S2 positions — and
// every sub-bucket's ISA window is assembled in LDS and written whole.  SA is a permutation, so every
// bucket's size is known without counting: bucket b holds exactly the positions [b << S, (b + 1) << S).
// Each partition pass stages its tile of pairs in LDS by digit, so the runs it writes are contiguous.
constexpr int PP_T = 512, PP_I = 8, PP_TILE = PP_T * PP_I;    // partition tiles: 4096 pairs (48 KiB of LDS:
                                                               // three workgroups per CU)
constexpr int PW_MAX = 14;                                     // sub-buckets of <= 2^14 positions (64 KiB)

__global__ __launch_bounds__(256) void k_hs_tied(const uint32_t* __restrict__ J, const uint32_t* __restrict__ G,
                                                 uint64_t A, const uint32_t* __restrict__ head_slot,
                                                 uint32_t* __restrict__ hs, uint64_t n, uint64_t groups,
                                                 uint32_t* __restrict__ err) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint32_t j = J[a], g = G[a];
    if (j < n && g < groups) hs[j] = head_slot[g];
    else atomicOr(err, 1u);
  }
}

// cur[i] = i << sh (the cursors of buckets whose sizes are exact powers of two)
__global__ __launch_bounds__(256) void k_pos_cursors(uint64_t* __restrict__ cur, uint64_t nb, int sh) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nb; i += (uint64_t)gridDim.x * 256)
    cur[i] = i << sh;
}

// One partition pass: LEVEL 1 reads (SA[j], hs[j]) over tiles of [0, n) and partitions by p >> s_hi (256
// digits); LEVEL 2 reads the level-1 pairs over tiles aligned to level-1 buckets (2^s_hi positions, so a tile
// never straddles two) and partitions by (p >> s_lo) inside the bucket.  The digit's cursor is
// cur[p >> s_lo] (LEVEL 2) or cur[p >> s_hi] (LEVEL 1).
template <int LEVEL>
__global__ __launch_bounds__(PP_T, 3) void k_pos_part(const uint32_t* __restrict__ sa, const uint32_t* __restrict__ hs,
                                                     const uint64_t* __restrict__ pin, uint64_t n, int s_hi, int s_lo,
                                                     unsigned long long* __restrict__ cur, uint64_t* __restrict__ pout,
                                                     uint32_t* __restrict__ err) {
  __shared__ uint64_t stage[PP_TILE];
  __shared__ uint32_t cnt[1024], lst[1024];
  __shared__ unsigned long long gb[1024];
  __shared__ uint32_t wsum[PP_T / 64];
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int dbits = LEVEL == 1 ? 8 : s_hi - s_lo;   // <= 10
  const uint32_t nd = 1u << dbits;
  uint64_t t0, t1;
  if (LEVEL == 1) {
    t0 = (uint64_t)blockIdx.x * PP_TILE;
    t1 = t0 + PP_TILE < n ? t0 + PP_TILE : n;
  } else {   // tiles per level-1 bucket: 2^s_hi / PP_TILE (s_hi >= 13 > log2(PP_TILE))
    const uint64_t tpb = (1ull << s_hi) / PP_TILE;
    const uint64_t b = blockIdx.x / tpb;
    t0 = (b << s_hi) + (blockIdx.x % tpb) * PP_TILE;
    const uint64_t be = ((b + 1) << s_hi) < n ? ((b + 1) << s_hi) : n;
    t1 = t0 + PP_TILE < be ? t0 + PP_TILE : be;
  }
  if (t0 >= t1) return;   // (uniform: past the text's last bucket)
  for (uint32_t i = tid; i < nd; i += PP_T) cnt[i] = 0;
  __syncthreads();
  uint64_t pr[PP_I];
  uint32_t rk[PP_I];
#pragma unroll
  for (int k = 0; k < PP_I; ++k) {
    const uint64_t j = t0 + (uint64_t)k * PP_T + tid;
    rk[k] = 0;
    pr[k] = 0;
    if (j < t1) {
      pr[k] = LEVEL == 1 ? ((uint64_t)sa[j] << 32) | hs[j] : pin[j];
      if ((pr[k] >> 32) >= n) {   // (only a corrupt SA: dropped, reported; no write past the pair array)
        atomicOr(err, 1u);
        pr[k] = ~0ull;
        continue;
      }
      const uint32_t d = (uint32_t)((pr[k] >> 32) >> (LEVEL == 1 ? s_hi : s_lo)) & (nd - 1);
      rk[k] = atomicAdd(&cnt[d], 1u);
    }
  }
  __syncthreads();
  // exclusive digit starts inside the tile (nd <= 1024: two per thread) and the runs' global destinations
  {
    uint32_t c0 = tid < nd ? cnt[tid] : 0u, c1 = tid + PP_T < nd ? cnt[tid + PP_T] : 0u;
    const uint32_t a0 = c0, a1 = c1;
    const uint32_t i0 = dpp_incl_sum(a0);
    if (lane == 63) wsum[wv] = i0;
    __syncthreads();
    uint32_t carry = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < PP_T / 64; ++w) {
      carry += (uint32_t)w < wv ? wsum[w] : 0u;
      tot += wsum[w];
    }
    __syncthreads();
    const uint32_t i1 = dpp_incl_sum(a1);
    if (lane == 63) wsum[wv] = i1;
    if (tid < nd) {
      lst[tid] = carry + i0 - a0;
      const uint64_t key = LEVEL == 1 ? (uint64_t)tid : (t0 >> s_lo) - ((t0 >> s_lo) & (nd - 1)) + tid;
      gb[tid] = c0 ? atomicAdd(cur + key, (unsigned long long)c0) : 0ull;
    }
    __syncthreads();
    if (tid + PP_T < nd) {
      uint32_t carry1 = tot;
#pragma unroll
      for (int w = 0; w < PP_T / 64; ++w) carry1 += (uint32_t)w < wv ? wsum[w] : 0u;
      lst[tid + PP_T] = carry1 + i1 - a1;
      const uint64_t key = (t0 >> s_lo) - ((t0 >> s_lo) & (nd - 1)) + tid + PP_T;
      gb[tid + PP_T] = c1 ? atomicAdd(cur + key, (unsigned long long)c1) : 0ull;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < PP_I; ++k) {
    const uint64_t j = t0 + (uint64_t)k * PP_T + tid;
    if (j < t1 && pr[k] != ~0ull) {
      const uint32_t d = (uint32_t)((pr[k] >> 32) >> (LEVEL == 1 ? s_hi : s_lo)) & (nd - 1);
      stage[lst[d] + rk[k]] = pr[k];
    }
  }
  __syncthreads();
  const uint32_t m = lst[nd - 1] + cnt[nd - 1];   // (every kept pair is staged in [0, m))
#pragma unroll
  for (int k = 0; k < PP_I; ++k) {
    const uint32_t sidx = (uint32_t)k * PP_T + tid;
    if (sidx < m) {
      const uint64_t q = stage[sidx];
      const uint32_t d = (uint32_t)((q >> 32) >> (LEVEL == 1 ? s_hi : s_lo)) & (nd - 1);
      const uint64_t dst = gb[d] + (sidx - lst[d]);
      if (dst < n) pout[dst] = q;
      else atomicOr(err, 1u);
    }
  }
}

// one sub-bucket of 2^s_lo positions per workgroup: its pairs (exactly the positions of its range) scattered
// into an LDS window, written out whole
__global__ __launch_bounds__(512) void k_pos_write(const uint64_t* __restrict__ pin, uint64_t n, int s_lo,
                                                   uint32_t* __restrict__ isa, uint32_t* __restrict__ err) {
  __shared__ uint32_t win[1u << PW_MAX];
  const uint64_t lo = (uint64_t)blockIdx.x << s_lo;
  const uint64_t hi = lo + (1ull << s_lo) < n ? lo + (1ull << s_lo) : n;
  for (uint64_t a = lo + threadIdx.x; a < hi; a += 512) {
    const uint64_t q = pin[a];
    const uint64_t o = (q >> 32) - lo;
    if (o < hi - lo) win[(uint32_t)o] = (uint32_t)q;
    else atomicOr(err, 1u);
  }
  __syncthreads();
  for (uint64_t a = lo + threadIdx.x; a < hi; a += 512) isa[a] = win[(uint32_t)(a - lo)];
}

// doubling keys: (dense group ordinal << ib) | (ISA[p + h] + 1, or 0 past the end), value = position.  A linked
// position's ISA is that of the position its link names plus the link's slot delta (hk_seground.hpp)
template <typename V>
__global__ __launch_bounds__(256) void k_dbl_keys(const V* __restrict__ P, const uint32_t* __restrict__ G, uint64_t A,
                                                  const V* __restrict__ isa, uint64_t n, uint64_t h, int ib,
                                                  uint64_t* __restrict__ keys, V* __restrict__ vals,
                                                  const uint32_t* __restrict__ lnk, uint64_t lh) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const V p = P[a];
    const uint64_t q = (uint64_t)p + h;
    uint64_t s = 0;
    if (q < n) {
      V v = isa[q];
      if constexpr (sizeof(V) == 4) {
        if (lnk && (v & LK_BIT)) {
          const uint64_t e = q + (uint64_t)(v & ~LK_BIT) * lh;
          v = e < n ? isa[e] + lnk[q] : 0;   // (e < n always: a link names a position of its target group)
        }
      }
      s = (uint64_t)v + 1;
    }
    keys[a] = ((uint64_t)G[a] << ib) | s;
    vals[a] = p;
  }
}

// ---- row-major forms of the grouping kernels: a tile's GR_I rows of GR_T consecutive items, item
// k * GR_T + tid of thread tid, so every load and the compacted stores are coalesced (the thread-
// contiguous forms above touch 64 lines per wave instruction).  Order-dependent quantities (the group
// head's slot, the compaction offsets) come from one block scan per row.
__device__ __forceinline__ void row_neighbors(const uint64_t* __restrict__ keys, uint64_t j, uint64_t A, int cs,
                                              bool& h, bool& hn, uint64_t& cur, uint64_t& prev) {
  cur = keys[j];
  prev = j ? keys[j - 1] : 0;
  const uint64_t nxt = j + 1 < A ? keys[j + 1] : 0;
  h = j == 0 || (cur >> cs) != (prev >> cs);
  hn = j + 1 >= A || (nxt >> cs) != (cur >> cs);
}

// k_refine_stats, row-major
__global__ __launch_bounds__(GR_T) void k_refine_stats_rows(const uint64_t* __restrict__ keys, uint64_t A, int cs,
                                                            uint32_t* __restrict__ tact,
                                                            uint32_t* __restrict__ thead) {
  __shared__ uint32_t ra[GR_T / 64];
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  uint32_t c = 0;   // tied | tied heads << 16 (<= 4096 each per tile)
#pragma unroll 4
  for (int k = 0; k < GR_I; ++k) {
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    if (j >= A) break;
    bool h, hn;
    uint64_t cur, prev;
    row_neighbors(keys, j, A, cs, h, hn, cur, prev);
    if (!(h && hn)) c += h ? 0x10001u : 1u;
  }
  c = wave_sum<uint32_t>(c);
  if ((threadIdx.x & 63) == 0) ra[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int i = 0; i < GR_T / 64; ++i) t += ra[i];
    tact[blockIdx.x] = t & 0xFFFFu;
    thead[blockIdx.x] = t >> 16;
  }
}

// Refinement grouping step, row-major: SA of every suffix, BWT of the settled ones, tied suffixes compacted
// with their group ordinal.  FROM_KEY (initial round, J == identity, SA already in place): the BWT of
// every suffix is the key's low field and P is read only for tied suffixes.
template <typename V, bool FROM_KEY>
__global__ __launch_bounds__(GR_T) void k_refine_apply_rows(
    const uint64_t* __restrict__ keys, const V* __restrict__ P, const uint32_t* __restrict__ J, uint64_t A,
    int cs, const uint64_t* __restrict__ act_off, const uint64_t* __restrict__ head_off, V* __restrict__ sa,
    uint8_t* __restrict__ bwt, const uint8_t* __restrict__ inv, uint64_t pmask, const uint8_t* __restrict__ t,
    uint64_t n, V* __restrict__ oP, uint32_t* __restrict__ oJ, uint32_t* __restrict__ oG,
    uint32_t* __restrict__ head_slot, uint8_t* __restrict__ oB) {
  __shared__ uint32_t wc[2][GR_T / 64];
  __shared__ uint8_t INV[512];
  if (FROM_KEY) {
    INV[threadIdx.x] = inv[threadIdx.x];
    INV[threadIdx.x + 256] = inv[threadIdx.x + 256];
    __syncthreads();
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  uint64_t run_o = act_off[blockIdx.x], run_g = head_off[blockIdx.x];
  for (int k = 0; k < GR_I; ++k) {   // (uniform: every thread runs every row's scan)
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    const bool valid = j < A;
    uint32_t a = 0, th = 0, jv = 0;
    uint8_t bc = 0;
    V p = 0;
    if (valid) {
      bool h, hn;
      uint64_t cur, prev;
      row_neighbors(keys, j, A, cs, h, hn, cur, prev);
      a = (h && hn) ? 0u : 1u;
      th = a && h ? 1u : 0u;
      jv = FROM_KEY ? (uint32_t)j : (J ? J[j] : (uint32_t)j);
      if (!FROM_KEY || a) p = P[j];
      if (FROM_KEY) {
        bc = INV[(uint32_t)(cur & pmask)];
        if (bwt) bwt[j] = bc;
      }
    }
    const uint32_t ci = dpp_incl_sum(a | th << 16);
    if (lane == 63) wc[k & 1][w] = ci;
    __syncthreads();
    uint32_t pre = 0, row = 0;
#pragma unroll
    for (int i = 0; i < GR_T / 64; ++i) {
      const uint32_t x = wc[k & 1][i];
      pre += i < w ? x : 0u;
      row += x;
    }
    if (valid) {
      if (!FROM_KEY && sa) sa[jv] = p;   // (every slot: prefix doubling builds its ISA from this SA)
      if (a) {
        const uint32_t inc = pre + ci;
        const uint64_t o = run_o + (inc & 0xFFFFu) - 1, g = run_g + (inc >> 16);
        if (th && head_slot) head_slot[g - 1] = jv;
        oP[o] = p;
        oJ[o] = jv;
        oG[o] = (uint32_t)(g - 1);
        if (FROM_KEY && oB) oB[o] = bc;   // (the tied suffix's BWT byte travels with it to the next round)
      } else if (!FROM_KEY && bwt) {
        bwt[jv] = t[p == 0 ? n - 1 : (uint64_t)p - 1];
      }
    }
    run_o += row & 0xFFFFu;
    run_g += row >> 16;
  }
}

// k_dbl_stats, row-major
__global__ __launch_bounds__(GR_T) void k_dbl_stats_rows(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ J, uint64_t A, int ib,
                                                         uint64_t* __restrict__ tile_last,
                                                         uint32_t* __restrict__ tile_act,
                                                         uint32_t* __restrict__ tile_heads) {
  __shared__ uint64_t red[GR_T / 64];
  __shared__ uint32_t redc[GR_T / 64];
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  uint64_t last = 0;
  uint32_t c = 0;
#pragma unroll 4
  for (int k = 0; k < GR_I; ++k) {
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    if (j >= A) break;
    bool h, hn;
    uint64_t cur, prev;
    row_neighbors(keys, j, A, 0, h, hn, cur, prev);
    if (h) {
      const uint64_t v = (j << 1 | ((j == 0 || (cur >> ib) != (prev >> ib)) ? 1u : 0u)) + 1;
      last = v > last ? v : last;
    }
    if (!(h && hn)) c += h ? 0x10001u : 1u;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t tt = __shfl_xor(last, o, 64);
    last = last > tt ? last : tt;
  }
  c = wave_sum<uint32_t>(c);
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = last;
    redc[threadIdx.x >> 6] = c;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t m = 0;
    uint32_t t = 0;
    for (int i = 0; i < GR_T / 64; ++i) {
      m = m > red[i] ? m : red[i];
      t += redc[i];
    }
    tile_last[blockIdx.x] = m;
    tile_act[blockIdx.x] = t & 0xFFFFu;
    tile_heads[blockIdx.x] = t >> 16;
  }
}

// k_dbl_apply, row-major
template <typename V>
__global__ __launch_bounds__(GR_T) void k_dbl_apply_rows(
    const uint64_t* __restrict__ keys, const V* __restrict__ P, const uint32_t* __restrict__ J, uint64_t A, int ib,
    bool keep_same, const uint64_t* __restrict__ carry_last, const uint64_t* __restrict__ act_off,
    const uint64_t* __restrict__ head_off, uint64_t lo, V* __restrict__ isa, uint64_t* __restrict__ pairs,
    V* __restrict__ sa, uint8_t* __restrict__ bwt, const uint8_t* __restrict__ t, uint64_t n, V* __restrict__ oP,
    uint32_t* __restrict__ oJ, uint32_t* __restrict__ oG, uint32_t* __restrict__ head_slot) {
  __shared__ uint64_t wm[2][GR_T / 64];
  __shared__ uint32_t wc[2][GR_T / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t tbase = (uint64_t)blockIdx.x * GR_TILE;
  // 1 + (list index << 1 | first) of the last group head so far (0: none), tied so far, tied heads so far.
  // (The list index, not the head's slot: the tie list holds whole groups in any order of groups.  A
  // group's slots are contiguous and ascending along the list, so the head's slot is jv - (j - index).)
  uint64_t run_h = carry_last[blockIdx.x], run_o = act_off[blockIdx.x], run_g = head_off[blockIdx.x];
  for (int k = 0; k < GR_I; ++k) {   // (uniform: every thread runs every row's scans)
    const uint64_t j = tbase + (uint64_t)k * GR_T + threadIdx.x;
    const bool valid = j < A;
    uint32_t a = 0, th = 0, jv = 0;
    uint64_t hv = 0;
    V p = 0;
    if (valid) {
      bool h, hn;
      uint64_t cur, prev;
      row_neighbors(keys, j, A, 0, h, hn, cur, prev);
      jv = J[j];
      p = P[j];
      a = (h && hn) ? 0u : 1u;
      th = a && h ? 1u : 0u;
      if (h) hv = (j << 1 | ((j == 0 || (cur >> ib) != (prev >> ib)) ? 1u : 0u)) + 1;
    }
    const uint64_t mi = wave_incl_max<uint64_t>(hv);
    const uint32_t ci = dpp_incl_sum(a | th << 16);
    if (lane == 63) {
      wm[k & 1][w] = mi;
      wc[k & 1][w] = ci;
    }
    __syncthreads();
    uint64_t hm = run_h, rowm = run_h;
    uint32_t pre = 0, row = 0;
#pragma unroll
    for (int i = 0; i < GR_T / 64; ++i) {
      const uint64_t x = wm[k & 1][i];
      const uint32_t c = wc[k & 1][i];
      if (i < w) {
        hm = hm > x ? hm : x;
        pre += c;
      }
      rowm = rowm > x ? rowm : x;
      row += c;
    }
    hm = hm > mi ? hm : mi;
    if (valid) {
      const uint64_t g = hm - 1;   // this suffix's group head: index << 1 | first (j's head is at or before j)
      const uint64_t v = lo + (jv - (j - (g >> 1)));
      if (pairs) {
        pairs[2 * j] = (uint64_t)p;
        pairs[2 * j + 1] = v;
      } else if (!(keep_same && (g & 1))) {
        isa[p] = (V)v;
      }
      if (a) {
        const uint32_t inc = pre + ci;
        const uint64_t o = run_o + (inc & 0xFFFFu) - 1, gg = run_g + (inc >> 16);
        if (th) head_slot[gg - 1] = jv;
        oP[o] = p;
        oJ[o] = jv;
        oG[o] = (uint32_t)(gg - 1);
      } else {   // settled: its final SA / BWT entry
        sa[jv] = p;
        bwt[jv] = t[p == 0 ? n - 1 : (uint64_t)p - 1];
      }
    }
    run_h = rowm;
    run_o += row & 0xFFFFu;
    run_g += row >> 16;
  }
}

__global__ __launch_bounds__(256) void k_bwt(const uint8_t* __restrict__ t, const uint32_t* __restrict__ sa,
                                             uint64_t n, uint8_t* __restrict__ bwt) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256) {
    const uint32_t p = sa[j];
    bwt[j] = t[p == 0 ? n - 1 : p - 1];
  }
}

__global__ __launch_bounds__(256) void k_bwt64(const uint8_t* __restrict__ t, const uint64_t* __restrict__ sa,
                                               uint64_t n, uint8_t* __restrict__ bwt) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256) {
    const uint64_t p = sa[j];
    bwt[j] = t[p == 0 ? n - 1 : p - 1];
  }
}

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

struct Alpha256 { uint8_t s[256]; };

__global__ __launch_bounds__(256) void k_synth(uint8_t* __restrict__ t, uint64_t n, Alpha256 al, int sigma,
                                               uint64_t seed, uint8_t term) {
  __shared__ uint8_t A[256];
  A[threadIdx.x] = al.s[threadIdx.x];
  __syncthreads();
  const uint64_t key = seed * 0xD1B54A32D192ED03ull;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    if (i + 1 == n) {
      t[i] = term;
    } else {
      const uint64_t r = splitmix64(key ^ i);
      t[i] = A[(uint32_t)(r >> 32) % (uint32_t)sigma];
    }
  }
}

int bits_of_u64(uint64_t v) {
  int b = 0;
  while (v) {
    ++b;
    v >>= 1;
  }
  return b;
}

// Segmented sort of a round's list (keys / vals in slot 0, grouped by the dense ordinals G): each group of
// <= SEG_MAX members sorted in place by its head thread; a larger group is left, flagged in ix.grp_big and
// in *d_big (sort_big_groups finishes it)
template <typename V>
void seg_sort_groups(Index& ix, uint64_t* k0, V* v0, const uint32_t* G, uint64_t A, uint64_t groups,
                     unsigned int* d_big, const char* name) {
  hipStream_t s = ix.stream;
  ix.grp_big.ensure(groups + 16);
  HK_HIP(hipMemsetAsync(d_big, 0, 4, s));
  HK_HIP(hipMemsetAsync(ix.grp_big.p, 0, groups, s));
  TimedLaunch tm(ix.timer, name, (double)A * (2 * 8 + 2 * sizeof(V) + 4));
  k_seg_sort16<V><<<grid_for(A), 256, 0, s>>>(k0, v0, G, A, d_big, ix.grp_big.as<uint8_t>());
  HK_HIP(hipGetLastError());
}

// The members of the groups seg_sort_groups left, gathered in list order, radix-sorted on key bits
// [0, bits) (the group ordinal is in the top bits) and scattered back to their list positions: only the
// large groups' members pass through the radix sort, not the whole list
template <typename V>
void sort_big_groups(Index& ix, uint64_t* k0, V* v0, const uint32_t* G, uint64_t A, int bits) {
  hipStream_t s = ix.stream;
  const uint64_t nt = ceil_div(A, GR_TILE);
  ix.tile_b.ensure((nt + 1) * 4);
  ix.tile_a.ensure((nt + 2) * 8);
  const uint8_t* gbig = ix.grp_big.as<uint8_t>();
  {
    TimedLaunch tm(ix.timer, "sa_big_groups", (double)A * 5);
    k_big_count_rows<<<(unsigned)nt, GR_T, 0, s>>>(G, gbig, A, ix.tile_b.as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nt, true, s);
  uint64_t* const rb = ix.rb();
  HK_HIP(hipMemcpyAsync(&rb[3], ix.tile_a.as<uint64_t>() + nt, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  const uint64_t B = rb[3];
  if (!B) return;
  for (int i = 0; i < 2; ++i) {
    ix.big_k[i].ensure(B * 8 + 16);
    ix.big_v[i].ensure(B * sizeof(V) + 16);
  }
  ix.big_j.ensure(B * 4 + 16);
  uint64_t* bk[2] = {ix.big_k[0].as<uint64_t>(), ix.big_k[1].as<uint64_t>()};
  V* bv[2] = {ix.big_v[0].as<V>(), ix.big_v[1].as<V>()};
  {
    TimedLaunch tm(ix.timer, "sa_big_groups", (double)A * 5 + (double)B * (8 + 2 * sizeof(V) + 4 + 8));
    k_big_compact_rows<V><<<(unsigned)nt, GR_T, 0, s>>>(k0, v0, G, gbig, A, ix.tile_a.as<uint64_t>(), bk[0], bv[0],
                                                        ix.big_j.as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  const int sl = radix_sort_pairs<V>(ix.sw, ix.timer, bk, bv, 0, B, 0, bits, false, s);
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  {
    TimedLaunch tm(ix.timer, "sa_big_groups", (double)B * (8 + sizeof(V) + 4 + 8 + sizeof(V)));
    k_big_scatter<V><<<grid_for(B), 256, 0, s>>>(bk[sl], bv[sl], ix.big_j.as<uint32_t>(), B, k0, v0);
    HK_HIP(hipGetLastError());
  }
}

// One doubling regroup over a sorted list (row kernels: stats, scans, apply): ISA of every member (or (position,
// ISA) pairs), SA / BWT of the settled ones, the tied ones into (oP, oJ, oG) from index 0.  d_flag (nullable): a
// device flag read back with the totals into *h_flag.  Returns (tied, groups).
template <typename V>
std::pair<uint64_t, uint64_t> dbl_apply_list(Index& ix, const uint64_t* keys, const V* vals, const uint32_t* J,
                                             uint64_t A, int ib, bool keep_same, uint64_t* pairs, V* oP, uint32_t* oJ,
                                             uint32_t* oG, const unsigned int* d_flag = nullptr,
                                             unsigned int* h_flag = nullptr) {
  hipStream_t s = ix.stream;
  const uint64_t nt = ceil_div(A, GR_TILE);
  ix.tile_a.ensure((nt + 2) * 8);
  ix.tile_b.ensure((nt + 1) * 4);
  ix.tile_c.ensure((nt + 1) * 8);
  ix.tile_d.ensure((nt + 2) * 8);
  DevBuf& tb2 = ix.tile_e;
  tb2.ensure((nt + 2) * 12 + 16);
  uint64_t* tl = ix.tile_a.as<uint64_t>();
  uint32_t* ta = ix.tile_b.as<uint32_t>();
  uint64_t* cl = ix.tile_c.as<uint64_t>();
  uint64_t* ao = ix.tile_d.as<uint64_t>();
  uint32_t* th = tb2.as<uint32_t>();
  uint64_t* ho = reinterpret_cast<uint64_t*>(tb2.as<uint8_t>() + ((nt + 2) * 4 + 7) / 8 * 8);
  {
    TimedLaunch tm(ix.timer, "sa_group_stats", (double)A * 8);
    k_dbl_stats_rows<<<(unsigned)nt, GR_T, 0, s>>>(keys, J, A, ib, tl, ta, th);
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_max_u64(ix.sw, tl, cl, nt, s);
  scan_exclusive_u32_to_u64(ix.sw, ta, ao, nt, true, s);
  scan_exclusive_u32_to_u64(ix.sw, th, ho, nt, true, s);
  {
    TimedLaunch tm(ix.timer, "sa_group_apply", (double)A * (8 + 2 * sizeof(V) + 4 + 1 + 1 + (pairs ? 16 : sizeof(V))));
    k_dbl_apply_rows<V><<<(unsigned)nt, GR_T, 0, s>>>(
        keys, vals, J, A, ib, keep_same, cl, ao, ho, ix.sharded ? ix.shard_lo : 0, ix.isa.as<V>(), pairs,
        ix.sa.as<V>(), ix.bwt.as<uint8_t>(), ix.text.as<uint8_t>(), ix.n, oP, oJ, oG, ix.head_slot.as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  uint64_t* const tot = ix.rb();   // pinned: the copies land without a staging hop
  HK_HIP(hipMemcpyAsync(&tot[0], ao + nt, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipMemcpyAsync(&tot[1], ho + nt, 8, hipMemcpyDeviceToHost, s));
  tot[2] = 0;
  if (d_flag) HK_HIP(hipMemcpyAsync(&tot[2], d_flag, 4, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (h_flag) *h_flag = (unsigned int)tot[2];
  return {tot[0], tot[1]};
}

template <typename V>
std::pair<uint64_t, uint64_t> refine_step(Index& ix, const KeyGeom& kg, const uint64_t* keys, const V* P,
                                          const uint32_t* J, uint64_t A, int cs, bool from_key, bool write_sa,
                                          V* oP, uint32_t* oJ, uint32_t* oG, uint32_t* head_slot,
                                          const unsigned int* d_flag = nullptr, unsigned int* h_flag = nullptr,
                                          uint8_t* oB = nullptr);

// One round's sort + regroup through LDS items of whole groups (hk_seground.hip).  The round's keys (G in the
// top bits) and positions are in keys[0] / vals[0], list act[cur]; the next list goes to act[cur ^ 1].  The
// big groups (over SR_W members) go first: their members gathered with their SA slots, radix-sorted on key
// bits [0, bits) and regrouped by the row kernels as a list of their own into the front of the next list;
// the items append after them.  mode 0: chunk refinement (SA of every slot, BWT of the settled), 1: doubling
// (ISA).  Returns the next list's (tied, groups).
template <typename V>
std::pair<uint64_t, uint64_t> seg_round(Index& ix, const KeyGeom& kg, int mode, int cur, uint64_t A, uint64_t groups,
                                        int bits, int ib, const uint8_t* lB = nullptr) {
  hipStream_t s = ix.stream;
  uint64_t* const k0 = ix.keys[0].as<uint64_t>();
  V* const v0 = ix.vals[0].as<V>();
  const uint32_t* G = ix.act[cur][2].as<uint32_t>();
  const uint32_t* J = ix.act[cur][1].as<uint32_t>();
  V* oP = ix.act[cur ^ 1][0].as<V>();
  uint32_t* oJ = ix.act[cur ^ 1][1].as<uint32_t>();
  uint32_t* oG = ix.act[cur ^ 1][2].as<uint32_t>();
  uint64_t nbg = 0;
  // the previous round wrote this list's group heads and window bounds when it produced this very list
  const bool ready = ix.sr_plan_g != nullptr && ix.sr_plan_g == ix.act[cur][2].p;
  ix.sr_plan_g = nullptr;
  const uint64_t B = sr_plan(ix, cur, G, A, groups, ready, &nbg);
  // links in the first doubling round only: every chain then runs through groups of that one round, so a linked
  // group's members share their chain (the group copy of lk_resolve relies on it); later rounds link far less
  const bool link = mode == 1 && ix.dbl.link && sizeof(V) == 4 && ix.dbl.ltag == 0 && ix.dbl.h <= lk_max_offset();
  if (link) lk_sizes(ix, cur, A, groups);   // (before the big groups' apply rewrites head_slot)
  std::pair<uint64_t, uint64_t> r0{0, 0};
  if (B) {
    const uint64_t nt = ceil_div(A, GR_TILE);
    ix.tile_b.ensure((nt + 1) * 4);
    ix.tile_a.ensure((nt + 2) * 8);
    const uint8_t* gbig = ix.grp_big.as<uint8_t>();
    {
      TimedLaunch tm(ix.timer, "sa_big_groups", (double)A * 5);
      k_big_count_rows<<<(unsigned)nt, GR_T, 0, s>>>(G, gbig, A, ix.tile_b.as<uint32_t>());
      HK_HIP(hipGetLastError());
    }
    scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nt, true, s);
    for (int i = 0; i < 2; ++i) {
      ix.big_k[i].ensure(B * 8 + 16);
      ix.big_v[i].ensure(B * sizeof(V) + 16);
    }
    ix.big_j.ensure(B * 4 + 16);
    uint64_t* bk[2] = {ix.big_k[0].as<uint64_t>(), ix.big_k[1].as<uint64_t>()};
    V* bv[2] = {ix.big_v[0].as<V>(), ix.big_v[1].as<V>()};
    {
      TimedLaunch tm(ix.timer, "sa_big_groups", (double)A * 5 + (double)B * (8 + 2 * sizeof(V) + 4 + 8));
      k_big_compact_rows<V><<<(unsigned)nt, GR_T, 0, s>>>(k0, v0, G, gbig, A, ix.tile_a.as<uint64_t>(), bk[0], bv[0],
                                                          ix.big_j.as<uint32_t>(), J);
      HK_HIP(hipGetLastError());
    }
    const int sl = radix_sort_pairs<V>(ix.sw, ix.timer, bk, bv, 0, B, 0, bits, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    if (mode == 0)
      r0 = refine_step<V>(ix, kg, bk[sl], bv[sl], ix.big_j.as<uint32_t>(), B, 0, false, true, oP, oJ, oG,
                          ix.head_slot.as<uint32_t>());
    else
      r0 = dbl_apply_list<V>(ix, bk[sl], bv[sl], ix.big_j.as<uint32_t>(), B, ib, true, nullptr, oP, oJ, oG);
    sr_heads(ix, cur ^ 1, oG, 0, r0.first, A, r0.second);   // (the items kernel writes the rest of the plan)
  }
  SrRoundArgs<V> a{};
  a.keys = k0;
  a.vals = v0;
  a.G = G;
  a.J = J;
  a.oP = oP;
  a.oJ = oJ;
  a.oG = oG;
  a.head_slot = ix.head_slot.as<uint32_t>();
  a.sa = ix.sa.as<V>();
  a.bwt = ix.bwt.as<uint8_t>();
  a.t = ix.text.as<uint8_t>();
  a.B = mode == 0 ? lB : nullptr;
  a.n = ix.n;
  a.isa = mode ? ix.isa.as<V>() : nullptr;
  a.lo = ix.sharded ? ix.shard_lo : 0;
  a.keep_same = 1;
  a.hp_next = ix.sr_hp[cur ^ 1].as<uint32_t>();
  a.win_next = ix.sr_win[cur ^ 1].as<uint32_t>();
  uint64_t linked = 0;
  if (link) {
    a.lnk = ix.lk_lnk.as<uint32_t>();
    a.gsz = ix.lk_gsz.as<uint8_t>();
    ix.dbl.lk_h = (uint32_t)ix.dbl.h;
    a.h = (uint32_t)ix.dbl.h;
    ++ix.dbl.ltag;
    a.ib = ib;
  }
  const std::pair<uint64_t, uint64_t> r = sr_items_round<V>(ix, mode, a, A, r0.first, r0.second, &linked);
  ix.sr_plan_g = ix.act[cur ^ 1][2].p;
  if (link) lk_after_round(ix, linked, (uint32_t)ix.dbl.h);
  return r;
}

// one doubling round over the active list: keys, sort, regroup.  Single GPU and one-GPU slices: the LDS item
// round (seg_round).  Sharded slices (the rank exchange needs every member's (position, ISA) pair in list
// order): groups of < 4 members on average sorted in place (seg_sort_groups), the few large ones by
// sort_big_groups, the round applied at once (its large-group flag rides in the read-back) and redone after
// sort_big_groups only if a large group was left — once one was, the next rounds read the flag first; larger
// average groups: the radix sort of the whole list.
template <typename V>
void dbl_round_t(Index& ix, uint64_t K) {
  auto& st = ix.dbl;
  hipStream_t s = ix.stream;
  const uint64_t A = st.A;
  const int cur = st.cur;
  const int gbits = st.groups > 1 ? bits_of_u64(st.groups - 1) : 0;
  const int ib = bits_of_u64(ix.n);   // ISA + 1 <= n
  if (gbits + ib > 64) throw ApiError{-6, "prefix doubling: too many tied groups for one 64-bit key"};
  // the output lists (a parked slice of build_sa_slices released them while it waited)
  ix.act[cur ^ 1][0].ensure(A * sizeof(V) + 16);
  ix.act[cur ^ 1][1].ensure(A * 4 + 16);
  ix.act[cur ^ 1][2].ensure(A * 4 + 16);
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  V* vp[2] = {ix.vals[0].as<V>(), ix.vals[1].as<V>()};
  {
    TimedLaunch tm(ix.timer, "sa_pair_keys", (double)A * (2 * sizeof(V) + 4 + 8 + sizeof(V)));
    k_dbl_keys<V><<<grid_for(A), 256, 0, s>>>(ix.act[cur][0].as<V>(), ix.act[cur][2].as<uint32_t>(), A,
                                              ix.isa.as<V>(), ix.n, st.h, ib, kp[0], vp[0],
                                              st.link ? ix.lk_lnk.as<uint32_t>() : nullptr, st.lk_h);
    HK_HIP(hipGetLastError());
  }
  std::pair<uint64_t, uint64_t> r{0, 0};
  const bool exchange = ix.sharded && !ix.slices_local;
  if (!exchange) {
    r = seg_round<V>(ix, KeyGeom{}, 1, cur, A, st.groups, gbits + ib, ib);
    st.npairs = 0;
  } else {
    ix.sr_plan_g = nullptr;
    const bool direct = A >= 4 * st.groups;
    unsigned int* d_big = reinterpret_cast<unsigned int*>(ix.small.as<uint8_t>() + 4356);   // small+4356: flag
    const uint32_t* G = ix.act[cur][2].as<uint32_t>();
    int sl = 0;
    bool spec = false;
    if (direct) {
      sl = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vp, 0, A, 0, gbits + ib, false, s);
      ix.info[0] += ix.sw.passes_run;
      ix.info[1] += ix.sw.passes_skipped;
    } else {
      seg_sort_groups<V>(ix, kp[0], vp[0], G, A, st.groups, d_big, "sa_pair_segsort");
      if (st.big) {
        uint64_t* const rb = ix.rb();
        rb[2] = 0;
        HK_HIP(hipMemcpyAsync(&rb[2], d_big, 4, hipMemcpyDeviceToHost, s));
        HK_HIP(hipStreamSynchronize(s));
        st.big = (uint32_t)rb[2] != 0;
        if (st.big) sort_big_groups<V>(ix, kp[0], vp[0], G, A, gbits + ib);
      } else {
        spec = true;
      }
    }
    ix.upd.ensure(A * 16 + 16);
    uint64_t* pairs = ix.upd.as<uint64_t>();
    V* oP = ix.act[cur ^ 1][0].as<V>();
    uint32_t* oJ = ix.act[cur ^ 1][1].as<uint32_t>();
    uint32_t* oG = ix.act[cur ^ 1][2].as<uint32_t>();
    const uint32_t* J = ix.act[cur][1].as<uint32_t>();
    unsigned int h_big = 0;
    // keep_same: skip the ISA entries a round leaves unchanged (pairs carry every entry anyway)
    r = dbl_apply_list<V>(ix, kp[sl], vp[sl], J, A, ib, true, pairs, oP, oJ, oG, spec ? d_big : nullptr, &h_big);
    if (spec && h_big) {   // a group over SEG_MAX members was left unsorted: redo the round
      st.big = true;
      // (the redo rewrites every pair, list entry and group head of the first attempt; an SA / BWT slot it
      // wrote for a suffix it wrongly took as settled is rewritten by the slot's final owner)
      sort_big_groups<V>(ix, kp[0], vp[0], G, A, gbits + ib);
      r = dbl_apply_list<V>(ix, kp[0], vp[0], J, A, ib, false, pairs, oP, oJ, oG);
    }
    st.npairs = A;
  }
  st.cur ^= 1;
  st.A = r.first;
  st.groups = r.second;
  st.h += K;
  ix.info.push_back(st.A);
  ix.info[2] += 1ull << 32;
}

// one refinement grouping step (stats + scans + apply); returns (tied, groups)
template <typename V>
std::pair<uint64_t, uint64_t> refine_step(Index& ix, const KeyGeom& kg, const uint64_t* keys, const V* P,
                                          const uint32_t* J, uint64_t A, int cs, bool from_key, bool write_sa,
                                          V* oP, uint32_t* oJ, uint32_t* oG, uint32_t* head_slot,
                                          const unsigned int* d_flag, unsigned int* h_flag, uint8_t* oB) {
  hipStream_t s = ix.stream;
  const uint64_t nt = ceil_div(A, GR_TILE);
  ix.tile_b.ensure((nt + 1) * 4);
  ix.tile_c.ensure((nt + 1) * 4);
  ix.tile_a.ensure((nt + 2) * 8);
  ix.tile_d.ensure((nt + 2) * 8);
  {
    TimedLaunch tm(ix.timer, "sa_refine_stats", (double)A * 8);
    k_refine_stats_rows<<<(unsigned)nt, GR_T, 0, s>>>(keys, A, cs, ix.tile_b.as<uint32_t>(), ix.tile_c.as<uint32_t>());
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nt, true, s);
  scan_exclusive_u32_to_u64(ix.sw, ix.tile_c.as<uint32_t>(), ix.tile_d.as<uint64_t>(), nt, true, s);
  uint8_t* bwt = ix.bwt.as<uint8_t>();
  const uint8_t* inv = ix.small.as<uint8_t>() + 3072;
  {
    TimedLaunch tm(ix.timer, "sa_refine_apply", (double)A * (8 + sizeof(V) + (write_sa ? sizeof(V) + 4 : 0) + 1));
    if (from_key)
      k_refine_apply_rows<V, true><<<(unsigned)nt, GR_T, 0, s>>>(
          keys, P, J, A, cs, ix.tile_a.as<uint64_t>(), ix.tile_d.as<uint64_t>(), write_sa ? ix.sa.as<V>() : nullptr,
          bwt, inv, (1ull << kg.pb) - 1, ix.text.as<uint8_t>(), ix.n, oP, oJ, oG, head_slot, oB);
    else
      k_refine_apply_rows<V, false><<<(unsigned)nt, GR_T, 0, s>>>(
          keys, P, J, A, cs, ix.tile_a.as<uint64_t>(), ix.tile_d.as<uint64_t>(), write_sa ? ix.sa.as<V>() : nullptr,
          bwt, inv, 0, ix.text.as<uint8_t>(), ix.n, oP, oJ, oG, head_slot, nullptr);
    HK_HIP(hipGetLastError());
  }
  uint64_t* const tot = ix.rb();
  HK_HIP(hipMemcpyAsync(&tot[0], ix.tile_a.as<uint64_t>() + nt, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipMemcpyAsync(&tot[1], ix.tile_d.as<uint64_t>() + nt, 8, hipMemcpyDeviceToHost, s));
  if (d_flag) {   // a caller's device flag rides in the same round trip
    tot[2] = 0;
    HK_HIP(hipMemcpyAsync(&tot[2], d_flag, 4, hipMemcpyDeviceToHost, s));
  }
  HK_HIP(hipStreamSynchronize(s));
  if (h_flag) *h_flag = d_flag ? (unsigned int)tot[2] : 0u;
  return {tot[0], tot[1]};
}

}  // namespace

// ---------------------------------------------------------------- geometry
int mixed_radix_bits(uint64_t R, int q) {
  unsigned __int128 p = 1;
  for (int i = 0; i < q; ++i) {
    p *= R;
    if (p > ((unsigned __int128)1 << 64)) return 65;
  }
  p -= 1;
  int b = 0;
  while (p) {
    ++b;
    p >>= 1;
  }
  return b;
}

// Symbols per key: minimise (radix passes) * n + 30 * (expected tied suffixes), the latter from the
// iid collision rate sum(p_c^2)^q of the symbol histogram (ties are refined, not wrong — this only
// decides speed; texts with repeats tie more, refinement/doubling absorb that).
KeyGeom key_geometry(Index& ix, bool with_prev) {
  compute_alphabet(ix);
  KeyGeom g{};
  g.R = (uint64_t)ix.sigma + 1;
  int pbits = 1;
  while ((1 << pbits) < ix.sigma + 1) ++pbits;
  g.pb = with_prev ? pbits : 0;
  double p2 = 0;
  const double n = (double)(ix.n ? ix.n : 1);
  for (int c = 0; c < 256; ++c) p2 += ((double)ix.byte_hist[c] / n) * ((double)ix.byte_hist[c] / n);
  double best = 1e300;
  for (int q = 1; q <= 64; ++q) {
    const int sb = mixed_radix_bits(g.R, q);
    if (g.pb + sb > 64) break;
    const double ties = std::min(n, n * n * std::pow(p2, (double)q));
    const double cost = (double)((sb + 7) / 8) * n + 30.0 * ties;   // a tie costs ~30 element-passes (measured)
    if (cost <= best) {
      best = cost;
      g.q = q;
      g.sym_bits = sb;
    }
  }
  g.key_bits = g.pb + g.sym_bits;
  for (int c = 0; c < 256; ++c) g.lut[c] = ix.code_of[c] < 0 ? 0 : (uint16_t)(ix.code_of[c] + 1);
  memset(g.inv, 0, sizeof(g.inv));
  for (int k = 0; k < ix.sigma; ++k) g.inv[k + 1] = ix.syms[k];
  return g;
}

// device copies of the LUTs: small+2048 = lut (u16[256]), small+3072 = inv (u8[512])
void upload_geometry(Index& ix, const KeyGeom& kg) {
  ix.small.ensure(8192);
  if (kg.keyed) {   // small+2560 = lutk, +4608 = lutp (u16[256]), +3584 = skey (u64[72]), +7168 = srank (u32[72])
    // +7456 = k2d (u16[256]); the ranges in between (4096: locate / fallback counters, 5120: digit
    // histogram) are reset by their users before use.  Staged in pinned memory: one upload.
    if (ix.geom_ev) HK_HIP(hipEventSynchronize(ix.geom_ev));   // the previous upload has read the staging
    ix.small_host.ensure(8192 + 128);   // (after the wait: a regrowth would free the staging in flight)
    uint8_t* hs = ix.small_host.as<uint8_t>();
    memcpy(hs + 2048, kg.lut, 512);
    memcpy(hs + 3072, kg.inv, 512);
    memcpy(hs + 2560, kg.lutk, 512);
    memcpy(hs + 4608, kg.lutp, 512);
    memcpy(hs + 3584, kg.skey, sizeof(kg.skey));
    memcpy(hs + 7168, kg.srank, sizeof(kg.srank));
    memcpy(hs + 7456, kg.k2d, sizeof(kg.k2d));
    static_assert(7456 + sizeof(kg.k2d) <= 8192, "geometry tables fit the small buffer");
    HK_HIP(hipMemcpyAsync(ix.small.as<uint8_t>() + 2048, hs + 2048, 7456 + sizeof(kg.k2d) - 2048,
                          hipMemcpyHostToDevice, ix.stream));
    // no wait here: the next upload (or histogram landing) waits for this event before reusing the staging
    if (!ix.geom_ev) HK_HIP(hipEventCreateWithFlags(&ix.geom_ev, hipEventDisableTiming));
    HK_HIP(hipEventRecord(ix.geom_ev, ix.stream));
  } else {
    HK_HIP(hipMemcpyAsync(ix.small.as<uint8_t>() + 2048, kg.lut, 512, hipMemcpyHostToDevice, ix.stream));
    HK_HIP(hipMemcpyAsync(ix.small.as<uint8_t>() + 3072, kg.inv, 512, hipMemcpyHostToDevice, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));   // kg may be a host temporary
  }
}

template <typename V>
void refine_loop(Index& ix, const KeyGeom& kg, int cur, uint64_t A, uint64_t groups, bool allow_doubling,
                 const uint8_t* B0);

// Refinement of tied groups after the initial sort of m suffixes (their sorted keys in keys[slot],
// positions in vals[slot] — which the caller has adopted as ix.sa).  With allow_doubling (single
// GPU, u32 positions) the loop switches to ISA-based prefix doubling after kChunkRounds rounds.
template <typename V>
void refine_after_sort(Index& ix, const KeyGeom& kg, int slot, uint64_t m, bool allow_doubling) {
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  for (int i = 0; i < 2; ++i) {
    ix.act[i][0].ensure(m * sizeof(V) + 16);
    ix.act[i][1].ensure(m * 4 + 16);
    ix.act[i][2].ensure(m * 4 + 16);
  }
  ix.head_slot.ensure(m * 4 + 16);
  ix.bwt.ensure(m + 64);
  // initial round: keys compared without the prev field; SA already in place; BWT from keys
  // (the tied suffixes' BWT bytes, from the keys' prev field, travel with the list into the first chunk round)
  ix.act_b.ensure(m + 16);
  auto r0 = refine_step<V>(ix, kg, kp[slot], ix.sa.as<V>(), nullptr, m, kg.pb, true, false,
                           ix.act[0][0].as<V>(), ix.act[0][1].as<uint32_t>(), ix.act[0][2].as<uint32_t>(),
                           ix.head_slot.as<uint32_t>(), nullptr, nullptr, ix.act_b.as<uint8_t>());
  ix.info.push_back(r0.first);
  refine_loop<V>(ix, kg, 0, r0.first, r0.second, allow_doubling, ix.act_b.as<uint8_t>());
}

// The tied suffixes (P, J = SA slot, G = dense group ordinal in list order: whole groups in any order,
// each one's slots contiguous and ascending along the list) are in act[cur];
// each round sorts them by (G, next symbols from offset h) and re-groups.
template <typename V>
void refine_loop(Index& ix, const KeyGeom& kg, int cur, uint64_t A, uint64_t groups, bool allow_doubling,
                 const uint8_t* B0) {
  hipStream_t s = ix.stream;
  ix.sr_plan_g = nullptr;   // (the list in act[cur] came from another producer)
  const uint16_t* d_lut = reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048);
  const uint32_t* d_srank = reinterpret_cast<const uint32_t*>(ix.small.as<uint8_t>() + 7168);
  const uint64_t s_start = kg.keyed ? kg.s_start : ~0ull;
  const uint32_t nS = kg.keyed ? kg.nS : 0u;
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  V* vp[2] = {ix.vals[0].as<V>(), ix.vals[1].as<V>()};
  uint64_t h = (uint64_t)kg.q;
  int rounds = 0;
  uint64_t A_prev = 0;
  const bool local_dbl = allow_doubling || ix.slices_local;   // doubling needs no rank exchange here
  const uint64_t m_all = ix.sharded ? ix.shard_hi - ix.shard_lo : ix.n;
  while (A > 0 && rounds < kChunkRounds) {
    // after the first chunk round (it also places the short suffixes), a round that settled under two fifths
    // of its tied suffixes, or a list still holding over a quarter of all suffixes (natural-language text:
    // 108M of 200M), hands over to prefix doubling: a doubling round doubles the compared prefix for one
    // ISA gather per suffix, a chunk round reads the next chunk of T' per suffix (1 GiB protein-like text:
    // handing over after one chunk round instead of four, 142.5 -> 134.1 ms per build)
    if (local_dbl && rounds > 0 && (A * 5 > A_prev * 3 || A > m_all / 4)) break;
    int gbits = 0;
    while (gbits < 64 && (1ull << gbits) < groups) ++gbits;
    auto fits = [&](int qq) {   // G in the top gbits, chunk + nS (<= R^qq - 1 + nS) below
      if (mixed_radix_bits(kg.R, qq) > 64 - gbits) return false;
      unsigned __int128 top = 1;
      for (int i = 0; i < qq; ++i) top *= kg.R;
      top = top - 1 + nS;
      return top < ((unsigned __int128)1 << (64 - gbits));
    };
    int qn = 0;
    while (qn < 64 && fits(qn + 1)) ++qn;
    if (qn < 1) break;   // too many groups for a chunk key: prefix doubling takes over
    ++rounds;
    A_prev = A;
    {
      TimedLaunch tm(ix.timer, "sa_refine_keys", (double)A * (sizeof(V) * 2 + 4 + 8));
      k_refine_keys<V><<<grid_for(A), 256, 0, s>>>(ix.act[cur][0].as<V>(), ix.act[cur][2].as<uint32_t>(), A,
                                                   ix.text.as<uint8_t>(), ix.n, d_lut, kg.R, qn, gbits, h, kp[0],
                                                   vp[0], s_start, nS, d_srank);
      HK_HIP(hipGetLastError());
    }
    // sort inside each group + regroup: LDS items of whole groups, the groups of over SR_W members by a
    // global radix sort first (seg_round)
    // (B0: the BWT bytes of this list, the first round's only)
    const std::pair<uint64_t, uint64_t> r = seg_round<V>(ix, kg, 0, cur, A, groups, 64, 0, rounds == 1 ? B0 : nullptr);
    cur ^= 1;
    A = r.first;
    groups = r.second;
    ix.info.push_back(A);
    h += (uint64_t)qn;
  }
  ix.info[2] = (uint64_t)rounds;
  ix.dbl = Index::DblState{};
  if (A == 0) return;
  // ---- prefix doubling from order h over the A tied suffixes (repetitive texts)
  ix.dbl.cur = cur;
  ix.dbl.A = A;
  ix.dbl.groups = groups;
  ix.dbl.h = h;
  ix.dbl.pending = true;
  if (!allow_doubling) {   // sharded slice: the rank exchange drives the rounds (hk_shard.hip)
    if (!ix.slices_local) dbl_emit_groups(ix);   // (one-GPU slices: emitted once the full ISA exists)
    return;
  }
  // single GPU: ISA of every position from the full SA, tied suffixes at their head's slot
  dbl_ensure_isa(ix);
  if (!ix.sharded && !ix.sa_pos64 && ix.n < 0xFFFFFFFFull && ix.n >= (1ull << 16)) {
    dbl_isa_init_single(ix);
    // links (hk_seground.hpp; ISA values < 2^31 leave the top bit for the link mark) pay where long repeats keep
    // suffixes tied for many rounds: English-like 200 MiB (108M of 200M reach doubling) 67.7 -> 64.8 ms; on
    // protein-like 1 GiB (256M of 1G, shorter repeats) they cost 13 ms more than the rounds they save
    const bool many = ix.dbl.A * 3 >= ix.n;
    ix.dbl.link = ix.n < (1ull << 31) && !(ix.flags & kFlagNoLinks) && (many || (ix.flags & kFlagLinks));
    if (ix.dbl.link) lk_begin(ix);
  } else {
    dbl_isa_segment(ix, ix.sa.p, ix.n, 0);
    dbl_emit_groups(ix);
  }
  int drounds = 0;
  while (ix.dbl.A > 0) {
    if (++drounds > 64) throw ApiError{-7, "prefix doubling did not converge"};
    dbl_round(ix, ix.dbl.h);
  }
  if (ix.dbl.link) {
    lk_resolve(ix);
    ix.dbl.link = false;
  }
  ix.dbl.pending = false;
}

template void refine_after_sort<uint32_t>(Index&, const KeyGeom&, int, uint64_t, bool);
template void refine_after_sort<uint64_t>(Index&, const KeyGeom&, int, uint64_t, bool);
std::pair<uint64_t, uint64_t> refine_step_u32(Index& ix, const KeyGeom& kg, const uint64_t* keys,
                                              const uint32_t* P, const uint32_t* J, uint64_t A, int cs,
                                              uint32_t* oP, uint32_t* oJ, uint32_t* oG) {
  return refine_step<uint32_t>(ix, kg, keys, P, J, A, cs, false, true, oP, oJ, oG, ix.head_slot.as<uint32_t>());
}

template void refine_loop<uint32_t>(Index&, const KeyGeom&, int, uint64_t, uint64_t, bool, const uint8_t*);
template void refine_loop<uint64_t>(Index&, const KeyGeom&, int, uint64_t, uint64_t, bool, const uint8_t*);

// ---------------------------------------------------------------- prefix doubling steps
void dbl_ensure_isa(Index& ix) { ix.isa.ensure(ix.n * (ix.sa_pos64 ? 8 : 4) + 16); }

void dbl_isa_segment(Index& ix, const void* d_sa, uint64_t count, uint64_t lo) {
  if (!count) return;
  if (lo + count > ix.n) throw ApiError{-4, "ISA segment out of range"};
  TimedLaunch tm(ix.timer, "sa_isa_scatter", (double)count * (ix.sa_pos64 ? 16 : 8));
  if (ix.sa_pos64)
    k_isa_from_sa<uint64_t><<<grid_for(count), 256, 0, ix.stream>>>(static_cast<const uint64_t*>(d_sa), count, lo,
                                                                     ix.isa.as<uint64_t>());
  else
    k_isa_from_sa<uint32_t><<<grid_for(count), 256, 0, ix.stream>>>(static_cast<const uint32_t*>(d_sa), count, lo,
                                                                     ix.isa.as<uint32_t>());
  HK_HIP(hipGetLastError());
}

// ISA at the switch to doubling on one GPU (u32 positions, not sharded): see k_pos_part
void dbl_isa_init_single(Index& ix) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  auto& st = ix.dbl;
  uint32_t* hs = ix.vals[0].as<uint32_t>();   // (free until the first round's keys)
  uint64_t* p1 = ix.keys[1].as<uint64_t>();
  uint64_t* p2 = ix.keys[0].as<uint64_t>();
  ix.sr_cnt.ensure(64);
  uint32_t* err = reinterpret_cast<uint32_t*>(ix.sr_cnt.as<uint8_t>() + 48);
  HK_HIP(hipMemsetAsync(err, 0, 4, s));
  {
    TimedLaunch tm(ix.timer, "sa_isa_scatter", (double)n * 4 + (double)st.A * 12);
    fill_iota<uint32_t>(hs, n, s);
    if (st.A)
      k_hs_tied<<<grid_for(st.A), 256, 0, s>>>(ix.act[st.cur][1].as<uint32_t>(), ix.act[st.cur][2].as<uint32_t>(), st.A,
                                                ix.head_slot.as<uint32_t>(), hs, n, st.groups, err);
    HK_HIP(hipGetLastError());
  }
  const int lgn = bits_of_u64(n - 1);
  const int s_hi = std::max(lgn - 8, 13);                    // level-1 buckets (<= 256), >= one tile each
  const int s_lo = std::max(std::min(s_hi - 1, PW_MAX), s_hi - 10);   // sub-buckets: <= 2^14 positions, <= 1024 per bucket
  if (s_lo > PW_MAX) throw ApiError{-6, "ISA init: text too long for the position scatter"};
  const uint64_t nb1 = ceil_div(n, 1ull << s_hi), nb2 = ceil_div(n, 1ull << s_lo);
  ix.tile_c.ensure(nb2 * 8 + 16);
  unsigned long long* cur = ix.tile_c.as<unsigned long long>();
  {
    TimedLaunch tm(ix.timer, "sa_isa_scatter", (double)n * (4 + 4 + 8));
    k_pos_cursors<<<(unsigned)std::min<uint64_t>(ceil_div(nb1, 256), 4096), 256, 0, s>>>(
        reinterpret_cast<uint64_t*>(cur), nb1, s_hi);
    k_pos_part<1><<<(unsigned)ceil_div(n, PP_TILE), PP_T, 0, s>>>(ix.sa.as<uint32_t>(), hs, nullptr, n, s_hi, s_lo, cur,
                                                                   p1, err);
    HK_HIP(hipGetLastError());
  }
  {
    TimedLaunch tm(ix.timer, "sa_isa_scatter", (double)n * 16);
    k_pos_cursors<<<(unsigned)std::min<uint64_t>(ceil_div(nb2, 256), 4096), 256, 0, s>>>(
        reinterpret_cast<uint64_t*>(cur), nb2, s_lo);
    const uint64_t tpb = (1ull << s_hi) / PP_TILE;
    k_pos_part<2><<<(unsigned)(nb1 * tpb), PP_T, 0, s>>>(nullptr, nullptr, p1, n, s_hi, s_lo, cur, p2, err);
    HK_HIP(hipGetLastError());
  }
  {
    TimedLaunch tm(ix.timer, "sa_isa_scatter", (double)n * (8 + 4));
    k_pos_write<<<(unsigned)nb2, 512, 0, s>>>(p2, n, s_lo, ix.isa.as<uint32_t>(), err);
    HK_HIP(hipGetLastError());
  }
  uint64_t* const rb = ix.rb();
  rb[3] = 0;
  HK_HIP(hipMemcpyAsync(&rb[3], err, 4, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if ((uint32_t)rb[3]) throw ApiError{-7, "prefix doubling: the SA handed to the ISA scatter is not a permutation"};
}

void dbl_emit_groups(Index& ix) {
  auto& st = ix.dbl;
  const uint64_t A = st.A;
  uint64_t* pairs = nullptr;
  if (ix.sharded && !ix.slices_local) {
    ix.upd.ensure(A * 16 + 16);
    pairs = ix.upd.as<uint64_t>();
  }
  const uint64_t lo = ix.sharded ? ix.shard_lo : 0;
  if (A) {
    if (ix.sa_pos64)
      k_dbl_emit<uint64_t><<<grid_for(A), 256, 0, ix.stream>>>(ix.act[st.cur][0].as<uint64_t>(),
                                                               ix.act[st.cur][2].as<uint32_t>(), A,
                                                               ix.head_slot.as<uint32_t>(), lo, ix.isa.as<uint64_t>(),
                                                               pairs);
    else
      k_dbl_emit<uint32_t><<<grid_for(A), 256, 0, ix.stream>>>(ix.act[st.cur][0].as<uint32_t>(),
                                                               ix.act[st.cur][2].as<uint32_t>(), A,
                                                               ix.head_slot.as<uint32_t>(), lo, ix.isa.as<uint32_t>(),
                                                               pairs);
    HK_HIP(hipGetLastError());
  }
  st.npairs = pairs ? A : 0;
  HK_HIP(hipStreamSynchronize(ix.stream));
}

void dbl_apply_pairs(Index& ix, const uint64_t* d_pairs, uint64_t count) {
  if (!count) return;
  TimedLaunch tm(ix.timer, "sa_isa_update", (double)count * (16 + (ix.sa_pos64 ? 8 : 4)));
  if (ix.sa_pos64)
    k_dbl_apply_pairs<uint64_t><<<grid_for(count), 256, 0, ix.stream>>>(d_pairs, count, ix.isa.as<uint64_t>());
  else
    k_dbl_apply_pairs<uint32_t><<<grid_for(count), 256, 0, ix.stream>>>(d_pairs, count, ix.isa.as<uint32_t>());
  HK_HIP(hipGetLastError());
}

void dbl_round(Index& ix, uint64_t K) {
  if (!ix.dbl.A) return;
  if (K == 0) throw ApiError{-1, "prefix doubling: K must be positive"};
  if (ix.sa_pos64) dbl_round_t<uint64_t>(ix, K);
  else dbl_round_t<uint32_t>(ix, K);
}

void pack_keys(const uint8_t* d_text, uint64_t n, uint64_t lo, uint64_t count, const uint16_t* d_lut, uint64_t R,
               int q, int pb, uint64_t* d_keys, hipStream_t s, uint64_t* d_hist0) {
  if (d_hist0) HK_HIP(hipMemsetAsync(d_hist0, 0, 256 * 8, s));
  if (!count) return;
  const uint64_t g = std::min<uint64_t>(ceil_div(count, PK_TILE), 4096);
  const KeyChunks kc = key_chunks(R, q);
  k_pack_keys<<<(unsigned)g, 256, 0, s>>>(d_text, n, lo, count, d_lut, R, q, pb, kc.ck, kc.Rck, kc.Rlast, d_keys,
                                          reinterpret_cast<unsigned long long*>(d_hist0));
  HK_HIP(hipGetLastError());
}

void synth_text(uint8_t* d_text, uint64_t n, const uint8_t* alphabet, int sigma, uint64_t seed,
                uint8_t terminator, hipStream_t s) {
  Alpha256 al{};
  for (int i = 0; i < sigma; ++i) al.s[i] = alphabet[i];
  k_synth<<<grid_for(n), 256, 0, s>>>(d_text, n, al, sigma, seed, terminator);
  HK_HIP(hipGetLastError());
}

__global__ __launch_bounds__(256) void k_widen_u32(const uint32_t* __restrict__ in, uint64_t* __restrict__ out,
                                                   uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) out[i] = in[i];
}

// SA[lo, lo + c) as u64 into a host buffer: widened on the GPU in 32M-entry chunks (device staging),
// each chunk copied straight into the caller's buffer (no host-side conversion pass)
void sa_to_host_u64(Index& ix, uint64_t lo, uint64_t c, uint64_t* out) {
  hipStream_t s = ix.stream;
  constexpr uint64_t CH = 1ull << 25;
  DevBuf tmp;
  tmp.ensure(std::min<uint64_t>(c, CH) * 8);
  for (uint64_t o = 0; o < c; o += CH) {
    const uint64_t k = std::min<uint64_t>(CH, c - o);
    k_widen_u32<<<grid_for(k, 256, 8192), 256, 0, s>>>(ix.sa.as<uint32_t>() + lo + o, tmp.as<uint64_t>(), k);
    HK_HIP(hipGetLastError());
    HK_HIP(hipMemcpyAsync(out + o, tmp.p, k * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
  }
}

// byte counts of T'[lo, hi) (lo a multiple of 16) into d_out[256] (u64)
void byte_hist_range(Index& ix, uint64_t lo, uint64_t hi, unsigned long long* d_out) {
  hipStream_t s = ix.stream;
  HK_HIP(hipMemsetAsync(d_out, 0, 256 * 8, s));
  if (hi <= lo) return;
  TimedLaunch t(ix.timer, "byte_hist", (double)(hi - lo));
  // every counter copy (4 lanes of the workgroup) stays below 2^16: <= 8192 bytes per lane
  const uint64_t cap = std::max<uint64_t>(2048, ceil_div(hi - lo, (uint64_t)256 * 8192));
  k_byte_hist<<<(unsigned)std::min<uint64_t>(ceil_div((hi - lo) / 16 + 1, (uint64_t)256), cap), 256, 0, s>>>(
      ix.text.as<uint8_t>() + lo, hi - lo, d_out);
  HK_HIP(hipGetLastError());
}

// alphabet, C over bytes and dense codes from the byte histogram (utils/utils.py:16-24)
void set_alphabet(Index& ix, const uint64_t* h) {
  for (int b = 0; b < 256; ++b) ix.byte_hist[b] = h[b];
  ix.sigma = 0;
  uint64_t acc = 0;
  for (int b = 0; b < 256; ++b) {
    ix.Cbyte[b] = acc;
    acc += ix.byte_hist[b];
    ix.code_of[b] = -1;
    if (ix.byte_hist[b]) {
      ix.Ccode[ix.sigma] = ix.Cbyte[b];
      ix.code_of[b] = (int16_t)ix.sigma;
      ix.syms[ix.sigma++] = (uint8_t)b;
    }
  }
  ix.Cbyte[256] = acc;
  ix.Ccode[ix.sigma] = acc;
  ix.have_alpha = true;
}

void compute_alphabet(Index& ix) {
  if (ix.have_alpha) return;
  hipStream_t s = ix.stream;
  ix.small.ensure(8192);
  byte_hist_range(ix, 0, ix.n, ix.small.as<unsigned long long>());
  // both read-backs land in pinned slots (a pageable destination costs a staged, synchronous copy each)
  if (ix.geom_ev) HK_HIP(hipEventSynchronize(ix.geom_ev));   // (before any regrowth of the staging)
  ix.small_host.ensure(8192 + 128);
  uint8_t* const hs = ix.small_host.as<uint8_t>();
  HK_HIP(hipMemcpyAsync(hs, ix.small.p, 256 * 8, hipMemcpyDeviceToHost, s));
  // the text's last bytes (the keyed geometry's short suffixes) in the same round trip
  const uint64_t nt = std::min<uint64_t>(ix.n, 70);
  if (nt) HK_HIP(hipMemcpyAsync(hs + 8192, ix.text.as<uint8_t>() + (ix.n - nt), nt, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (nt) memcpy(ix.tail, hs + 8192, nt);
  uint64_t h[256];
  memcpy(h, hs, sizeof(h));
  ix.tail_valid = nt > 0;
  set_alphabet(ix, h);
}

void build_sa(Index& ix) {
  if (ix.n >= 0xFFFFFFFFull || (ix.flags & kFlagSlices)) {   // 64-bit positions: slices (hk_shard.hip)
    build_sa_slices(ix, slices_for(ix));
    return;
  }
  if (!(ix.flags & kFlagGlobalSort)) {
    build_sa_bucketed(ix);
    return;
  }
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
  // the prev field needs (q+1) symbols per key; for very small alphabets this still leaves q >= 20
  KeyGeom kg = key_geometry(ix, true);
  upload_geometry(ix, kg);
  ix.info[3] = (uint64_t)kg.q;
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(n * 8 + 16);
    ix.vals[i].ensure(n * 4 + 16);
  }
  uint64_t* d_hist0 = ix.small.as<uint64_t>() + 640;   // byte 5120 of the scratch
  {
    TimedLaunch t(ix.timer, "sa_pack_keys", (double)n * 9);
    pack_keys(ix.text.as<uint8_t>(), n, 0, n, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048),
              kg.R, kg.q, kg.pb, ix.keys[0].as<uint64_t>(), s, d_hist0);
  }
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  uint32_t* vp[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
  int slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, n, kg.pb, kg.key_bits, true, s, d_hist0);
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  // the sorted values are the SA candidate order: adopt that buffer as SA
  std::swap(ix.sa, ix.vals[slot]);
  ix.vals[slot].ensure(n * 4 + 16);
  refine_after_sort<uint32_t>(ix, kg, slot, n, true);
  HK_HIP(hipStreamSynchronize(s));
  ix.have_sa = true;
  ix.have_bwt = true;
}

void build_bwt(Index& ix) {
  if (!ix.have_sa) throw ApiError{-3, "build_bwt: suffix array not built"};
  if (ix.have_bwt) return;   // produced together with the SA
  if (ix.sharded) throw ApiError{-3, "build_bwt: sharded index holds only a slice"};
  ix.bwt.ensure(ix.n + 64);
  {
    TimedLaunch t(ix.timer, "bwt_gather", (double)ix.n * (4 + 1 + 1));
    k_bwt<<<grid_for(ix.n), 256, 0, ix.stream>>>(ix.text.as<uint8_t>(), ix.sa.as<uint32_t>(), ix.n,
                                                 ix.bwt.as<uint8_t>());
    HK_HIP(hipGetLastError());
  }
  HK_HIP(hipStreamSynchronize(ix.stream));
  ix.have_bwt = true;
}

void bwt_gather64(Index& ix, const uint64_t* d_sa) {
  ix.bwt.ensure(ix.n + 64);
  k_bwt64<<<grid_for(ix.n), 256, 0, ix.stream>>>(ix.text.as<uint8_t>(), d_sa, ix.n, ix.bwt.as<uint8_t>());
  HK_HIP(hipGetLastError());
}

void release_workspace(Index& ix) {
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].release();
    ix.vals[i].release();
    ix.seq[i].release();
    for (int k = 0; k < 3; ++k) ix.act[i][k].release();
    if (i == 0) ix.act_b.release();
  }
  ix.isa.release();
  ix.head_slot.release();
  ix.tile_a.release();
  ix.tile_b.release();
  ix.tile_c.release();
  ix.tile_d.release();
  ix.tile_e.release();
  ix.upd.release();
  ix.cp_part.release();
  ix.sel.release();
  ix.cp_cur.release();
  ix.cp_tiles.release();
  ix.sw.status.release();
  ix.sw.status_tiles = 0;
  ix.sw.scan_tmp.release();
  for (int i = 0; i < 2; ++i) {
    ix.big_k[i].release();
    ix.big_v[i].release();
  }
  ix.big_j.release();
  ix.grp_big.release();
  for (DevBuf* b : {&ix.sr_hp[0], &ix.sr_hp[1], &ix.sr_win[0], &ix.sr_win[1], &ix.sr_items, &ix.sr_cnt, &ix.lk_lnk,
                    &ix.lk_gsz, &ix.lk_tops, &ix.lk_grec})
    b->release();
  ix.sr_plan_g = nullptr;
  ix.fused.reset();
  ix.fused_recs.release();
  ix.fused_ws.release();
  ix.fused_host.release();
}

}  // namespace hk
