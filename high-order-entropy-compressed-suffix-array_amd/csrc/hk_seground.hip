// hk_seground.hip — the sort + regroup step of one refinement (chunk) round or prefix-doubling round over
// the tie list: each tied group is ordered by its members' next symbols / ISA[p + h]
// (csa/suffix_array.py:131-134 orders suffixes by their whole text; the rounds extend the compared prefix).
//
// The tie list holds whole groups: G = dense group ordinal, ascending along the list; the members' SA
// slots J are contiguous and ascending along the list.  A round's keys (the caller's key kernel: G in the
// top bits, the next chunk or ISA[p + h] + 1 below) only need ordering INSIDE each group, so instead of
// radix-sorting the whole list over every key bit (8 global passes over ~10^8 pairs on natural-language
// text) the list is cut into items of whole groups:
//   * windows of SR_W list entries; item w = the groups whose head lies in window w, except a last group of
//     more than SR_W members (a "big" group, k_sr_items) — so an item holds fewer than 2 * SR_W entries;
//   * one workgroup per item (k_sr_round): the item's keys and positions are staged in LDS and sorted there
//     — one thread per group when no group has more than SR_NET (8) members (pairs dominate late doubling rounds),
//     else stable LSD passes of 8 bits over only the bits that vary inside the item — then regrouped in
//     the same workgroup: settled suffixes write their SA / BWT entries, tied ones are appended to the
//     next list through one 64-bit atomic per item (entries | groups << 33, so both are reserved in one
//     operation and G stays ascending along the new list), doubling rounds write ISA;
//   * big groups: gathered, radix-sorted in global memory and regrouped by the row kernels (hk_sa.hip)
//     into the front of the next list, before the items append.
// The round's work is then one read and one write of the list plus LDS work, instead of a full radix
// sort plus a grouping pass.

#include "hk_index.hpp"
#include "hk_seground.hpp"

namespace hk {
namespace {

constexpr int SR_T = 512;
constexpr int SR_E = SR_CAP / SR_T;   // 8 entries per thread
constexpr int SR_NW = SR_T / 64;
// the largest group a thread sorts in registers (bitonic network); an item with a larger group takes the LDS
// radix passes.  8, not 16: the 16-key network needs 113-123 VGPRs, over the 80 that three workgroups per CU allow
constexpr int SR_NET = 8;
constexpr uint32_t SR_NONE = 0xFFFFFFFFu;

// heads: hp[G[a]] = a; first / last head of every window w (win[2w], win[2w + 1])
// (over list entries [lo, hi), lo a multiple of SR_HB — the list's front, or all of it).  Four entries per
// thread (one 16-byte load), the predecessor of a thread's first entry from the lane below, and one atomic
// pair per block of SR_HB entries (a block lies in one window): the per-wave atomics on the same two words
// serialised at the L2
constexpr uint32_t SR_HB = 1024;
static_assert(SR_W % SR_HB == 0, "a heads block lies in one window");
__global__ __launch_bounds__(256) void k_sr_heads(const uint32_t* __restrict__ G, uint64_t lo, uint64_t hi,
                                                  uint32_t* __restrict__ hp, uint32_t* __restrict__ win) {
  __shared__ uint32_t rmin[4], rmax[4];
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (uint64_t b = lo + (uint64_t)blockIdx.x * SR_HB; b < hi; b += (uint64_t)gridDim.x * SR_HB) {   // (uniform)
    const uint64_t a0 = b + 4ull * threadIdx.x;
    uint32_t g[4];
    if (a0 + 4 <= hi) {
      const uint4 v = *reinterpret_cast<const uint4*>(G + a0);
      g[0] = v.x;
      g[1] = v.y;
      g[2] = v.z;
      g[3] = v.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] = a0 + k < hi ? G[a0 + k] : 0u;
    }
    // the entry before a0: the lane below's last, lane 0 from memory
    uint32_t prev = __shfl_up(g[3], 1, 64);
    if (lane == 0 && a0 > 0 && a0 - 1 < hi) prev = G[a0 - 1];
    uint32_t fmin = SR_NONE, fmax = 0;
    bool any = false;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t a = a0 + k;
      const uint32_t before = k ? g[k - 1] : prev;
      if (a < hi && (a == 0 || before != g[k])) {
        hp[g[k]] = (uint32_t)a;
        fmin = fmin == SR_NONE ? (uint32_t)a : fmin;
        fmax = (uint32_t)a;
        any = true;
      }
    }
    const uint64_t m = ballot64(any);
    if (lane == 0) {
      rmin[wv] = SR_NONE;
      rmax[wv] = 0;
    }
    if (m) {
      const uint32_t lf = (uint32_t)__builtin_ctzll(m), ll = 63u - (uint32_t)__builtin_clzll(m);
      const uint32_t vmin = __shfl(fmin, (int)lf, 64), vmax = __shfl(fmax, (int)ll, 64);
      if (lane == 0) {
        rmin[wv] = vmin;
        rmax[wv] = vmax;
      }
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      uint32_t bmin = SR_NONE, bmax = 0;
      bool found = false;
      for (int w = 0; w < 4; ++w)
        if (rmin[w] != SR_NONE) {
          bmin = bmin == SR_NONE ? rmin[w] : bmin;
          bmax = rmax[w];
          found = true;
        }
      if (found) {
        const uint64_t w0 = b / SR_W;
        atomicMin(win + 2 * w0, bmin);
        atomicMax(win + 2 * w0 + 1, bmax);
      }
    }
    __syncthreads();
  }
}

// items[w] = {first entry, entries}; a window's last group of more than SR_W members is big: flagged in
// gbig, counted (cnt[0] entries, cnt[1] groups) and left out of the item
__global__ __launch_bounds__(256) void k_sr_items(const uint32_t* __restrict__ G, const uint32_t* __restrict__ hp,
                                                  uint64_t groups, uint64_t A, const uint32_t* __restrict__ win, uint64_t nw,
                                                  uint2* __restrict__ items, uint8_t* __restrict__ gbig,
                                                  unsigned long long* __restrict__ cnt, uint2* __restrict__ win_next) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256) {
    win_next[w] = make_uint2(SR_NONE, 0u);   // (the next list has at most as many windows)
    const uint32_t ws = win[2 * w];
    if (ws == SR_NONE) {
      items[w] = make_uint2(0u, 0u);
      continue;
    }
    const uint32_t wl = win[2 * w + 1];
    const uint32_t g = G[wl];
    const uint64_t end = (uint64_t)g + 1 < groups ? (uint64_t)hp[g + 1] : A;
    uint64_t we = end;
    if (end - wl > (uint64_t)SR_W) {
      gbig[g] = 1;
      atomicAdd(cnt, (unsigned long long)(end - wl));
      atomicAdd(cnt + 1, 1ull);
      we = wl;
    }
    items[w] = make_uint2(ws, (uint32_t)(we - ws));
  }
}

struct alignas(16) SrShared {
  uint64_t key[SR_CAP];             // the item's keys (entry order; the sort permutes idx); then per-position
                                    // regroup records (section 3)
  union {
    uint32_t g[SR_CAP];             // group ordinals, while the head mask is built
    uint16_t idx[2][SR_CAP];        // the order being sorted (entry indexes)
  } u;
  uint64_t hmask[SR_CAP / 64];      // bit i: a group starts at entry i (set past the item's end too)
  uint32_t whist[SR_NW][256];       // per-wave digit counts -> per-wave exclusive digit offsets
  union {
    uint64_t mtab[SR_NW][256];      // per-wave match masks (zero between uses)
    uint32_t pl[SR_CAP];            // after the sort: u32 positions in entry order
  } m;
  uint64_t lkall[SR_CAP / 64];      // doubling links: bit i = entry i's group is linked
  uint32_t lcnt, lgc;
  unsigned long long lgbase;
  uint32_t tstart[256];             // item-local exclusive digit start
  uint32_t wtot[SR_NW];
  uint64_t wor[SR_NW], wand[SR_NW];
  uint32_t wbig[SR_NW];
  uint32_t wmax[SR_NW], wcnt[SR_NW];
  uint32_t nwmin[4], nwmax[4];      // next list: first / last group head of each window this item's chunk touches
  uint64_t obase, gbase;
};

// bitonic network over N (key, entry) registers, the group's sz <= N members padded with ~0 keys
template <int N>
__device__ __forceinline__ void sr_net(const uint64_t* __restrict__ key, uint16_t* __restrict__ out, uint32_t i0,
                                       uint32_t sz) {
  uint64_t k[N];
  uint32_t e[N];
#pragma unroll
  for (int j = 0; j < N; ++j) {
    k[j] = (uint32_t)j < sz ? key[i0 + j] : ~0ull;
    e[j] = i0 + (uint32_t)j;
  }
#pragma unroll
  for (int size = 2; size <= N; size <<= 1) {
#pragma unroll
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
#pragma unroll
      for (int j = 0; j < N; ++j) {
        const int l = j ^ stride;
        if (l > j) {
          const bool up = (j & size) == 0;
          const bool sw = up ? k[j] > k[l] : k[j] < k[l];
          const uint64_t kj = k[j], kl = k[l];
          const uint32_t ej = e[j], el = e[l];
          k[j] = sw ? kl : kj;
          k[l] = sw ? kj : kl;
          e[j] = sw ? el : ej;
          e[l] = sw ? ej : el;
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < N; ++j)
    if ((uint32_t)j < sz) out[i0 + j] = (uint16_t)e[j];
}

__device__ __forceinline__ bool sr_head(const uint64_t* hm, uint32_t i) { return (hm[i >> 6] >> (i & 63)) & 1ull; }

// the next group head after entry i (the bits past the item's end are set)
__device__ __forceinline__ uint32_t sr_next_head(const uint64_t* hm, uint32_t i) {
  uint32_t w = (i + 1) >> 6;
  uint64_t b = hm[w] & (~0ull << ((i + 1) & 63));
  while (!b) b = hm[++w];
  return (w << 6) + (uint32_t)__builtin_ctzll(b);
}

// the group head at or before entry i (entry 0 is a head)
__device__ __forceinline__ uint32_t sr_prev_head(const uint64_t* hm, uint32_t i) {
  uint32_t w = i >> 6;
  uint64_t b = hm[w] & ((2ull << (i & 63)) - 1ull);
  while (!b) b = hm[--w];
  return (w << 6) + 63u - (uint32_t)__builtin_clzll(b);
}

// regroup record of a sorted position (section 3): run start, tied index, group index inside the item, flags
constexpr int RG_TIED = 36, RG_RH = 37, RG_FIRST = 38;

// MODE 0: chunk refinement round (every slot's SA entry written, settled suffixes' BWT); MODE 1: prefix
// doubling round (ISA of every member = its new group's head slot; SA / BWT of the settled ones)
template <typename V, int MODE>
__global__ __launch_bounds__(SR_T, 6) void k_sr_round(SrRoundArgs<V> a) {
  __shared__ SrShared sh;
  const uint2 it = a.items[blockIdx.x];
  const uint32_t m = it.y;
  if (m == 0) return;
  const uint64_t base = it.x;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  // ---- 1. stage (striped: entry k * SR_T + tid), the head mask, the varying key bits, group sizes.  The
  // entry's SA slot (and its u32 position) stay in registers until the write-out: no dependent load there
  constexpr bool P32 = sizeof(V) == 4;
  const bool links = P32 && MODE == 1 && a.lnk != nullptr;
  uint64_t kor = 0, kand = ~0ull;
  uint32_t jr[SR_E], pr[SR_E];
  const bool hasB = MODE == 0 && a.B != nullptr;
  uint32_t bq[(SR_E + 3) / 4] = {};   // the entries' BWT bytes (hasB), four per register
#pragma unroll
  for (int k = 0; k < SR_E; ++k) {
    const uint32_t i = (uint32_t)k * SR_T + tid;
    jr[k] = 0;
    pr[k] = 0;
    if (i < m) {
      const uint64_t key = a.keys[base + i];
      sh.key[i] = key;
      sh.u.g[i] = a.G[base + i];
      jr[k] = a.J[base + i];
      if constexpr (P32) pr[k] = (uint32_t)a.vals[base + i];
      if (hasB) bq[k >> 2] |= (uint32_t)a.B[base + i] << (8 * (k & 3));
      kor |= key;
      kand &= key;
    }
  }
  if (tid < 4) {
    sh.nwmin[tid] = SR_NONE;
    sh.nwmax[tid] = 0;
  }
  if (links) {
    if (tid < SR_CAP / 64) sh.lkall[tid] = 0;
    if (tid == 0) {
      sh.lcnt = 0;
      sh.lgc = 0;
    }
  }
  __syncthreads();
  uint32_t big = 0;
#pragma unroll
  for (int k = 0; k < SR_E; ++k) {
    const uint32_t i = (uint32_t)k * SR_T + tid;
    const bool h = i >= m || i == 0 || sh.u.g[i] != sh.u.g[i - 1];
    const uint64_t hb = ballot64(h);
    if (lane == 0) sh.hmask[i >> 6] = hb;
    if (i < m && i >= SR_NET && sh.u.g[i] == sh.u.g[i - SR_NET]) big = 1;   // a group of more than SR_NET members
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    kor |= __shfl_xor(kor, o, 64);
    kand &= __shfl_xor(kand, o, 64);
  }
  big = ballot64(big != 0) ? 1u : 0u;
  if (lane == 0) {
    sh.wor[wv] = kor;
    sh.wand[wv] = kand;
    sh.wbig[wv] = big;
  }
  __syncthreads();   // (every read of u.g is done: idx may overwrite it)
  // link candidates: a group head whose key names a tied group (ISA[p + h] + 1 > 0) of the same size
  // (gsz ^ size == 0); whether all its keys are equal is read off the sorted order below
  uint32_t lg[SR_E];
#pragma unroll
  for (int k = 0; k < SR_E; ++k) {
    const uint32_t i = (uint32_t)k * SR_T + tid;
    lg[k] = 1;
    if (links && i < m && sr_head(sh.hmask, i)) {
      const uint32_t sz = sr_next_head(sh.hmask, i) - i;
      const uint64_t kl = sh.key[i] & ((1ull << a.ib) - 1);
      if (sz >= 2 && sz < 255 && kl && kl <= a.n) lg[k] = (uint32_t)a.gsz[kl - 1] ^ sz;
    }
  }
  kor = 0;
  kand = ~0ull;
  big = 0;
#pragma unroll
  for (int w = 0; w < SR_NW; ++w) {
    kor |= sh.wor[w];
    kand &= sh.wand[w];
    big |= sh.wbig[w];
  }
  const uint64_t vary = kor ^ kand;
  int cur = 0;
#pragma unroll
  for (int k = 0; k < SR_E; ++k) {   // every entry first takes its own place
    const uint32_t i = (uint32_t)k * SR_T + tid;
    if (i < m) sh.u.idx[0][i] = (uint16_t)i;
  }

  // ---- 2. sort the item's groups (entries stay inside their group's range: G is in the keys' top bits)
  if (!big) {
    __syncthreads();
    for (uint32_t i = tid; i < m; i += SR_T) {
      if (!sr_head(sh.hmask, i)) continue;
      const uint32_t sz = sr_next_head(sh.hmask, i) - i;
      if (sz == 2) {
        if (sh.key[i + 1] < sh.key[i]) {
          sh.u.idx[0][i] = (uint16_t)(i + 1);
          sh.u.idx[0][i + 1] = (uint16_t)i;
        }
      } else if (sz > 2 && sz <= 4) {
        sr_net<4>(sh.key, sh.u.idx[0], i, sz);
      } else if (sz > 4) {
        sr_net<SR_NET>(sh.key, sh.u.idx[0], i, sz);
      }
    }
  } else if (vary) {
    const int lo = __builtin_ctzll(vary), hi = 64 - __builtin_clzll(vary);
    for (uint32_t i = tid; i < (uint32_t)SR_NW * 256; i += SR_T) (&sh.m.mtab[0][0])[i] = 0;
    for (int shf = lo; shf < hi; shf += 8) {
      if (((vary >> shf) & 255u) == 0) continue;   // (uniform: a digit with no varying bit orders nothing)
      if (tid < 256) {
#pragma unroll
        for (int w = 0; w < SR_NW; ++w) sh.whist[w][tid] = 0;
      }
      __syncthreads();
      // rank inside the wave (stable: wave-contiguous positions, item-major then lane), as k_onesweep
      uint32_t rk[SR_E];
      uint64_t* const mt = sh.m.mtab[wv];
#pragma unroll
      for (int k = 0; k < SR_E; ++k) {
        const uint32_t pos = wv * (SR_E * 64) + (uint32_t)k * 64 + lane;
        const bool valid = pos < m;
        const uint32_t id = valid ? sh.u.idx[cur][pos] : 0u;
        const uint32_t d = valid ? (uint32_t)(sh.key[id] >> shf) & 255u : 0u;
        if (valid) __hip_atomic_fetch_or(mt + d, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint64_t msk = __hip_atomic_load(mt + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        const uint32_t below = mbcnt(msk);
        const uint32_t prior = sh.whist[wv][d];
        if (valid && below == 0) {
          __hip_atomic_store(mt + d, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          sh.whist[wv][d] = prior + (uint32_t)__popcll(msk);
        }
        rk[k] = (prior + below) | (d << 10) | (id << 18);   // rank < 512, digit, entry < 4096
      }
      __syncthreads();
      if (wv < 4) {   // per digit (thread = digit): wave prefixes, then the item-local exclusive start
        uint32_t run = 0;
#pragma unroll
        for (int w = 0; w < SR_NW; ++w) {
          const uint32_t c = sh.whist[w][tid];
          sh.whist[w][tid] = run;
          run += c;
        }
        const uint32_t inc = dpp_incl_sum(run);
        if (lane == 63) sh.wtot[wv] = inc;
        sh.tstart[tid] = inc - run;
      }
      __syncthreads();
      if (wv < 4) {
        uint32_t carry = 0;
#pragma unroll
        for (int w = 0; w < 4; ++w) carry += (uint32_t)w < wv ? sh.wtot[w] : 0u;
        sh.tstart[tid] += carry;
      }
      __syncthreads();
#pragma unroll
      for (int k = 0; k < SR_E; ++k) {
        const uint32_t pos = wv * (SR_E * 64) + (uint32_t)k * 64 + lane;
        if (pos < m) {
          const uint32_t d = (rk[k] >> 10) & 255u;
          sh.u.idx[cur ^ 1][sh.tstart[d] + sh.whist[wv][d] + (rk[k] & 1023u)] = (uint16_t)(rk[k] >> 18);
        }
      }
      __syncthreads();   // (the next pass resets whist / tstart and reads this order)
      cur ^= 1;
    }
  }
  __syncthreads();
  const uint16_t* const ord = sh.u.idx[cur];
  // (the other order buffer is free now: it takes the BWT bytes in entry order)
  uint8_t* const bst = reinterpret_cast<uint8_t*>(sh.u.idx[cur ^ 1]);
  if (P32 || hasB) {   // (the match masks are done with: their space takes the positions)
#pragma unroll
    for (int k = 0; k < SR_E; ++k) {
      const uint32_t i = (uint32_t)k * SR_T + tid;
      if (i < m) {
        if constexpr (P32) sh.m.pl[i] = pr[k];
        if (hasB) bst[i] = (uint8_t)(bq[k >> 2] >> (8 * (k & 3)));
      }
    }
    __syncthreads();
  }
  if constexpr (P32 && MODE == 1) {
    if (links) {   // a stuck candidate (first and last sorted keys equal) is linked by its head thread
#pragma unroll
      for (int k = 0; k < SR_E; ++k) {
        const uint32_t i = (uint32_t)k * SR_T + tid;
        if (lg[k] == 0) {
          const uint32_t sz = sr_next_head(sh.hmask, i) - i;
          lg[k] = ~0u;
          if (sh.key[ord[i]] == sh.key[ord[i + sz - 1]]) {
            lg[k] = atomicAdd(&sh.lgc, 1u);   // (the group's record index inside the item)
            for (uint32_t b = i; b < i + sz;) {
              const uint32_t lo = b & 63u, c = min(64u - lo, i + sz - b);
              const uint64_t msk = (c == 64u ? ~0ull : ((1ull << c) - 1ull)) << lo;
              atomicOr(reinterpret_cast<unsigned long long*>(&sh.lkall[b >> 6]), (unsigned long long)msk);
              b += c;
            }
            atomicAdd(&sh.lcnt, sz);
          }
        }
      }
      __syncthreads();
      if (tid == 0 && sh.lcnt) {
        atomicAdd(a.lcount, (unsigned long long)sh.lcnt);
        sh.lgbase = atomicAdd(a.gcount, (unsigned long long)sh.lgc);
      }
      // every linked entry writes its own link (striped: the stores of a wave go out together): the group's
      // head slot is this entry's slot minus its distance to the head, K = its key (all equal in the group)
#pragma unroll
      for (int k = 0; k < SR_E; ++k) {
        const uint32_t i = (uint32_t)k * SR_T + tid;
        if (i < m && ((sh.lkall[i >> 6] >> (i & 63)) & 1ull)) {
          const uint32_t gh = sr_prev_head(sh.hmask, i);
          const uint32_t K = (uint32_t)(sh.key[i] & ((1ull << a.ib) - 1)) - 1u;
          const uint32_t p = sh.m.pl[i];
          a.lnk[p] = jr[k] - (i - gh) - K;   // (!= 0: another group's head; the ISA mark comes with the tiles)
        }
      }
      __syncthreads();
      if (sh.lcnt) {
#pragma unroll
        for (int k = 0; k < SR_E; ++k) {
          const uint32_t i = (uint32_t)k * SR_T + tid;
          // (a linked group's head: its lg[k] is the record index)
          if (i < m && sr_head(sh.hmask, i) && ((sh.lkall[i >> 6] >> (i & 63)) & 1ull)) {
            const uint32_t sz = sr_next_head(sh.hmask, i) - i;
            a.grec[sh.lgbase + lg[k]] = make_uint4(jr[k], sz, sh.m.pl[i], 0u);
          }
        }
      }
    }
  }

  // ---- 3. regroup.  (a) blocked (thread tid owns positions [tid * SR_E, tid * SR_E + SR_E)): run heads, tied
  // flags and the item-wide scans (max of run-head positions, tied | tied heads << 16); (b) the per-position
  // regroup records into the key plane; (c) striped: every global access coalesced across the wave
  const uint32_t p0 = tid * SR_E;
  uint32_t flags = 0;          // bit j: run head at p0 + j; bit 16 + j: tied
  uint32_t lmax = 0, lcnt = 0;
  {
    uint64_t prev = p0 > 0 && p0 < m ? sh.key[ord[p0 - 1]] : 0;
    bool have_prev = p0 > 0 && p0 < m;
    uint64_t kc = p0 < m ? sh.key[ord[p0]] : 0;
#pragma unroll
    for (int j = 0; j < SR_E; ++j) {
      const uint32_t i = p0 + (uint32_t)j;
      if (i < m) {
        const uint64_t kn = i + 1 < m ? sh.key[ord[i + 1]] : 0;
        const bool rh = !have_prev || kc != prev;
        const bool re = i + 1 >= m || kn != kc;
        const bool lk = links && ((sh.lkall[i >> 6] >> (i & 63)) & 1ull);   // (linked: neither tied nor settled)
        const bool tied = !lk && !(rh && re);
        if (rh) {
          flags |= 1u << j;
          lmax = i;
        }
        if (tied) {
          flags |= 1u << (16 + j);
          lcnt += rh ? 0x10001u : 1u;
        }
        prev = kc;
        have_prev = true;
        kc = kn;
      }
    }
  }
  const uint32_t imax = dpp_scan_u32(lmax, 0u, [](uint32_t x, uint32_t y) { return x > y ? x : y; });
  const uint32_t icnt = dpp_incl_sum(lcnt);
  if (lane == 63) {
    sh.wmax[wv] = imax;
    sh.wcnt[wv] = icnt;
  }
  __syncthreads();   // (also: every read of the key plane is done)
  uint32_t cmax = 0, ccnt = 0, tcnt = 0;
#pragma unroll
  for (int w = 0; w < SR_NW; ++w) {
    if ((uint32_t)w < wv) {
      cmax = cmax > sh.wmax[w] ? cmax : sh.wmax[w];
      ccnt += sh.wcnt[w];
    }
    tcnt += sh.wcnt[w];
  }
  // exclusive within the wave: the previous lane's inclusive value (wave_shr:1)
  const uint32_t pmax_w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)imax, 0x138, 0xf, 0xf, false);
  const uint32_t pcnt_w = (uint32_t)__builtin_amdgcn_update_dpp(0, (int)icnt, 0x138, 0xf, 0xf, false);
  uint32_t rmax = cmax > pmax_w ? cmax : pmax_w;
  uint32_t rcnt = ccnt + pcnt_w;
#pragma unroll
  for (int j = 0; j < SR_E; ++j) {
    const uint32_t i = p0 + (uint32_t)j;
    if (i >= m) break;
    const bool rh = (flags >> j) & 1u;
    const bool tied = (flags >> (16 + j)) & 1u;
    if (rh) rmax = i;
    if (tied && rh) rcnt += 0x10000u;
    // run start | tied index | group index inside the item | tied | run head | run starts its group
    sh.key[i] = (uint64_t)rmax | ((uint64_t)(rcnt & 0xFFFFu) << 12) | ((uint64_t)((rcnt >> 16) - (tied ? 1u : 0u)) << 24) |
                ((uint64_t)tied << RG_TIED) | ((uint64_t)rh << RG_RH) | ((uint64_t)sr_head(sh.hmask, rmax) << RG_FIRST);
    if (tied) rcnt += 1;
  }
  if (tid == 0) {
    const unsigned long long inc = (unsigned long long)(tcnt & 0xFFFFu) |
                                   ((unsigned long long)(tcnt >> 16) << 33);
    const unsigned long long old = atomicAdd(a.counter, inc);
    sh.obase = a.base_e + (old & ((1ull << 33) - 1));   // (after the big groups' entries / groups)
    sh.gbase = a.base_g + (old >> 33);
  }
  __syncthreads();
  const uint64_t obase = sh.obase, gbase = sh.gbase;
  const uint64_t w0 = obase / SR_W;
#pragma unroll
  for (int k = 0; k < SR_E; ++k) {
    const uint32_t i = (uint32_t)k * SR_T + tid;
    if (i < m) {
      if (links && ((sh.lkall[i >> 6] >> (i & 63)) & 1ull)) continue;
      const uint64_t r = sh.key[i];
      const uint32_t rs = (uint32_t)r & 0xFFFu;
      const bool tied = (r >> RG_TIED) & 1u, rh = (r >> RG_RH) & 1u;
      uint64_t p;
      if constexpr (P32) p = sh.m.pl[ord[i]];
      else p = (uint64_t)a.vals[base + ord[i]];
      const uint32_t slot = jr[k];   // (slots are contiguous inside a group: the run start's is slot - (i - rs))
      if (MODE == 1) {
        if (!(a.keep_same && ((r >> RG_FIRST) & 1u))) a.isa[p] = (V)(a.lo + (uint64_t)(slot - (i - rs)));
      } else if (a.sa) {
        a.sa[slot] = (V)p;   // (every slot: prefix doubling builds its ISA from this SA)
      }
      if (tied) {
        const uint64_t o = obase + ((r >> 12) & 0xFFFu);
        const uint64_t g = gbase + ((r >> 24) & 0xFFFu);
        a.oP[o] = (V)p;
        a.oJ[o] = slot;
        a.oG[o] = (uint32_t)g;
        if (rh) {
          a.head_slot[g] = slot;
          if (a.hp_next) {   // the next round's plan: this group's head, the windows' first / last heads
            a.hp_next[g] = (uint32_t)o;
            const uint32_t wl = (uint32_t)(o / SR_W - w0);
            atomicMin(&sh.nwmin[wl], (uint32_t)o);
            atomicMax(&sh.nwmax[wl], (uint32_t)o);
          }
        }
      } else {
        if (MODE == 1) a.sa[slot] = (V)p;
        a.bwt[slot] = hasB ? bst[ord[i]] : a.t[p == 0 ? a.n - 1 : p - 1];
      }
    }
  }
  if (a.hp_next) {
    __syncthreads();
    if (tid < 4 && sh.nwmin[tid] != SR_NONE) {
      atomicMin(a.win_next + 2 * (w0 + tid), sh.nwmin[tid]);
      atomicMax(a.win_next + 2 * (w0 + tid) + 1, sh.nwmax[tid]);
    }
  }
}

// ---- doubling links (see SrRoundArgs): the size of every tied group at its head slot, the chains of one round's
// links (ISA(p) = ISA(p + off) + delta composes), the SA / BWT entries of the linked groups at the end

__global__ __launch_bounds__(256) void k_lk_sizes(const uint32_t* __restrict__ head_slot, const uint32_t* __restrict__ hp,
                                                  uint64_t groups, uint64_t A, uint64_t n, uint8_t* __restrict__ gsz) {
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < groups; g += (uint64_t)gridDim.x * 256) {
    const uint64_t e = g + 1 < groups ? (uint64_t)hp[g + 1] : A;
    const uint32_t s = head_slot[g];
    if (s < n) gsz[s] = (uint8_t)(e - hp[g] < 255 ? e - hp[g] : 255);
  }
}

// The links of one round all have offset h, so their chains run down the columns of the positions laid out in
// rows of h.  A tile of R = LT_POS / h rows resolves every chain inside it in LDS: each column is split into
// segments, each walked bottom-up by one thread (run rows / summed delta, open when the run reaches the segment
// bottom), then the segments' carries are chained per column.  A run that reaches the tile bottom continues at
// the next tile's top row: those tile tops (ntiles x h entries) are pointer-jumped as a small array and added to
// the open runs afterwards (k_lk_open_fix).  One dense pass instead of log(chain) passes over every position.
constexpr int LT_T = 256;
constexpr uint32_t LT_POS = 4096;   // (25 KB of LDS: six tile workgroups per CU; links need h <= LT_POS)
constexpr uint32_t LT_OPEN = 0x80000000u, LT_OPEN16 = 0x8000u;   // (run rows <= LT_POS < 2^15)

__device__ __forceinline__ uint64_t lk_cv(uint32_t k, uint32_t d, bool open) {
  return ((uint64_t)(k | (open ? LT_OPEN : 0u)) << 32) | d;
}

__global__ __launch_bounds__(LT_T) void k_lk_tile(uint32_t* __restrict__ isa, uint32_t* __restrict__ lnk,
                                                  uint64_t n, uint32_t h, uint32_t R,
                                                  uint64_t* __restrict__ tops) {
  __shared__ uint32_t Dd[LT_POS];
  __shared__ uint16_t Kk[LT_POS];   // run rows from this row down (LT_OPEN16: reaches the segment bottom), 0: unlinked
  __shared__ uint64_t cin[LT_T];    // carry into each (column, segment) from below
  const uint32_t tid = threadIdx.x;
  const uint64_t base = (uint64_t)blockIdx.x * R * h;
  const uint32_t T = R * h;
  for (uint32_t i = tid; i < T; i += LT_T) {
    const uint64_t p = base + i;
    bool f = false;
    uint32_t d = 0;
    if (p < n) {   // (linked in this round: a nonzero slot delta; the lnk plane was zeroed)
      d = lnk[p];
      f = d != 0;
    }
    Kk[i] = f ? 1 : 0;
    Dd[i] = d;
  }
  __syncthreads();
  const uint32_t S = h < (uint32_t)LT_T ? (uint32_t)LT_T / h : 1u;   // segments per column
  const uint32_t RS = (R + S - 1) / S;                                // rows per segment
  for (uint32_t w = tid; w < h * S; w += LT_T) {
    const uint32_t c = w / S, sg = w % S;
    const uint32_t r0 = sg * RS, r1 = min(R, r0 + RS);
    uint32_t k = 0, d = 0;
    bool open = true;
    for (uint32_t r = r1; r-- > r0;) {
      const uint32_t i = r * h + c;
      if (Kk[i]) {
        k += 1;
        d += Dd[i];
        Kk[i] = (uint16_t)(k | (open ? LT_OPEN16 : 0u));
        Dd[i] = d;
      } else {
        k = 0;
        d = 0;
        open = false;
      }
    }
  }
  __syncthreads();
  if (S > 1) {   // (h < LT_T: h * S <= LT_T carries)
    for (uint32_t c = tid; c < h; c += LT_T) {
      uint64_t carry = lk_cv(0, 0, true);
      for (uint32_t sg = S; sg-- > 0;) {
        cin[c * S + sg] = carry;
        const uint32_t r0 = sg * RS;
        if (r0 >= R) continue;
        const uint32_t i = r0 * h + c;
        const uint32_t kv = Kk[i];
        if (!kv) {
          carry = lk_cv(0, 0, false);
        } else if (kv & LT_OPEN16) {
          const uint32_t ck = (uint32_t)(carry >> 32);
          carry = lk_cv((kv & ~LT_OPEN16) + (ck & ~LT_OPEN), Dd[i] + (uint32_t)carry, (ck & LT_OPEN) != 0);
        } else {
          carry = lk_cv(kv, Dd[i], false);
        }
      }
    }
  }
  __syncthreads();
  for (uint32_t w = tid; w < h * S; w += LT_T) {
    const uint32_t c = w / S, sg = w % S;
    const uint64_t cr = S > 1 ? cin[c * S + sg] : lk_cv(0, 0, true);
    const uint32_t crk = (uint32_t)(cr >> 32);
    const uint32_t r0 = sg * RS, r1 = min(R, r0 + RS);
    for (uint32_t r = r0; r < r1; ++r) {
      const uint32_t i = r * h + c;
      const uint32_t kv = Kk[i];
      if (!kv) {
        if (r == 0) tops[(uint64_t)blockIdx.x * h + c] = 0;
        continue;
      }
      uint32_t k = kv & ~LT_OPEN16, d = Dd[i];
      bool open = false;
      if (kv & LT_OPEN16) {
        k += crk & ~LT_OPEN;
        d += (uint32_t)cr;
        open = (crk & LT_OPEN) != 0;
      }
      isa[base + i] = LK_BIT | k;   // k hops of h (open: to the next tile's top row of this column)
      lnk[base + i] = d;
      if (r == 0) tops[(uint64_t)blockIdx.x * h + c] = lk_cv(k, d, open);
    }
  }
}

// tile tops: (k | open, d) per (tile, column); an open entry continues at the entry h further.  Wyllie pointer
// jumping with ping-pong buffers: acc (k, d) and the next entry (~0: none)
__global__ __launch_bounds__(256) void k_lk_tops_init(const uint64_t* __restrict__ tops, uint64_t m, uint32_t h,
                                                      uint64_t* __restrict__ acc, uint64_t* __restrict__ nxt) {
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
    const uint64_t v = tops[e];
    const uint32_t k = (uint32_t)(v >> 32);
    acc[e] = ((uint64_t)(k & ~LT_OPEN) << 32) | (uint32_t)v;
    nxt[e] = (k & LT_OPEN) && e + h < m ? e + h : ~0ull;
  }
}

__global__ __launch_bounds__(256) void k_lk_tops_jump(const uint64_t* __restrict__ acc, const uint64_t* __restrict__ nxt,
                                                      uint64_t m, uint64_t* __restrict__ acc2, uint64_t* __restrict__ nxt2,
                                                      unsigned int* __restrict__ flag) {
  bool any = false;
  for (uint64_t e = (uint64_t)blockIdx.x * 256 + threadIdx.x; e < m; e += (uint64_t)gridDim.x * 256) {
    uint64_t a = acc[e], x = nxt[e];
    if (x != ~0ull) {
      const uint64_t b = acc[x];
      a = ((((a >> 32) + (b >> 32)) & 0xFFFFFFFFull) << 32) | (uint32_t)((uint32_t)a + (uint32_t)b);
      x = nxt[x];
      any = true;
    }
    acc2[e] = a;
    nxt2[e] = x;
  }
  if (ballot64(any) && (threadIdx.x & 63) == 0) atomicOr(flag, 1u);
}

// runs that reached their tile's bottom: add the resolved top of the next tile in their column
__global__ __launch_bounds__(256) void k_lk_open_fix(uint32_t* __restrict__ isa, uint32_t* __restrict__ lnk,
                                                     uint64_t n, uint32_t h, uint32_t R,
                                                     const uint64_t* __restrict__ acc, uint64_t m) {
  const uint64_t T = (uint64_t)R * h;
  // four positions per thread (one 16-byte load of the ISA marks); most positions are unlinked or closed
  const uint64_t nq = (n + 3) / 4;
  for (uint64_t qd = (uint64_t)blockIdx.x * 256 + threadIdx.x; qd < nq; qd += (uint64_t)gridDim.x * 256) {
    const uint64_t p0 = 4 * qd;
    uint32_t v[4];
    if (p0 + 4 <= n) {
      const uint4 w = *reinterpret_cast<const uint4*>(isa + p0);
      v[0] = w.x; v[1] = w.y; v[2] = w.z; v[3] = w.w;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = p0 + k < n ? isa[p0 + k] : 0u;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint64_t p = p0 + k;
      if (!(v[k] & LK_BIT)) continue;
      const uint64_t hops = v[k] & ~LK_BIT;
      const uint64_t q = p + hops * h;
      const uint64_t t = p / T;
      if (q < (t + 1) * T) continue;   // closed inside the tile
      const uint64_t e = (t + 1) * h + (p % T) % h;
      if (e >= m) continue;            // (never: a run cannot leave the text)
      const uint64_t b = acc[e];
      isa[p] = LK_BIT | (uint32_t)(hops + (b >> 32));
      lnk[p] += (uint32_t)b;
    }
  }
}

// a linked group's slice of the SA is its chain end's slice shifted by the chain's offset: the members' images
// p + OFF are unlinked suffixes whose final slots are [s - D, s - D + size) (f(p) = ISA(p + OFF) + D maps the
// members onto [s, s + size)), and with links from one round only every member shares the head's {OFF, D}
__global__ __launch_bounds__(256) void k_lk_resolve(const uint4* __restrict__ grec, uint64_t g0, uint64_t g1,
                                                    const uint32_t* __restrict__ lnk, const uint32_t* __restrict__ isa,
                                                    uint32_t h, const uint8_t* __restrict__ t,
                                                    uint64_t n, uint32_t* __restrict__ sa, uint8_t* __restrict__ bwt,
                                                    unsigned int* __restrict__ flag) {
  bool bad = false;
  for (uint64_t g = g0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; g < g1; g += (uint64_t)gridDim.x * 256) {
    const uint4 r = grec[g];
    const uint32_t v = isa[r.z];
    const uint64_t off64 = (uint64_t)(v & ~LK_BIT) * h;
    const uint32_t off = (uint32_t)off64, ke = r.x - lnk[r.z];
    if (!(v & LK_BIT) || off64 >= n || (uint64_t)ke + r.y > n || (uint64_t)r.x + r.y > n) {
      bad = true;
      continue;
    }
    for (uint32_t i0 = 0; i0 < r.y; i0 += 4) {   // four members' loads in flight together
      uint32_t p[4];
      uint8_t b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) p[j] = i0 + j < r.y ? sa[ke + i0 + j] : off;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bad |= p[j] < off;
        p[j] = p[j] < off ? 0u : p[j] - off;
        b[j] = i0 + j < r.y ? t[p[j] == 0 ? n - 1 : p[j] - 1] : (uint8_t)0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (i0 + j < r.y) {
          sa[r.x + i0 + j] = p[j];
          bwt[r.x + i0 + j] = b[j];
        }
    }
  }
  if (ballot64(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 2u);
}

}  // namespace

// ---------------------------------------------------------------- host
namespace {
// window bounds of a list of up to A entries: {first head (none: ~0), last head} per window
__global__ __launch_bounds__(256) void k_sr_win_reset(uint2* __restrict__ win, uint64_t nw) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nw; w += (uint64_t)gridDim.x * 256)
    win[w] = make_uint2(SR_NONE, 0u);
}
}  // namespace

static void sr_windows_reset(Index& ix, int slot, uint64_t A) {
  const uint64_t nw = ceil_div(A, (uint64_t)SR_W);
  ix.sr_win[slot].ensure(nw * 8 + 16);
  if (!nw) return;
  k_sr_win_reset<<<(unsigned)std::min<uint64_t>(ceil_div(nw, 256), 4096), 256, 0, ix.stream>>>(
      ix.sr_win[slot].as<uint2>(), nw);
  HK_HIP(hipGetLastError());
}

void sr_heads(Index& ix, int slot, const uint32_t* G, uint64_t lo, uint64_t hi, uint64_t A, uint64_t groups) {
  if (hi <= lo) return;
  if (lo % SR_HB) throw ApiError{-1, "sr_heads: range start not block aligned"};
  ix.sr_hp[slot].ensure((groups + 1) * 4 + 16);
  TimedLaunch tm(ix.timer, "sa_round_plan", (double)(hi - lo) * 8);
  const unsigned g = (unsigned)std::min<uint64_t>(ceil_div(hi - lo, (uint64_t)SR_HB), 8192);
  k_sr_heads<<<g, 256, 0, ix.stream>>>(G, lo, hi, ix.sr_hp[slot].as<uint32_t>(), ix.sr_win[slot].as<uint32_t>());
  HK_HIP(hipGetLastError());
}

uint64_t sr_plan(Index& ix, int slot, const uint32_t* G, uint64_t A, uint64_t groups, bool heads_ready,
                 uint64_t* big_groups) {
  hipStream_t s = ix.stream;
  const uint64_t nw = ceil_div(A, (uint64_t)SR_W);
  ix.sr_hp[slot].ensure((groups + 1) * 4 + 16);
  ix.sr_items.ensure(nw * sizeof(uint2) + 16);
  ix.sr_cnt.ensure(64);
  ix.grp_big.ensure(groups + 16);
  // the next list's plan buffers (at most A entries, A / 2 groups); k_sr_items resets its windows
  ix.sr_hp[slot ^ 1].ensure((A / 2 + 8) * 4 + 16);
  ix.sr_win[slot ^ 1].ensure(nw * 8 + 16);
  if (!heads_ready) {
    sr_windows_reset(ix, slot, A);
    sr_heads(ix, slot, G, 0, A, A, groups);
  }
  HK_HIP(hipMemsetAsync(ix.grp_big.p, 0, groups, s));
  HK_HIP(hipMemsetAsync(ix.sr_cnt.p, 0, 40, s));   // big counts, the round's counter, linked entries
  {
    TimedLaunch tm(ix.timer, "sa_round_plan", (double)nw * 16);
    const unsigned g2 = (unsigned)std::min<uint64_t>(ceil_div(nw, 256), 4096);
    k_sr_items<<<g2, 256, 0, s>>>(G, ix.sr_hp[slot].as<uint32_t>(), groups, A, ix.sr_win[slot].as<uint32_t>(), nw,
                                  ix.sr_items.as<uint2>(), ix.grp_big.as<uint8_t>(), ix.sr_cnt.as<unsigned long long>(),
                                  ix.sr_win[slot ^ 1].as<uint2>());
    HK_HIP(hipGetLastError());
  }
  uint64_t* const rb = ix.rb();
  HK_HIP(hipMemcpyAsync(&rb[0], ix.sr_cnt.p, 16, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (big_groups) *big_groups = rb[1];
  return rb[0];
}

template <typename V>
std::pair<uint64_t, uint64_t> sr_items_round(Index& ix, int mode, SrRoundArgs<V> args, uint64_t A, uint64_t tied0,
                                             uint64_t groups0, uint64_t* linked) {
  hipStream_t s = ix.stream;
  const uint64_t nw = ceil_div(A, (uint64_t)SR_W);
  unsigned long long* ctr = ix.sr_cnt.as<unsigned long long>() + 2;   // (zeroed by sr_plan)
  uint64_t* const rb = ix.rb();
  rb[4] = 0;
  args.items = ix.sr_items.as<uint2>();
  args.counter = ctr;
  args.base_e = tied0;
  args.base_g = groups0;
  if (args.lnk) {
    args.lcount = ix.sr_cnt.as<unsigned long long>() + 4;   // (zeroed by sr_plan)
    args.gcount = ix.sr_cnt.as<unsigned long long>() + 10;
    args.grec = ix.lk_grec.as<uint4>();
  }
  if (nw) {
    TimedLaunch tm(ix.timer, mode ? "sa_round_dbl" : "sa_round_chunk",
                   (double)A * (8 + 2 * sizeof(V) + 8 + 4 + 4));
    if (mode) k_sr_round<V, 1><<<(unsigned)nw, SR_T, 0, s>>>(args);
    else k_sr_round<V, 0><<<(unsigned)nw, SR_T, 0, s>>>(args);
    HK_HIP(hipGetLastError());
  }
  HK_HIP(hipMemcpyAsync(&rb[3], ctr, 8, hipMemcpyDeviceToHost, s));
  if (args.lnk) {
    HK_HIP(hipMemcpyAsync(&rb[4], args.lcount, 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipMemcpyAsync(&rb[5], args.gcount, 8, hipMemcpyDeviceToHost, s));
  }
  HK_HIP(hipStreamSynchronize(s));
  if (linked) *linked = args.lnk ? rb[4] : 0;
  if (args.lnk) ix.dbl.lround.push_back(rb[5]);   // (the groups linked up to this round)
  return {tied0 + (rb[3] & ((1ull << 33) - 1)), groups0 + (rb[3] >> 33)};
}

// ---- doubling links (host)
void lk_begin(Index& ix) {
  const uint64_t n = ix.n;
  ix.lk_lnk.ensure(n * 4 + 16);
  ix.lk_gsz.ensure(n + 16);
  ix.sr_cnt.ensure(128);   // [4]: linked entries of a round, [9]: jump flags, [10]: linked groups
  ix.lk_grec.ensure((ix.dbl.A / 2 + 16) * sizeof(uint4));   // (a linked group has >= 2 members)
  HK_HIP(hipMemsetAsync(ix.lk_gsz.p, 0, n, ix.stream));
  HK_HIP(hipMemsetAsync(ix.lk_lnk.p, 0, n * 4, ix.stream));
  HK_HIP(hipMemsetAsync(ix.sr_cnt.as<unsigned long long>() + 10, 0, 8, ix.stream));
  ix.dbl.lround.clear();
  ix.dbl.nlinked = 0;
  ix.dbl.ltag = 0;
}

uint64_t lk_max_offset() { return LT_POS; }

void lk_sizes(Index& ix, int slot, uint64_t A, uint64_t groups) {
  if (!groups) return;
  TimedLaunch tm(ix.timer, "sa_link", (double)groups * 12);
  k_lk_sizes<<<(unsigned)std::min<uint64_t>(ceil_div(groups, 256), 16384), 256, 0, ix.stream>>>(
      ix.head_slot.as<uint32_t>(), ix.sr_hp[slot].as<uint32_t>(), groups, A, ix.n, ix.lk_gsz.as<uint8_t>());
  HK_HIP(hipGetLastError());
}

static unsigned int lk_flag_read(Index& ix, unsigned int* d_flag) {
  uint64_t* const rb = ix.rb();
  rb[5] = 0;
  HK_HIP(hipMemcpyAsync(&rb[5], d_flag, 4, hipMemcpyDeviceToHost, ix.stream));
  HK_HIP(hipStreamSynchronize(ix.stream));
  return (unsigned int)rb[5];
}

void lk_after_round(Index& ix, uint64_t linked, uint32_t h) {
  if (!linked) return;
  if (h < 1 || h > LT_POS) throw ApiError{-7, "prefix doubling: link offset beyond the link tiles"};
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  unsigned int* flag = reinterpret_cast<unsigned int*>(ix.sr_cnt.as<unsigned long long>() + 9);
  // this round's chains (all of offset h) inside LDS tiles, then across tiles
  const uint32_t R = LT_POS / h;
  const uint64_t T = (uint64_t)R * h, nt = ceil_div(n, T), m = nt * h;
  ix.lk_tops.ensure(m * 8 * 5 + 64);
  uint64_t* tops = ix.lk_tops.as<uint64_t>();
  uint64_t* acc[2] = {tops + m, tops + 2 * m};
  uint64_t* nxt[2] = {tops + 3 * m, tops + 4 * m};
  {
    TimedLaunch tm(ix.timer, "sa_link", (double)n * 4 + (double)linked * 16);
    k_lk_tile<<<(unsigned)nt, LT_T, 0, s>>>(ix.isa.as<uint32_t>(), ix.lk_lnk.as<uint32_t>(), n, h, R, tops);
    HK_HIP(hipGetLastError());
  }
  const unsigned gm = (unsigned)std::min<uint64_t>(ceil_div(m, 256), 16384);
  {
    TimedLaunch tm(ix.timer, "sa_link", (double)m * 24);
    k_lk_tops_init<<<gm, 256, 0, s>>>(tops, m, h, acc[0], nxt[0]);
    HK_HIP(hipGetLastError());
  }
  int c = 0;
  for (int pass = 0;; ++pass) {
    if (pass > 40) throw ApiError{-7, "prefix doubling: link tiles did not converge"};
    HK_HIP(hipMemsetAsync(flag, 0, 4, s));
    {
      TimedLaunch tm(ix.timer, "sa_link", (double)m * 48);
      k_lk_tops_jump<<<gm, 256, 0, s>>>(acc[c], nxt[c], m, acc[c ^ 1], nxt[c ^ 1], flag);
      HK_HIP(hipGetLastError());
    }
    c ^= 1;
    if (!lk_flag_read(ix, flag)) break;
  }
  {
    TimedLaunch tm(ix.timer, "sa_link", (double)n * 4 + (double)linked * 16);
    k_lk_open_fix<<<(unsigned)std::min<uint64_t>(ceil_div(n, 1024), 16384), 256, 0, s>>>(ix.isa.as<uint32_t>(), ix.lk_lnk.as<uint32_t>(), n, h, R, acc[c], m);
    HK_HIP(hipGetLastError());
  }
  ix.dbl.nlinked += linked;   // (every link names an unlinked position now)
}

void lk_resolve(Index& ix) {
  if (!ix.dbl.nlinked || ix.dbl.lround.empty()) return;
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n, ng = ix.dbl.lround.back();
  unsigned int* flag = reinterpret_cast<unsigned int*>(ix.sr_cnt.as<unsigned long long>() + 9);
  HK_HIP(hipMemsetAsync(flag, 0, 4, s));
  {
    TimedLaunch tm(ix.timer, "sa_link", (double)ng * 24 + (double)ix.dbl.nlinked * 9);
    k_lk_resolve<<<(unsigned)std::min<uint64_t>(ceil_div(ng, 256), 16384), 256, 0, s>>>(
        ix.lk_grec.as<uint4>(), 0, ng, ix.lk_lnk.as<uint32_t>(), ix.isa.as<uint32_t>(), ix.dbl.lk_h,
        ix.text.as<uint8_t>(), n, ix.sa.as<uint32_t>(),
        ix.bwt.as<uint8_t>(), flag);
    HK_HIP(hipGetLastError());
  }
  if (lk_flag_read(ix, flag)) throw ApiError{-7, "prefix doubling: a linked group found no slots"};
}

template std::pair<uint64_t, uint64_t> sr_items_round<uint32_t>(Index&, int, SrRoundArgs<uint32_t>, uint64_t, uint64_t,
                                                                 uint64_t, uint64_t*);
template std::pair<uint64_t, uint64_t> sr_items_round<uint64_t>(Index&, int, SrRoundArgs<uint64_t>, uint64_t, uint64_t,
                                                                 uint64_t, uint64_t*);

}  // namespace hk
