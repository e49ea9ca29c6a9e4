// hk_bsort.hip — the LDS bucket sorts of the single-GPU and sliced bucket builds (split out of hk_bucket.hip).
//
// One workgroup sorts one work item (whole buckets of the cursor partition, <= 9056 / 18432 suffixes)
// and writes SA and BWT in sorted order; suffixes with equal keys go to the tie list for the refinement
// (hk_sa.hip).  Replaces build_suffix_array (csa/suffix_array.py:131-134) + bwt_transform (csa/bwt.py:3-13)
// for the suffixes of one item.  Three kernels:
//   k_bucket_sort_rec   record-plane sort, sigma <= 8 packed records (the 1 GiB headline's items);
//   k_bucket_sort_fast  MSD bins + slot planes, any packed or key/value item with <= 30 varying bits;
//   k_bucket_sort       LSD passes over the varying bits, every item the others decline.

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "hk_bucket.hpp"
#include "hk_index.hpp"

namespace hk {
namespace {

// ------------------------------------------------------------ 4. LDS bucket sort
template <int T>
struct alignas(16) BsSharedT {
  // (+4: the fast path stages its output at final index + the SA pointer's misalignment, section 7)
  uint32_t buf[T * BS_I + 4];    // u32 plane: local key exchange; positions at the end
  uint16_t aux[T * BS_I + 4];    // u16 plane: original-slot exchange (prev codes packed in the key),
                                 // or the prev codes by original slot (when they do not fit the key)
  uint64_t mt[T / 64][256];      // per-wave match masks (lanes holding a digit), zero between items;
                                 // mt[0..1] double as the scan's per-group prefixes
  uint32_t whist[T / 64][256];   // digit counts per wave -> destination base per wave
  uint32_t wloc[256];            // scan: wave-local exclusive digit start
  uint32_t wsum[4];
  uint64_t rv[2][T / 64];
  uint8_t inv[256];
};
using BsShared = BsSharedT<BS_T>;   // the LSD passes (k_bucket_sort) always run 1024-thread items


// One workgroup sorts items[blockIdx.x] = {start, count} of the bucket-grouped (keys, vals): LSD
// radix passes over the key bits that vary inside the range (wave ballot ranking in two
// independent chains per thread, one 1024-thread scan of the 32 x 256 counts, LDS exchange of the
// local key and original-slot planes), then SA[start + r] / BWT[start + r] in sorted order and
// equal keys to the tie list.  The BWT code rides in the key word above the varying bits when it
// fits (one exchange phase per pass), else it waits in LDS by original slot.
// Key layout: [sym, sb bits][prev code, pb bits][position bits 32.., hb bits] (hb > 0 only for
// the 64-bit positions of sharded builds: values hold the low 32 bits, V = uint64_t outputs).
// the keys of work item `it` in slot order (slot s0 + 64 k of thread (wave, lane)); zeros past its end
__device__ __forceinline__ void bs_load_keys(const uint64_t* __restrict__ keys, uint2 it, uint64_t (&key)[BS_I]) {
  const uint64_t* __restrict__ kb = keys + it.x;
  const uint32_t sl = (threadIdx.x >> 6) * BS_WSPAN + (threadIdx.x & 63);
#pragma unroll
  for (int k = 0; k < BS_I; ++k) key[k] = sl + 64u * k < it.y ? kb[sl + 64u * k] : 0;
}

// ---- fast path: one MSD counting pass, then the bins settled in parallel
// The order among equal keys does not matter (they go to the tie list and are refined), so the LDS
// sort need not be stable.  One pass bins the suffixes by the top BF_BITS of their local key with LDS
// atomics (the returned count is a rank inside the bin, in any order) and scatters one u32 record per
// suffix, (remaining key bits << 15 | original slot), to its bin.  The bins hold ~1.1 suffixes for iid
// text: every thread settles 16 bins of one or two records with straight-line code (the record's final
// index, by slot, into the u16 plane) and lists the rarer bins of 3+ records, which one thread each
// then insertion-sorts (the slot breaks ties, so the order is total).  Equal keys are listed by final
// index and written to the tie list from the staged planes.  Replaces three stable LSD passes whose
// match-mask ranking and scatters spent half of their LDS cycles in bank conflicts
// (profiles/r2_sq_counters.json).  Items with a bin over BF_MAXBIN (skewed keys), more than 30 varying
// key bits or overflowing lists take the LSD passes (k_bucket_sort).
// Workgroups of T = 1024 (18 432-suffix items, 14-bit bins, one per CU) or 512 threads (9216-suffix
// items of 2^17 buckets, 13-bit bins, ~80 KiB of LDS: two per CU, so one item's key loads overlap
// the other's LDS phases).  Bins hold ~1.1 suffixes either way.
constexpr uint32_t BF_MAXBIN = 32;

// LDS of the fast path: T threads, I suffixes per thread (capacity T * I)
template <int T, int I>
struct alignas(16) BfShared {
  static constexpr int CAP = T * I;
  static constexpr int BITS = CAP <= 9216 ? 13 : 14;   // ~1.1 suffixes per bin
  static constexpr int BINS = 1 << BITS;
  uint32_t buf[CAP + 4];       // positions by slot, records by bin, positions by final index (+4: section 7)
  uint16_t aux[CAP + 4];       // final index by slot, then prev codes by final index
  uint32_t H2[BINS / 2 + 1];   // u16 bin counters / starts, two per word, zero on entry (+1: the
                               // reads of a next bin's start past the last bin stay in bounds)
  uint16_t lists[BINS / 2];    // listed bins (first half), tied records (second half)
  uint32_t wloc[2 * (T / 64)];
  uint32_t wsum[4];
  uint64_t red[4 * (T / 64)];
  uint8_t inv[256];
};

// PK: xs holds the packed records (sym = record >> xsh, position = the low pbits bits) and the
// positions come from them instead of a value plane.
template <typename V, bool TRACE, int T, int I, bool PK = false, bool X32 = false>
__device__ __forceinline__ bool bucket_sort_fast(BfShared<T, I>& sh, uint2 it, const uint64_t (&xs)[I],
                                                 const uint32_t (&pvr)[(I + 1) / 2], uint32_t vmask, uint32_t s0,
                                                 uint64_t xmin, int lo, int width, int pb, int xsh, int pbits,
                                                 int term, const uint32_t* __restrict__ vb,
                                                 V* __restrict__ sab, uint8_t* __restrict__ bwb,
                                                 uint64_t* __restrict__ tie_k, V* __restrict__ tie_v,
                                                 unsigned long long* __restrict__ tie_n, uint64_t (&ts)[8]) {
  using SH = BfShared<T, I>;
  constexpr int BF_BITS = SH::BITS, BF_BINS = SH::BINS;   // u16 counters, two per u32
  constexpr uint32_t BF_BIGCAP = BF_BINS / 4;   // bins of 3+ records (u16 bin ids, first half of lists)
  constexpr uint32_t BF_TIECAP = BF_BINS / 4;   // tied records (u16 final index | head << 15, second half)
  constexpr int NP = BF_BINS / 2 / T;           // counter words (bin pairs) per thread
  constexpr int IH = (I + 1) / 2;
  static_assert(NP == 4 || NP == 8, "8 or 16 bin counters per thread");
  const uint32_t start = it.x, cnt = it.y;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fb = width < BF_BITS ? width : BF_BITS;
  const int kb = width - fb;                              // key bits below the bin (<= 16)
  const uint32_t wmask = width >= 32 ? ~0u : ((1u << width) - 1);
  const uint32_t lowmask = (1u << kb) - 1;
  const uint32_t pmask = (1u << pb) - 1;
  uint32_t* const H2 = sh.H2;
  const uint16_t* const H = reinterpret_cast<const uint16_t*>(H2);
  uint16_t* const blist = sh.lists;
  uint16_t* const tlist = blist + BF_BIGCAP;
  uint32_t* const nctr = sh.wsum;   // [0] listed three-record bins, [1] tied records, [2] larger listed bins
  uint32_t lk[I], r0[IH], vv[I];
  // ---- 1. bin histogram; the atomic's return value is the suffix's rank inside its bin
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const bool valid = (vmask >> k) & 1u;
    if (X32)
      lk[k] = (((uint32_t)(xs[k] >> 32) >> (xsh - 32)) - (uint32_t)xmin) >> lo & wmask;
    else
      lk[k] = (uint32_t)(((PK ? xs[k] >> xsh : xs[k]) - xmin) >> lo) & wmask;
    // packed: the position waits in the u32 plane by slot (free until the records' scatter), so no
    // register holds it across the histogram and the scan
    if (PK) sh.buf[s0 + 64u * k] = (uint32_t)xs[k] & (uint32_t)((1ull << pbits) - 1);
    uint32_t r = 0;
    if (valid) {
      const uint32_t bin = lk[k] >> kb, sh16 = 16u * (bin & 1u);
      r = (atomicAdd(&H2[bin >> 1], 1u << sh16) >> sh16) & 0xFFFFu;   // counts <= 18432: no carry
    }
    if (k < IH) r0[k] = r; else r0[k - IH] |= r << 16;
  }
  __syncthreads();
  if (TRACE) ts[2] = stamp();
  // ---- 2. exclusive scan of the 16384 counters (16 per thread) and the largest bin
  uint32_t w8[NP], tsum = 0, tmax = 0;
  {
#pragma unroll
    for (int q = 0; q < NP / 4; ++q) {
      const uint4 a = reinterpret_cast<const uint4*>(H2)[(NP / 4) * tid + q];
      w8[4 * q] = a.x; w8[4 * q + 1] = a.y; w8[4 * q + 2] = a.z; w8[4 * q + 3] = a.w;
    }
#pragma unroll
    for (int i = 0; i < NP; ++i) {
      const uint32_t c0 = w8[i] & 0xFFFFu, c1 = w8[i] >> 16;
      tmax = c0 > tmax ? c0 : tmax;
      tmax = c1 > tmax ? c1 : tmax;
      w8[i] = tsum | ((tsum + c0) << 16);   // exclusive starts of the pair, relative to the thread
      tsum += c0 + c1;
    }
  }
  const uint32_t inc = dpp_incl_sum(tsum);
  tmax = dpp_reduce_u32(tmax, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
  uint32_t* const wtot = sh.wloc;    // per-wave totals / maxima
  if (lane == 63) wtot[wv] = inc;
  if (lane == 0) wtot[(T / 64) + wv] = tmax;
  __syncthreads();
  uint32_t carry = 0, bmax = 0;
#pragma unroll
  for (int w = 0; w < (T / 64); ++w) {
    carry += (uint32_t)w < wv ? wtot[w] : 0u;
    bmax = wtot[(T / 64) + w] > bmax ? wtot[(T / 64) + w] : bmax;
  }
  if (bmax > BF_MAXBIN) return false;   // skewed keys: the LSD passes
  {
    const uint32_t b0 = carry + inc - tsum;
    const uint32_t b2 = b0 | (b0 << 16);   // starts <= 18432: no carry between the halves
#pragma unroll
    for (int q = 0; q < NP / 4; ++q)
      reinterpret_cast<uint4*>(H2)[(NP / 4) * tid + q] =
          make_uint4(b2 + w8[4 * q], b2 + w8[4 * q + 1], b2 + w8[4 * q + 2], b2 + w8[4 * q + 3]);
  }
  if (tid == 0) { nctr[0] = 0; nctr[1] = 0; nctr[2] = 0; }
  __syncthreads();
  if (TRACE) ts[3] = stamp();
  // ---- 3. positions (coalesced; in flight during the bin work) and records to their bins
  if (PK) {   // packed: from the u32 plane (phase 1), before the records overwrite it
#pragma unroll
    for (int k = 0; k < I; ++k) vv[k] = sh.buf[s0 + 64u * k];
    __syncthreads();
  } else {
#pragma unroll
    for (int k = 0; k < I; ++k) vv[k] = ((vmask >> k) & 1u) ? vb[s0 + 64u * k] : 0u;
  }
#pragma unroll
  for (int k = 0; k < I; ++k) {
    if ((vmask >> k) & 1u) {
      const uint32_t r = k < IH ? (r0[k] & 0xFFFFu) : (r0[k - IH] >> 16);
      sh.buf[H[lk[k] >> kb] + r] = ((lk[k] & lowmask) << 15) | (s0 + 64u * k);
    }
  }
  __syncthreads();
  if (TRACE) ts[4] = stamp();
  // ---- 4. bins of one or two records settle in place: final index by slot into aux; 3+ are listed
  uint32_t bigm = 0, big4 = 0;
  {
    uint32_t pr[BF_BINS / 2 / T], nx[BF_BINS / 2 / T];
#pragma unroll
    for (int j = 0; j < BF_BINS / 2 / T; ++j) {
      const uint32_t m = tid + T * j;   // bins 2m, 2m + 1
      pr[j] = H2[m];
      const uint32_t nw = H2[m + 1];   // (unconditional; the last bin's end is the item's count)
      nx[j] = m + 1 < (uint32_t)BF_BINS / 2 ? (nw & 0xFFFFu) : cnt;
    }
#pragma unroll
    for (int j = 0; j < BF_BINS / 2 / T; ++j) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {   // branch-free: the loads of all 16 bins issue together
        const uint32_t s = h ? pr[j] >> 16 : pr[j] & 0xFFFFu;
        const uint32_t c = (h ? nx[j] : pr[j] >> 16) - s;
        const bool some = c - 1u < 2u, two = c == 2;
        // unconditional reads (s + 1 <= cnt + 1 stays inside the plane): the loads of all 16 bins issue
        // back to back instead of one exec-masked branch each
        const uint32_t x0 = sh.buf[s], y0 = sh.buf[s + 1];
        const uint32_t x = some ? x0 : 0u;
        const uint32_t y = two ? y0 : x;
        const uint32_t a = x < y ? x : y, b = x < y ? y : x;
        if (some) sh.aux[a & 0x7FFFu] = (uint16_t)s;
        if (two) sh.aux[b & 0x7FFFu] = (uint16_t)(s + 1);
        if (two && (x >> 15) == (y >> 15)) {   // equal keys (rare)
          const uint32_t t = atomicAdd(&nctr[1], 2u);
          if (t + 2 <= BF_TIECAP) {
            tlist[t] = (uint16_t)(s | 0x8000u);
            tlist[t + 1] = (uint16_t)(s + 1);
          }
        }
        bigm |= (c == 3 ? 1u : 0u) << (2 * j + h);
        big4 |= (c >= 4 ? 1u : 0u) << (2 * j + h);
      }
    }
  }
  {   // wave-aggregated appends of the listed bins: three-record bins from the front of the list,
      // larger ones from its back (so that each loop of section 5 runs one code path per wave)
    const uint32_t nb = __popc(bigm), nb4 = __popc(big4);
    const uint32_t binc = dpp_incl_sum(nb | (nb4 << 16));   // both counts <= 64 * 16
    uint32_t bbase = 0;
    if (lane == 63 && (binc & 0xFFFFu)) bbase = atomicAdd(&nctr[0], binc & 0xFFFFu);
    if (lane == 63 && (binc >> 16)) bbase |= atomicAdd(&nctr[2], binc >> 16) << 16;
    bbase = __shfl(bbase, 63, 64);
    uint32_t b3 = (bbase & 0xFFFFu) + (binc & 0xFFFFu) - nb, b4 = (bbase >> 16) + (binc >> 16) - nb4;
    while (bigm) {
      const int q = __builtin_ctz(bigm);
      bigm &= bigm - 1;
      if (b3 < BF_BIGCAP) blist[b3] = (uint16_t)(2u * (tid + T * (q >> 1)) + (q & 1));
      ++b3;
    }
    while (big4) {
      const int q = __builtin_ctz(big4);
      big4 &= big4 - 1;
      if (b4 < BF_BIGCAP) blist[BF_BIGCAP - 1 - b4] = (uint16_t)(2u * (tid + T * (q >> 1)) + (q & 1));
      ++b4;
    }
  }
  __syncthreads();
  if (TRACE) ts[5] = stamp();
  const uint32_t nbig3 = nctr[0], nbig4 = nctr[2];
  if (nbig3 + nbig4 > BF_BIGCAP) return false;
  // ---- 5. listed bins, one thread each.  Three records (3/4 of the listed bins for iid text): three
  // compares rank them.  Then up to 8 records ranked in registers (all loads in flight together),
  // larger bins insertion-sorted in place; final indices by slot, equal keys listed
  for (uint32_t i = tid; i < nbig3; i += T) {
    const uint32_t s = H[blist[i]];
    const uint32_t x = sh.buf[s], y = sh.buf[s + 1], z = sh.buf[s + 2];   // distinct (the slots differ)
    const uint32_t xy = x < y, xz = x < z, yz = y < z;
    sh.aux[x & 0x7FFFu] = (uint16_t)(s + (xy ^ 1u) + (xz ^ 1u));
    sh.aux[y & 0x7FFFu] = (uint16_t)(s + xy + (yz ^ 1u));
    sh.aux[z & 0x7FFFu] = (uint16_t)(s + xz + yz);
    const uint32_t kx = x >> 15, ky = y >> 15, kz = z >> 15;
    if (kx == ky || kx == kz || ky == kz) {   // equal keys (rare): every record of a group, the smallest heads it
      const uint32_t r[3] = {x, y, z};
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        uint32_t below = 0, eq = 0, eqb = 0;
#pragma unroll
        for (int o = 0; o < 3; ++o) {
          if (o == q) continue;
          const bool e15 = (r[o] >> 15) == (r[q] >> 15);
          below += r[o] < r[q] ? 1u : 0u;
          eq |= e15 ? 1u : 0u;
          eqb |= (e15 && r[o] < r[q]) ? 1u : 0u;
        }
        if (eq) {
          const uint32_t t = atomicAdd(&nctr[1], 1u);
          if (t < BF_TIECAP) tlist[t] = (uint16_t)((s + below) | (eqb ? 0u : 0x8000u));
        }
      }
    }
  }
  for (uint32_t i = tid; i < nbig4; i += T) {
    const uint32_t bn = blist[BF_BIGCAP - 1 - i];
    const uint32_t hn = H[bn + 1];   // (unconditional read, in bounds by the spare word)
    const uint32_t s = H[bn], e = bn + 1 < (uint32_t)BF_BINS ? hn : cnt;
    const uint32_t c = e - s;
    if (c <= 8) {
      uint32_t r[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // unconditional reads (s + 7 <= cnt + 3 for c >= 4); pads rank last
        const uint32_t v = sh.buf[s + q];
        r[q] = (uint32_t)q < c ? v : ~0u;
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t below = 0, eq = 0, eqb = 0;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          if (o == q) continue;
          const bool e15 = (r[o] >> 15) == (r[q] >> 15);
          below += r[o] < r[q] ? 1u : 0u;
          eq |= e15 ? 1u : 0u;
          eqb |= (e15 && r[o] < r[q]) ? 1u : 0u;
        }
        if ((uint32_t)q < c) {
          sh.aux[r[q] & 0x7FFFu] = (uint16_t)(s + below);
          if (eq) {   // equal keys (rare); the smallest slot heads the group
            const uint32_t t = atomicAdd(&nctr[1], 1u);
            if (t < BF_TIECAP) tlist[t] = (uint16_t)((s + below) | (eqb ? 0u : 0x8000u));
          }
        }
      }
      continue;
    }
    for (uint32_t p = s + 1; p < e; ++p) {
      const uint32_t x = sh.buf[p];
      uint32_t q = p;
      while (q > s) {
        const uint32_t y = sh.buf[q - 1];
        if (y < x) break;
        sh.buf[q] = y;
        --q;
      }
      sh.buf[q] = x;
    }
    uint32_t x = sh.buf[s], rs = s;
    sh.aux[x & 0x7FFFu] = (uint16_t)s;
    for (uint32_t p = s + 1; p <= e; ++p) {
      const uint32_t y = p < e ? sh.buf[p] : ~0u;
      if (p < e) sh.aux[y & 0x7FFFu] = (uint16_t)p;
      if ((y >> 15) != (x >> 15)) {   // a run of equal keys ends at p (key bits < 2^16, so ~0u differs)
        if (p - rs >= 2) {
          const uint32_t t = atomicAdd(&nctr[1], p - rs);
          for (uint32_t q = rs; q < p; ++q)
            if (t + (q - rs) < BF_TIECAP) tlist[t + (q - rs)] = (uint16_t)(q | (q == rs ? 0x8000u : 0u));
        }
        rs = p;
      }
      x = y;
    }
  }
  __syncthreads();
  if (TRACE) ts[6] = stamp();
  const uint32_t ntie = nctr[1];
  if (ntie > BF_TIECAP) return false;
  // tie-list space: one global atomic per workgroup, by thread 0; only wave 0 waits for it (it writes
  // the tied records after its share of the SA and BWT)
  unsigned long long tbase = 0;
  if (tid == 0 && ntie) tbase = atomicAdd(tie_n, (unsigned long long)ntie);
  // ---- 6. stage (position, prev code) by final index f, at f + al: al = the SA pointer's position
  // inside its 4-entry group, so that every 4 staged entries are one aligned 16-B SA store (two for u64
  // positions) and one aligned 4-B BWT store (both outputs start at the same index, so the BWT pointer
  // shares the misalignment whenever both arrays are 16-B aligned; else the per-entry stores)
  const uint32_t al = (uint32_t)(((uintptr_t)sab / sizeof(V)) & 3u);
  const bool vec = al == (uint32_t)((uintptr_t)bwb & 3u);
  const uint32_t sto = vec ? al : 0u;
  uint32_t fin[IH];
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const uint32_t fa = sh.aux[s0 + 64u * k];   // (unconditional: the slot is inside the plane)
    const uint32_t f = ((vmask >> k) & 1u) ? fa : 0u;
    if (k < IH) fin[k] = f; else fin[k - IH] |= f << 16;
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < I; ++k) {
    if ((vmask >> k) & 1u) {
      const uint32_t f = (k < IH ? (fin[k] & 0xFFFFu) : (fin[k - IH] >> 16)) + sto;
      sh.buf[f] = vv[k];
      sh.aux[f] = (uint16_t)(k < IH ? (pvr[k] & 0xFFFFu) : (pvr[k - IH] >> 16));
    }
  }
  __syncthreads();
  // ---- 7. SA / BWT in sorted order, then the tied records
  auto bwt_byte = [&](uint32_t pos, uint32_t pv) -> uint32_t {
    return PK && pos == 0 && (pv >> pb) == 0 && term >= 0 ? (uint32_t)term : (uint32_t)sh.inv[pv & pmask];
  };
  if (vec) {
    // groups of 4 staged entries; the BWT bytes of <= 8 codes by one v_perm_b32 from the 8-byte table
    const uint32_t ng = (cnt + al + 3) >> 2;
    const uint32_t tlo = reinterpret_cast<const uint32_t*>(sh.inv)[0];
    const uint32_t thi = reinterpret_cast<const uint32_t*>(sh.inv)[1];
    for (uint32_t q = tid; q < ng; q += T) {
      const uint4 p4 = reinterpret_cast<const uint4*>(sh.buf)[q];
      const uint2 a2 = reinterpret_cast<const uint2*>(sh.aux)[q];
      const uint32_t pos[4] = {p4.x, p4.y, p4.z, p4.w};
      const uint32_t pv[4] = {a2.x & 0xFFFFu, a2.x >> 16, a2.y & 0xFFFFu, a2.y >> 16};
      uint32_t bw;
      if (pb <= 3) {
        const uint32_t sel = (pv[0] & pmask) | (pv[1] & pmask) << 8 | (pv[2] & pmask) << 16 | (pv[3] & pmask) << 24;
        bw = __builtin_amdgcn_perm(thi, tlo, sel);
        if (PK && term >= 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (pos[j] == 0 && (pv[j] >> pb) == 0) bw = (bw & ~(0xFFu << (8 * j))) | ((uint32_t)term << (8 * j));
        }
      } else {
        bw = 0;
#pragma unroll
        for (int j = 0; j < 4; ++j) bw |= bwt_byte(pos[j], pv[j]) << (8 * j);
      }
      const uint32_t g = 4u * q;
      if (g >= al && g + 4 <= cnt + al) {   // a whole group: aligned vector stores
        V* const dst = sab + (g - al);
        if (sizeof(V) == 4) {
          *reinterpret_cast<uint4*>(dst) = p4;
        } else {
          uint4* const d4 = reinterpret_cast<uint4*>(dst);
          d4[0] = make_uint4(pos[0], pv[0] >> pb, pos[1], pv[1] >> pb);
          d4[1] = make_uint4(pos[2], pv[2] >> pb, pos[3], pv[3] >> pb);
        }
        *reinterpret_cast<uint32_t*>(bwb + (g - al)) = bw;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t r = g + j;
          if (r >= al && r < cnt + al) {
            sab[r - al] = (V)(((uint64_t)(pv[j] >> pb) << 32) | pos[j]);
            bwb[r - al] = (uint8_t)(bw >> (8 * j));
          }
        }
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const uint32_t r = s0 + 64u * k;
      if (r < cnt) {
        const uint32_t pv = sh.aux[r], pos = sh.buf[r];
        sab[r] = (V)(((uint64_t)(pv >> pb) << 32) | pos);
        bwb[r] = (uint8_t)bwt_byte(pos, pv);
      }
    }
  }
  if (wv == 0 && ntie) {
    const uint64_t tb = __shfl(tbase, 0, 64);
    // the tied records in slot order (the refinement takes the tie list as runs of whole groups, each
    // group's records consecutive and its head first): wave 0 alone sets bit masks of the tied and the
    // head final indices over the bin lists (free after section 5) and walks them in order
    if (ntie <= 64) {   // (most items) a record per lane, ranked by its final index against the others
      const uint32_t e = lane < ntie ? tlist[lane] : 0xFFFFu, q = e & 0x7FFFu;
      uint32_t r = 0;
      for (uint32_t i = 0; i < ntie; ++i) r += (tlist[i] & 0x7FFFu) < q ? 1u : 0u;
      if (lane < ntie) {
        const uint32_t f = q + sto;
        const uint32_t pv = sh.aux[f];
        tie_k[tb + r] = (((uint64_t)start + q) << 1) | (e >> 15);
        tie_v[tb + r] = (V)(((uint64_t)(pv >> pb) << 32) | sh.buf[f]);
      }
      return true;
    }
    uint32_t* const tbits = reinterpret_cast<uint32_t*>(blist);
    const uint32_t nwd = (cnt + 31) / 32;
    static_assert(2 * ((SH::CAP + 31) / 32) * 4 <= BF_BIGCAP * 2, "tie bit masks fit the bin lists");
    for (uint32_t i = lane; i < 2 * nwd; i += 64) tbits[i] = 0;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    for (uint32_t i = lane; i < ntie; i += 64) {
      const uint32_t e = tlist[i], q = e & 0x7FFFu;
      atomicOr(&tbits[q >> 5], 1u << (q & 31));
      if (e >> 15) atomicOr(&tbits[nwd + (q >> 5)], 1u << (q & 31));
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
    uint32_t run = 0;
    for (uint32_t w0 = 0; w0 < nwd; w0 += 64) {   // 64 mask words per step, ranked by a wave scan
      const uint32_t w = w0 + lane;
      uint32_t bits = w < nwd ? tbits[w] : 0u;
      const uint32_t hw = w < nwd ? tbits[nwd + w] : 0u;
      const uint32_t c = __popc(bits);
      const uint32_t inc = wave_incl_sum<uint32_t>(c);
      uint32_t r = run + inc - c;
      while (bits) {
        const uint32_t b = __builtin_ctz(bits);
        bits &= bits - 1;
        const uint32_t q = 32 * w + b, f = q + sto;
        const uint32_t pv = sh.aux[f];
        tie_k[tb + r] = (((uint64_t)start + q) << 1) | ((hw >> b) & 1u);
        tie_v[tb + r] = (V)(((uint64_t)(pv >> pb) << 32) | sh.buf[f]);
        ++r;
      }
      run += __shfl(inc, 63, 64);
    }
  }
  return true;
}

// One work item of the LDS bucket sort, its keys in `key` (slot order).
template <bool WIDE, bool TRACE, typename V>
__device__ __forceinline__ void bucket_sort_item(BsShared& sh, uint2 it, const uint64_t (&key)[BS_I],
                                                 uint32_t item, const uint64_t* __restrict__ keys,
                                                 const uint32_t* __restrict__ vals, int pb, int sb, int hb,
                                                 uint64_t symbias, V* __restrict__ sa, uint8_t* __restrict__ bwt,
                                                 uint64_t* __restrict__ tie_k, V* __restrict__ tie_v,
                                                 unsigned long long* __restrict__ tie_n,
                                                 uint64_t* __restrict__ trace) {
  uint64_t ts[8] = {0};
  if (TRACE) ts[0] = stamp();
  const uint32_t start = it.x, cnt = it.y;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  // workgroup-uniform bases: every per-item index below is a 32-bit offset from them
  const uint32_t* __restrict__ vb = vals + start;
  V* __restrict__ sab = sa + start;
  uint8_t* __restrict__ bwb = bwt + start;
  // slot of item k is s0 + 64 k (immediate LDS offsets); bit k of vmask = slot k holds a suffix
  uint32_t s0 = wv * BS_WSPAN + lane;
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < BS_I; ++k) vmask |= (s0 + 64u * k < cnt ? 1u : 0u) << k;
  const uint64_t symmask = sb >= 64 ? ~0ull : ((1ull << sb) - 1);
  const uint32_t pmask = (1u << pb) - 1;
  const int pbe = pb + hb;                       // sym field starts here
  const uint32_t himask = (1u << hb) - 1;
  for (uint32_t i = tid; i < BS_V * 256; i += BS_T) (&sh.whist[0][0])[i] = 0;
  for (uint32_t i = tid; i < BS_W * 256; i += BS_T) (&sh.mt[0][0])[i] = 0;

  // ---- the item's smallest sym field, and the varying-bit range of the sym fields above it
  // (local keys are sym - min: a bin that straddles a power of two stays narrow)
  uint64_t xmin = ~0ull;
#pragma unroll
  for (int k = 0; k < BS_I; ++k)
    if ((vmask >> k) & 1u) {
      const uint64_t x = ((key[k] >> pbe) & symmask) - symbias;
      xmin = x < xmin ? x : xmin;
    }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t t = __shfl_xor(xmin, o, 64);
    xmin = t < xmin ? t : xmin;
  }
  if (lane == 0) sh.rv[0][wv] = xmin;
  __syncthreads();
#pragma unroll
  for (int w = 0; w < BS_W; ++w) xmin = sh.rv[0][w] < xmin ? sh.rv[0][w] : xmin;
  const uint64_t base = symbias + xmin;
  uint64_t vor = 0, vand = ~0ull;
#pragma unroll
  for (int k = 0; k < BS_I; ++k) {
    if ((vmask >> k) & 1u) {
      const uint64_t sym = ((key[k] >> pbe) & symmask) - base;
      vor |= sym;
      vand &= sym;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    vor |= __shfl_xor(vor, o, 64);
    vand &= __shfl_xor(vand, o, 64);
  }
  __syncthreads();   // every wave has read rv[0]
  if (lane == 0) {
    sh.rv[0][wv] = vor;
    sh.rv[1][wv] = vand;
  }
  __syncthreads();
  vor = 0;
  vand = ~0ull;
#pragma unroll
  for (int w = 0; w < BS_W; ++w) {
    vor |= sh.rv[0][w];
    vand &= sh.rv[1][w];
  }
  const uint64_t var = vor ^ vand;
  const int lo = var ? __builtin_ctzll(var) : 0;
  const int width = var ? 64 - __builtin_clzll(var) - lo : 0;
  const bool packprev = !WIDE && width + pb + hb <= 32;
  const uint32_t kmask = width >= 32 ? ~0u : ((1u << width) - 1);

  // live through the passes: the local key plane(s) and the original slot, 16 bits per item
  // packed two to a register (as are the per-pass ranks)
  uint32_t klo[BS_I], khi[BS_I], ix2[BS_H];
#pragma unroll
  for (int k = 0; k < BS_I; ++k) {
    // varying bits only (the constant bits above them would collide with the packed prev code)
    const uint64_t lk = ((((key[k] >> pbe) & symmask) - base) >> lo) & (width >= 64 ? ~0ull : ((1ull << width) - 1));
    // prev code and position high bits ride together: in the key word above the varying bits, or
    // in the u16 plane by original slot
    const uint32_t pv = ((uint32_t)(key[k] >> hb) & pmask) | (((uint32_t)key[k] & himask) << pb);
    klo[k] = (uint32_t)lk | (packprev ? pv << width : 0u);
    khi[k] = WIDE ? (uint32_t)(lk >> 32) : 0u;
    if (!packprev && ((vmask >> k) & 1u)) sh.aux[s0 + 64u * k] = (uint16_t)pv;
  }
  // ix2[j] = original slots of items j (low half) and j + BS_H (high half)
#pragma unroll
  for (int j = 0; j < BS_H; ++j) ix2[j] = (s0 + 64u * j) | ((s0 + 64u * (j + BS_H)) << 16);
  uint16_t* buf16 = reinterpret_cast<uint16_t*>(sh.buf);
  __syncthreads();
  if (TRACE) ts[1] = stamp();

  auto half = [](const uint32_t* a2, int k) -> uint32_t {
    return k < BS_H ? (a2[k] & 0xFFFFu) : (a2[k - BS_H] >> 16);
  };
  // ---- radix passes over the varying bits (uniform digits skipped)
  for (int d0 = 0; d0 < width; d0 += 8) {
    const uint32_t dmask = (uint32_t)((var >> lo) >> d0) & 255u;
    if (!dmask) continue;
    const int nb = 32 - __clz(dmask);   // highest varying bit of the digit + 1
    const uint32_t dm = (1u << nb) - 1;
    auto digit_of = [&](int k) -> uint32_t {
      if (!WIDE) return (klo[k] >> d0) & dm;
      return (uint32_t)((((uint64_t)khi[k] << 32) | klo[k]) >> d0) & dm;
    };
    asm volatile("" : "+v"(s0));   // slot addresses are cheap: recompute them per pass
    // ranking (stable: item-major, then lane): each lane ORs its bit into the wave's mask of its
    // digit and reads the mask back — the lanes sharing the digit — instead of 8 ballots; the
    // group's lowest lane advances the wave's digit count and clears the mask
    uint32_t rk2[BS_H];
#pragma unroll
    for (int k = 0; k < BS_I; ++k) {
      const bool valid = (vmask >> k) & 1u;
      const uint32_t dg = digit_of(k);
      uint64_t* ms = &sh.mt[wv][dg];
      if (valid) __hip_atomic_fetch_or(ms, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint64_t m = __hip_atomic_load(ms, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      const uint32_t below = mbcnt(m);
      const uint32_t prior = sh.whist[wv][dg];
      if (valid && below == 0) {
        __hip_atomic_store(ms, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        sh.whist[wv][dg] = prior + (uint32_t)__popcll(m);
      }
      const uint32_t wr = (prior + below) & 0xFFFFu;
      if (k < BS_H) rk2[k] = wr; else rk2[k - BS_H] |= wr << 16;
    }
    __syncthreads();
    if (TRACE && d0 == 0) ts[6] = stamp();
    // scan of the 16 x 256 counts by all 1024 threads: group g = tid >> 8 owns waves 4g .. 4g+3
    // of digit d = tid & 255
    {
      uint32_t(*gpre)[256] = reinterpret_cast<uint32_t(*)[256]>(&sh.mt[0][0]);
      const uint32_t d = tid & 255u, g = tid >> 8;
      uint32_t c4[4], run = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) c4[i] = sh.whist[4 * g + i][d];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        sh.whist[4 * g + i][d] = run;
        run += c4[i];
      }
      gpre[g][d] = run;
      __syncthreads();
      if (tid < 256) {
        uint32_t gp = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const uint32_t v = gpre[q][d];
          gpre[q][d] = gp;
          gp += v;
        }
        const uint32_t inc = wave_incl_sum<uint32_t>(gp);
        if (lane == 63) sh.wsum[wv] = inc;
        sh.wloc[d] = inc - gp;
      }
      __syncthreads();
      uint32_t carry = 0;
      for (uint32_t w = 0; w < (d >> 6); ++w) carry += sh.wsum[w];
      const uint32_t base = sh.wloc[d] + carry + gpre[g][d];
#pragma unroll
      for (int i = 0; i < 4; ++i) sh.whist[4 * g + i][d] += base;
      __syncthreads();
      reinterpret_cast<uint32_t*>(&sh.mt[0][0])[tid] = 0;   // gpre back to clean match masks
    }
    if (TRACE && d0 == 0) ts[7] = stamp();
    // destinations of all items first (the base reads issue back to back, one wait), in place of
    // the ranks; empty slots (only when cnt < BS_CAP) all write to the free slot cnt, so the
    // exchange stores need no per-item branch
#pragma unroll
    for (int j = 0; j < BS_H; ++j) {
      const uint32_t a = sh.whist[wv][digit_of(j)] + (rk2[j] & 0xFFFFu);
      const uint32_t b = sh.whist[wv][digit_of(j + BS_H)] + (rk2[j] >> 16);
      rk2[j] = (((vmask >> j) & 1u) ? a : cnt) | ((((vmask >> (j + BS_H)) & 1u) ? b : cnt) << 16);
    }
    auto dst = [&](int k) -> uint32_t { return half(rk2, k); };
    if (packprev) {
      // one exchange phase: key word (with the prev code) and original slot together
#pragma unroll
      for (int k = 0; k < BS_I; ++k) {
        const uint32_t D = dst(k);
        sh.buf[D] = klo[k];
        sh.aux[D] = (uint16_t)half(ix2, k);
      }
      __syncthreads();
      for (uint32_t i = tid; i < BS_V * 256; i += BS_T) (&sh.whist[0][0])[i] = 0;
#pragma unroll
      for (int k = 0; k < BS_I; ++k) klo[k] = sh.buf[s0 + 64u * k];
#pragma unroll
      for (int j = 0; j < BS_H; ++j) ix2[j] = (uint32_t)sh.aux[s0 + 64u * j] | ((uint32_t)sh.aux[s0 + 64u * (j + BS_H)] << 16);
      __syncthreads();
    } else {
#pragma unroll
      for (int k = 0; k < BS_I; ++k)
        buf16[dst(k)] = (uint16_t)half(ix2, k);
      __syncthreads();
#pragma unroll
      for (int j = 0; j < BS_H; ++j) ix2[j] = (uint32_t)buf16[s0 + 64u * j] | ((uint32_t)buf16[s0 + 64u * (j + BS_H)] << 16);
      __syncthreads();
      if (WIDE) {
#pragma unroll
        for (int k = 0; k < BS_I; ++k)
          sh.buf[dst(k)] = khi[k];
        __syncthreads();
        uint32_t nh[BS_I];
#pragma unroll
        for (int k = 0; k < BS_I; ++k) nh[k] = sh.buf[s0 + 64u * k];
        __syncthreads();
#pragma unroll
        for (int k = 0; k < BS_I; ++k)
          sh.buf[dst(k)] = klo[k];
        __syncthreads();
        for (uint32_t i = tid; i < BS_V * 256; i += BS_T) (&sh.whist[0][0])[i] = 0;
#pragma unroll
        for (int k = 0; k < BS_I; ++k) {
          khi[k] = nh[k];
          klo[k] = sh.buf[s0 + 64u * k];
        }
        __syncthreads();
      } else {
#pragma unroll
        for (int k = 0; k < BS_I; ++k)
          sh.buf[dst(k)] = klo[k];
        __syncthreads();
        for (uint32_t i = tid; i < BS_V * 256; i += BS_T) (&sh.whist[0][0])[i] = 0;
#pragma unroll
        for (int k = 0; k < BS_I; ++k) klo[k] = sh.buf[s0 + 64u * k];
        __syncthreads();
      }
    }
  }

  // ---- this item's positions, in flight across the tie phase (measured faster than loading them
  // after it; touching the next item's lines ahead of time was slower).  The memory clobber keeps
  // the compiler from hoisting the loads into the passes, where registers are full.
  asm volatile("" ::: "memory");
  uint32_t vv[BS_I];
#pragma unroll
  for (int k = 0; k < BS_I; ++k) vv[k] = ((vmask >> k) & 1u) ? vb[s0 + 64u * k] : 0u;

  // ---- ties: equal local keys next to each other in sorted order
  if (TRACE) ts[2] = stamp();
  asm volatile("" : "+v"(s0));
#pragma unroll
  for (int k = 0; k < BS_I; ++k) sh.buf[s0 + 64u * k] = klo[k] & kmask;
  __syncthreads();
  uint32_t eqp = 0, eqn = 0;
#pragma unroll
  for (int k = 0; k < BS_I; ++k) {
    const uint32_t r = s0 + 64u * k;
    const uint32_t v = klo[k] & kmask;
    if ((vmask >> k) & 1u) {
      if (r > 0 && sh.buf[r - 1] == v) eqp |= 1u << k;
      if (r + 1 < cnt && sh.buf[r + 1] == v) eqn |= 1u << k;
    }
  }
  if (WIDE) {
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BS_I; ++k) sh.buf[s0 + 64u * k] = khi[k];
    __syncthreads();
#pragma unroll
    for (int k = 0; k < BS_I; ++k) {
      const uint32_t r = s0 + 64u * k;
      if ((vmask >> k) & 1u) {
        if (r > 0 && sh.buf[r - 1] != khi[k]) eqp &= ~(1u << k);
        if (r + 1 < cnt && sh.buf[r + 1] != khi[k]) eqn &= ~(1u << k);
      }
    }
  }
  const uint32_t tmask = eqp | eqn;
  const uint32_t hmask = tmask & ~eqp;
  // tie-list space: one global atomic per workgroup (a per-wave atomic on the single counter
  // serialises in L2 when ties are frequent), each thread's ties at a block-scanned offset
  const uint32_t nt = __popc(tmask & vmask);
  const uint32_t tinc = wave_incl_sum<uint32_t>(nt);
  uint32_t* const wt = reinterpret_cast<uint32_t*>(&sh.rv[0][0]);   // rv is free after the load
  if (lane == 63) wt[wv] = tinc;
  __syncthreads();
  if (tid == 0) {
    uint32_t tot = 0;
#pragma unroll
    for (int w = 0; w < BS_W; ++w) tot += wt[w];
    const uint64_t b = tot ? atomicAdd(tie_n, (unsigned long long)tot) : 0ull;
    sh.rv[1][0] = b;
  }
  __syncthreads();
  uint64_t tpos = sh.rv[1][0];   // the wave's ties follow the earlier waves' (slot order: wave-major)
  for (uint32_t w = 0; w < wv; ++w) tpos += wt[w];
  __syncthreads();

  // ---- SA / BWT in sorted order: the positions are loaded coalesced in original order, staged in
  // LDS by original slot and read back by the sorted index (no random global gathers)
  if (TRACE) ts[3] = stamp();
#pragma unroll
  for (int k = 0; k < BS_I; ++k)
    if ((vmask >> k) & 1u) sh.buf[s0 + 64u * k] = vv[k];
  __syncthreads();
  if (TRACE) ts[4] = stamp();
#pragma unroll
  for (int k = 0; k < BS_I; ++k) {
    const uint32_t r = s0 + 64u * k;
    const bool valid = (vmask >> k) & 1u;
    V p = 0;
    if (valid) {
      const uint32_t o = half(ix2, k);
      const uint32_t pv = packprev ? (klo[k] >> width) & ((1u << (pb + hb)) - 1) : (uint32_t)sh.aux[o];
      p = (V)(((uint64_t)(pv >> pb) << 32) | sh.buf[o]);
      sab[r] = p;
      bwb[r] = sh.inv[pv & pmask];
    }
    // in slot order (inside a wave: k-major, lane-minor), so that each group's records are consecutive
    // in the tie list and its head comes first
    const bool tie = valid && ((tmask >> k) & 1u);
    const uint64_t tb = ballot64(tie);
    if (tie) {
      const uint64_t at = tpos + mbcnt(tb);
      tie_k[at] = (((uint64_t)start + r) << 1) | ((hmask >> k) & 1u);
      tie_v[at] = p;
    }
    tpos += (uint32_t)__popcll(tb);
  }
  if (TRACE) {
    ts[5] = stamp();
    if (tid == 0)
      for (int i = 0; i < 8; ++i) trace[(uint64_t)item * 8 + i] = ts[i];
  }
}

// One workgroup per work item (one per CU at a time: the sort takes 158 KiB of LDS).
template <bool WIDE, bool TRACE = false, typename V = uint32_t>
__global__ __launch_bounds__(BS_T, 1) void k_bucket_sort(const uint64_t* __restrict__ keys,
                                                         const uint32_t* __restrict__ vals,
                                                         const uint2* __restrict__ items, int pb, int sb, int hb,
                                                         uint64_t symbias,
                                                         const uint8_t* __restrict__ inv, V* __restrict__ sa,
                                                         uint8_t* __restrict__ bwt, uint64_t* __restrict__ tie_k,
                                                         V* __restrict__ tie_v,
                                                         unsigned long long* __restrict__ tie_n,
                                                         uint64_t* __restrict__ trace) {
  __shared__ BsShared sh;
  if (threadIdx.x < 256) sh.inv[threadIdx.x] = inv[threadIdx.x];
  const uint2 it = items[blockIdx.x];
  uint64_t key[BS_I];
  bs_load_keys(keys, it, key);
  bucket_sort_item<WIDE, TRACE, V>(sh, it, key, blockIdx.x, keys, vals, pb, sb, hb, symbias, sa, bwt, tie_k,
                                   tie_v, tie_n, trace);
}

// Fast-path kernel: the same prologue (the item's sym range and varying bits), then the MSD + bin-rank
// sort; items it cannot take (wide keys, a bin over BF_MAXBIN) are appended to `fb` for k_bucket_sort.
// X32 (packed records whose sym field starts at bit >= 32): the sym is the record's high word shifted,
// so the prologue and the local keys work in 32-bit arithmetic.
template <typename V, bool TRACE, int T, int I, bool PK = false, bool X32 = false>
__global__ __launch_bounds__(T, (T * I <= 9216 ? 2 : 1) * T / 256) void k_bucket_sort_fast(const uint64_t* __restrict__ keys,
                                                              const uint32_t* __restrict__ vals,
                                                              const uint2* __restrict__ items, int pb, int sb, int hb,
                                                              uint64_t symbias, const uint8_t* __restrict__ inv,
                                                              V* __restrict__ sa, uint8_t* __restrict__ bwt,
                                                              uint64_t* __restrict__ tie_k, V* __restrict__ tie_v,
                                                              unsigned long long* __restrict__ tie_n,
                                                              uint2* __restrict__ fb, unsigned int* __restrict__ fb_n,
                                                              uint64_t* __restrict__ trace, PkGeom pg) {
  __shared__ BfShared<T, I> sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t ts[8] = {0};
  if (TRACE) ts[0] = stamp();
  // packed records with keyed prev codes: code c is dense code c + (c >= tcode), position 0's is the terminal
  const bool remap = PK && pg.tcode >= 0;
  if (tid < 256) sh.inv[tid] = inv[remap && tid >= (uint32_t)pg.tcode ? tid + 1 : tid];   // inv holds 512 entries
  const int term = remap ? (int)inv[pg.tcode] : -1;
  const int pbits = PK ? pg.pbits : 0;
  pb = PK ? pg.pb2 : pb;
  const uint2 it = items[blockIdx.x];
  const uint32_t s0 = wv * (I * 64) + lane;   // slot k of this thread: s0 + 64 k
  uint64_t key[I];
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < I; ++k) {
    key[k] = s0 + 64u * k < it.y ? keys[it.x + s0 + 64u * k] : 0;
    vmask |= (s0 + 64u * k < it.y ? 1u : 0u) << k;
  }

  const uint64_t symmask = sb >= 64 ? ~0ull : ((1ull << sb) - 1);
  const int pbe = pb + hb;
  for (uint32_t i = tid; i < (uint32_t)BfShared<T, I>::BINS / 2; i += T) sh.H2[i] = 0;
  // the sym fields once (key -> sym - symbias in place, the BWT code / position bits to pvr), then one
  // reduction of min, max, or, and: the low varying bit of the values is that of the values relative
  // to the minimum, and the relative width is bits((max - min) >> lo).  Branch-free over the item's
  // end (neutral values) for X32, so no record's fields wait in scratch across a masked block.
  using XT = std::conditional_t<X32, uint32_t, uint64_t>;
  const int xsh = pbits + pbe;   // packed: the sym field's first bit in the record
  const uint32_t pmask = (1u << pb) - 1, himask = (1u << hb) - 1;
  uint32_t pvr[(I + 1) / 2];
  XT xmin = (XT)~0ull, xmax = 0, vor = 0, vand = (XT)~0ull;
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const bool valid = (vmask >> k) & 1u;
    uint32_t pv;
    XT x;
    if (X32) {
      pv = (uint32_t)(key[k] >> pbits) & pmask;   // hb = 0, symbias = 0
      // u64 positions: their bits above 32 ride with the prev code (SA / tie values reassemble them)
      if (sizeof(V) == 8) pv |= ((uint32_t)(key[k] >> 32) & ((1u << pg.phb) - 1)) << pb;
      x = (XT)((uint32_t)(key[k] >> 32) >> (xsh - 32));
    } else {
      const uint64_t kl = PK ? key[k] >> pbits : key[k];   // packed: the record stays (positions)
      pv = ((uint32_t)(kl >> hb) & pmask) | (((uint32_t)kl & himask) << pb);
      x = (XT)(((kl >> pbe) & symmask) - symbias);
      if (!PK) key[k] = x;
    }
    if (k < (I + 1) / 2) pvr[k] = pv; else pvr[k - (I + 1) / 2] |= pv << 16;
    if (X32) {   // selects: no masked block (the 64-bit variants keep less live with the branch)
      xmin = valid && x < xmin ? x : xmin;
      xmax = valid && x > xmax ? x : xmax;
      vor |= valid ? x : (XT)0;
      vand &= valid ? x : (XT)~0ull;
    } else if (valid) {
      xmin = x < xmin ? x : xmin;
      xmax = x > xmax ? x : xmax;
      vor |= x;
      vand &= x;
    }
  }
  if constexpr (X32) {   // u32 fields: DPP reductions (no ds_bpermute round trips)
    xmin = dpp_reduce_u32(xmin, ~0u, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
    xmax = dpp_reduce_u32(xmax, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
    vor = dpp_reduce_u32(vor, 0u, [](uint32_t a, uint32_t b) { return a | b; });
    vand = dpp_reduce_u32(vand, ~0u, [](uint32_t a, uint32_t b) { return a & b; });
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const XT a0 = __shfl_xor(xmin, o, 64), a1 = __shfl_xor(xmax, o, 64);
      xmin = a0 < xmin ? a0 : xmin;
      xmax = a1 > xmax ? a1 : xmax;
      vor |= __shfl_xor(vor, o, 64);
      vand &= __shfl_xor(vand, o, 64);
    }
  }
  XT* const red = reinterpret_cast<XT*>(sh.red);   // [4][(T / 64)]
  if (lane == 0) {
    red[wv] = xmin;
    red[(T / 64) + wv] = xmax;
    red[2 * (T / 64) + wv] = vor;
    red[3 * (T / 64) + wv] = vand;
  }
  __syncthreads();
#pragma unroll
  for (int w = 0; w < (T / 64); ++w) {
    xmin = red[w] < xmin ? red[w] : xmin;
    xmax = red[(T / 64) + w] > xmax ? red[(T / 64) + w] : xmax;
    vor |= red[2 * (T / 64) + w];
    vand &= red[3 * (T / 64) + w];
  }
  const uint64_t var = (uint64_t)(vor ^ vand);
  const int lo = var ? __builtin_ctzll(var) : 0;
  const uint64_t span = (uint64_t)(xmax - xmin) >> lo;
  const int width = var ? 64 - __builtin_clzll(span) : 0;
  if (TRACE) ts[1] = stamp();
  const bool ok = width >= 1 && width <= 30 &&
                  bucket_sort_fast<V, TRACE, T, I, PK, X32>(sh, it, key, pvr, vmask, s0, (uint64_t)xmin, lo, width, pb,
                                                         xsh, pbits, term, vals + it.x,
                                             sa + it.x, bwt + it.x, tie_k, tie_v, tie_n, ts);
  if (!ok && tid == 0) fb[atomicAdd(fb_n, 1u)] = it;
  if (TRACE) {
    ts[7] = stamp();
    if (tid == 0)
      for (int i = 0; i < 8; ++i) trace[(uint64_t)blockIdx.x * 8 + i] = ts[i];
  }
}

// ---- record-plane sort (k_bucket_sort_rec): the 1 GiB sigma <= 8 headline's items
// One 512-thread workgroup per item of <= BR_CAP suffixes, packed records whose sym field lies in the high
// word (X32), u32 positions, prev codes of <= 3 bits.  The fast path above moves a suffix through four
// planes (u32 position by slot, u32 record by bin, u16 final index by slot, then u32 position and u16 prev
// code by final index): five random LDS accesses and ~9 barriers per item.  Here the record itself is
// the unit: the item's sym range fixes all but `width` key bits, the top 13 of them pick one of 8192 bins
// (u8 counters: the atomic's return is the rank inside the bin), and the record goes to its bin as ONE u64
// whose sym field is replaced by the key bits below the bin: (low key << xsh) | prev code << pbits |
// position.  The plane is then ordered bin by bin in place by plain u64 compares (the low key decides;
// equal low keys are equal keys): ~37 % of the bins of iid text hold one record (nothing to do), pairs
// (~18 %) are settled by the thread that owns their group of 16 bins, four per lane with their reads in
// flight together, and bins of 3+ records (~8 %) are listed and ranked one per thread.  The plane - now
// at final index + the SA pointer's misalignment - is written out as aligned 16-B SA / 4-B BWT groups.
// Two random LDS accesses per suffix where the fast path has five, seven barriers.  Round 6 on MI355X,
// 1 GiB sigma = 4 items: 4.70 -> 4.13 ms per launch; per-item cycles per phase by HKCSA_BS_TRACE=1
// in DESIGN.md section 4.  Slower variants measured and dropped: one thread per group settling all its
// bins in loops (dependent LDS chains: 4.9-6.0 ms), every record ranking itself against its bin (more LDS
// bytes), pairs and triples in one unconditional pass, 3+ bins by their owners, a four-record network for
// 3- and 4-record bins, and persistent workgroups prefetching the next item (5.5 ms).  The u8 counters
// need bins of < 64 records and groups of < 256 (checked by the counts' total and bit tests); items
// outside that, with local keys wider than 30 bits, or with a thread holding more than two tie runs go
// to the LSD passes (fb).  LDS: 81,904 B, two workgroups per CU.
constexpr int BR_T = 512, BR_I = 18;
constexpr int BR_BITS = 13, BR_BINS = 1 << BR_BITS, BR_NG = BR_BINS / 16;   // 16 bins per group, a group per thread
static_assert(BR_NG == BR_T, "one bin group per thread");
static_assert(BR_CAP <= (uint32_t)BR_T * BR_I, "capacity within the threads' slots");

struct alignas(16) BrShared {
  uint64_t rec[BR_CAP + 4];        // records at final index + al (al < 4)
  uint32_t cnt[BR_BINS / 4];       // u8 bin counters, then in-group exclusive prefixes
  uint16_t base[BR_NG + 8];        // group starts (+ al); [BR_NG] = count + al; [BR_NG + 4 ..] code table
  uint32_t scr[48];                // reductions / wave totals / failure flags / tie base
};
static_assert(sizeof(BrShared) <= 81920, "two workgroups per CU");

// X32: the sym field starts at bit >= 32 (texts of 2^30 suffixes and more, slices), so the prologue works in
// 32-bit arithmetic; else it is the record's bits >= xsh as a u64.
template <typename V, bool TRACE = false, bool X32 = true>
__global__ __launch_bounds__(BR_T, 4) void k_bucket_sort_rec(const uint64_t* __restrict__ keys,
                                                          const uint2* __restrict__ items,
                                                          const uint8_t* __restrict__ inv, V* __restrict__ sa,
                                                          uint8_t* __restrict__ bwt, uint64_t* __restrict__ tie_k,
                                                          V* __restrict__ tie_v,
                                                          unsigned long long* __restrict__ tie_n,
                                                          uint2* __restrict__ fb, unsigned int* __restrict__ fb_n,
                                                          PkGeom pg, uint64_t* __restrict__ trace = nullptr) {
  __shared__ BrShared sh;
  uint64_t ts[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (TRACE) ts[0] = stamp();
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint2 it = items[blockIdx.x];
  const uint32_t start = it.x, cnt = it.y;
  const int pbits = pg.pbits, pb = pg.pb2, xsh = pbits + pb;   // (X32: xsh >= 32)
  // the BWT byte of each keyed prev code (codes at or above the unique terminal's shift up by one)
  const bool remap = pg.tcode >= 0;
  uint8_t* const tab = reinterpret_cast<uint8_t*>(sh.base + BR_NG + 4);
  const uint32_t s0 = wv * (BR_I * 64) + lane;   // slot k of this thread: s0 + 64 k
  uint64_t key[BR_I];
  uint32_t vmask = 0;
#pragma unroll
  for (int k = 0; k < BR_I; ++k) {
    const bool valid = s0 + 64u * k < cnt;
    key[k] = valid ? keys[start + s0 + 64u * k] : 0;
    vmask |= (valid ? 1u : 0u) << k;
  }
  // (after the record loads: the table byte's wait then covers nothing the prologue does not need anyway)
  const uint8_t tv = tid < 8 ? inv[remap && tid >= (uint32_t)pg.tcode ? tid + 1 : tid] : 0;
  const int term = remap ? (int)inv[pg.tcode] : -1;
  reinterpret_cast<uint4*>(sh.cnt)[tid] = make_uint4(0u, 0u, 0u, 0u);   // the 8192 u8 counters
  using XT = std::conditional_t<X32, uint32_t, uint64_t>;
  auto symx = [&](int k) -> XT {
    if constexpr (X32) return (uint32_t)(key[k] >> 32) >> (xsh - 32);
    else return key[k] >> xsh;
  };
  // ---- 0. the item's sym range: min, max, or, and (the varying bits are those of the values relative
  // to the minimum)
  XT xmin = (XT)~0ull, xmax = 0, vor = 0, vand = (XT)~0ull;
#pragma unroll
  for (int k = 0; k < BR_I; ++k) {
    const bool valid = (vmask >> k) & 1u;
    const XT x = symx(k);
    xmin = valid && x < xmin ? x : xmin;
    xmax = valid && x > xmax ? x : xmax;
    vor |= valid ? x : (XT)0;
    vand &= valid ? x : (XT)~0ull;
  }
  // the per-wave results through LDS: u32 in scr (X32), u64 in the record plane (free until phase 3)
  XT* const red = X32 ? reinterpret_cast<XT*>(sh.scr) : reinterpret_cast<XT*>(sh.rec);
  if constexpr (X32) {
    xmin = dpp_reduce_u32(xmin, ~0u, [](uint32_t a, uint32_t b) { return a < b ? a : b; });
    xmax = dpp_reduce_u32(xmax, 0u, [](uint32_t a, uint32_t b) { return a > b ? a : b; });
    vor = dpp_reduce_u32(vor, 0u, [](uint32_t a, uint32_t b) { return a | b; });
    vand = dpp_reduce_u32(vand, ~0u, [](uint32_t a, uint32_t b) { return a & b; });
  } else {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const XT a0 = __shfl_xor(xmin, o, 64), a1 = __shfl_xor(xmax, o, 64);
      xmin = a0 < xmin ? a0 : xmin;
      xmax = a1 > xmax ? a1 : xmax;
      vor |= __shfl_xor(vor, o, 64);
      vand &= __shfl_xor(vand, o, 64);
    }
  }
  if (lane == 0) {
    red[wv] = xmin;
    red[8 + wv] = xmax;
    red[16 + wv] = vor;
    red[24 + wv] = vand;
  }
  if (tid < 8) tab[tid] = tv;
  __syncthreads();
#pragma unroll
  for (int w = 0; w < BR_T / 64; ++w) {
    xmin = red[w] < xmin ? red[w] : xmin;
    xmax = red[8 + w] > xmax ? red[8 + w] : xmax;
    vor |= red[16 + w];
    vand &= red[24 + w];
  }
  if (TRACE) ts[1] = stamp();
  const uint64_t var = (uint64_t)(vor ^ vand);
  const int lo = var ? __builtin_ctzll(var) : 0;
  const uint64_t spanx = (uint64_t)(xmax - xmin) >> lo;
  const int width = var ? 64 - __builtin_clzll(spanx) : 0;
  auto fallback = [&]() {
    if (tid == 0) fb[atomicAdd(fb_n, 1u)] = it;
  };
  if (width < 1 || width > 30) {   // (uniform) all keys equal, or wider than the records' low field
    fallback();
    return;
  }
  const int kb = width > BR_BITS ? width - BR_BITS : 0;   // key bits below the bin (<= 17)
  const uint32_t wmask = (1u << width) - 1, lowmask = (1u << kb) - 1;
  auto local = [&](int k) -> uint32_t { return (uint32_t)((symx(k) - xmin) >> lo) & wmask; };
  // ---- 1. u8 bin counters; the atomic's return is the suffix's rank inside its bin
  uint32_t rk[(BR_I + 3) / 4];
#pragma unroll
  for (int k = 0; k < (BR_I + 3) / 4; ++k) rk[k] = 0;
#pragma unroll
  for (int k = 0; k < BR_I; ++k) {
    if ((vmask >> k) & 1u) {
      const uint32_t bin = local(k) >> kb, sh8 = 8u * (bin & 3u);
      const uint32_t r = (atomicAdd(&sh.cnt[bin >> 2], 1u << sh8) >> sh8) & 0xFFu;
      rk[k >> 2] |= r << (8 * (k & 3));
    }
  }
  __syncthreads();
  if (TRACE) ts[2] = stamp();
  // ---- 2. group starts: thread t owns bins 16 t .. 16 t + 15 (one 16-B word of counters)
  const uint32_t al = (uint32_t)(((uintptr_t)(sa + start) / sizeof(V)) & 3u);
  const bool vec = al == (uint32_t)((uintptr_t)(bwt + start) & 3u);
  const uint32_t sto = vec ? al : 0u;   // the plane's offset: 4 staged records = one aligned SA group
  uint32_t pre[4], gs = 0;
  bool bad = false;
  {
    const uint4 c4 = reinterpret_cast<const uint4*>(sh.cnt)[tid];
    const uint32_t w[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      // in-group exclusive prefix per byte: exact while no bin reaches 64 and the group stays below 256
      pre[i] = w[i] * 0x01010101u - w[i] + gs * 0x01010101u;
      gs += __builtin_amdgcn_udot4(w[i], 0x01010101u, 0u, false);
      bad |= (w[i] & 0xC0C0C0C0u) != 0;
    }
    bad |= gs > 255;
  }
  const uint32_t ginc = dpp_incl_sum(gs);
  const uint64_t badw = __ballot(bad);
  if (lane == 63) sh.scr[32 + wv] = ginc;
  if (lane == 0) sh.scr[40 + wv] = badw ? 1u : 0u;
  __syncthreads();
  uint32_t carry = 0, total = 0, fail = 0;
#pragma unroll
  for (int w = 0; w < BR_T / 64; ++w) {
    const uint32_t t = sh.scr[32 + w];
    carry += (uint32_t)w < wv ? t : 0u;
    total += t;
    fail |= sh.scr[40 + w];
  }
  // (a u8 counter that wrapped carried into its neighbour or out of the word: the total shows it)
  if (fail || total != cnt) {
    fallback();
    return;
  }
  const uint32_t gb = sto + carry + ginc - gs;   // this group's first index in the plane
  sh.base[tid] = (uint16_t)gb;
  if (tid == BR_T - 1) sh.base[BR_NG] = (uint16_t)(sto + cnt);
  reinterpret_cast<uint4*>(sh.cnt)[tid] = make_uint4(pre[0], pre[1], pre[2], pre[3]);
  __syncthreads();
  if (TRACE) ts[3] = stamp();
  // ---- 3. every record to its bin: (low key << xsh) | (prev code, position).  Branch-free over the
  // item's end (invalid slots read group 0's entries and store nothing), chunks of 6 records' loads in
  // flight together (register pressure)
  {
    const uint8_t* const pre8 = reinterpret_cast<const uint8_t*>(sh.cnt);
    const uint64_t lom = (1ull << xsh) - 1;
#pragma unroll
    for (int k = 0; k < BR_I; ++k) {
      if (k % 6 == 0 && k) asm volatile("" ::: "memory");
      const bool valid = (vmask >> k) & 1u;
      const uint32_t lk = local(k), bin = valid ? lk >> kb : 0u;
      const uint32_t bs = sh.base[bin >> 4] + pre8[bin];
      const uint32_t r = (rk[k >> 2] >> (8 * (k & 3))) & 0xFFu;
      if (valid) sh.rec[bs + r] = ((uint64_t)(lk & lowmask) << xsh) | (key[k] & lom);
    }
  }
  const uint32_t ge = sh.base[tid + 1];   // (written before the last barrier)
  if (tid == 0) {   // (phase 2's flags were read before its last barrier)
    sh.scr[40] = 0;
    sh.scr[41] = 0;
    sh.scr[42] = 0;
  }
  __syncthreads();
  if (TRACE) ts[4] = stamp();
  // ---- 4. the bins in place.  Two-record bins (~18 % of the bins for iid text) by their group's thread:
  // one compare, all 16 bins' pairs read unconditionally in two batches of 8 (branch-free: a batch's reads
  // in flight together).  Bins of 3+ records (~8 %) go to a list in the counters' space (free now) and are
  // ranked one per thread: up to 8 records read at once and ranked by compares in registers, more (rare)
  // by insertion.  Equal keys (same bin, same low key) form a tie run; a thread keeps up to two runs
  // {first index, length} for the tie list (a third sends the item to the LSD passes).
  auto kx = [&](uint64_t r) -> uint64_t { return r >> xsh; };
  // (i may be run-time: two u64 halves and a shift, so that no register array is indexed - the compiler
  // turns a select chain over pre[] back into a scratch array)
  const uint64_t pre_lo = (uint64_t)pre[1] << 32 | pre[0], pre_hi = (uint64_t)pre[3] << 32 | pre[2];
  auto bstart = [&](int i) -> uint32_t {
    return gb + ((uint32_t)((i < 8 ? pre_lo : pre_hi) >> (8 * (i & 7))) & 0xFFu);
  };
  auto bend = [&](int i) -> uint32_t { return i < 15 ? bstart(i + 1) : ge; };
  uint32_t ltie = 0, run0 = 0, run1 = 0, nrun = 0;   // (two scalars: no dynamically indexed array)
  auto add_run = [&](uint32_t f, uint32_t len) {
    run0 = nrun == 0 ? f | len << 16 : run0;
    run1 = nrun == 1 ? f | len << 16 : run1;
    ++nrun;
    ltie += len;
  };
  // the pair bins of this group (a mask), then up to four pairs per lane with their reads in flight together,
  // the rest (lanes with more than four, ~7 % of them) one by one
  uint32_t m2 = 0, m3 = 0;
#pragma unroll
  for (int b = 0; b < 16; ++b) {
    const uint32_t c = bend(b) - bstart(b);
    m2 |= (c == 2 ? 1u : 0u) << b;
    m3 |= (c >= 3 ? 1u : 0u) << b;
  }
  auto pair = [&](uint32_t bs, uint64_t x, uint64_t y) {
    if (x > y) {
      sh.rec[bs] = y;
      sh.rec[bs + 1] = x;
    }
    if (kx(x) == kx(y)) add_run(bs, 2);
  };
  {
    uint32_t pa[4];
    uint64_t px[4], py[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {   // lanes out of pairs read records 0 and 1 (one broadcast address)
      const int b = m2 ? __builtin_ctz(m2) : 0;
      const uint32_t a = m2 ? bstart(b) : 0u;
      pa[j] = m2 ? a : ~0u;
      m2 &= m2 - 1;
      px[j] = sh.rec[a];
      py[j] = sh.rec[a + 1];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (pa[j] != ~0u) pair(pa[j], px[j], py[j]);
  }
  while (m2) {
    const uint32_t a = bstart(__builtin_ctz(m2));
    m2 &= m2 - 1;
    pair(a, sh.rec[a], sh.rec[a + 1]);
  }
  // {start | size << 16} of the 3+ bins: three-record bins from the front of the counters' space, larger
  // ones from its back, so that each loop below runs one code path per wave
  uint32_t* const blist = sh.cnt;
  constexpr uint32_t BL = BR_BINS / 4;
  {
    uint32_t m3only = 0;
#pragma unroll
    for (int b = 0; b < 16; ++b) m3only |= ((m3 >> b) & 1u) && bend(b) - bstart(b) == 3 ? 1u << b : 0u;
    uint32_t m4 = m3 & ~m3only;
    const uint32_t n3 = __popc(m3only), n4 = __popc(m4);
    const uint32_t binc = dpp_incl_sum(n3 | n4 << 16);   // (both <= 64 * 16)
    uint32_t wb = 0;
    if (lane == 63) wb = atomicAdd(&sh.scr[40], binc & 0xFFFFu) | atomicAdd(&sh.scr[42], binc >> 16) << 16;
    wb = (uint32_t)__builtin_amdgcn_readlane((int)wb, 63);
    uint32_t w3 = (wb & 0xFFFFu) + (binc & 0xFFFFu) - n3, w4 = (wb >> 16) + (binc >> 16) - n4;
    while (m3only) {
      const int b = __builtin_ctz(m3only);
      m3only &= m3only - 1;
      if (w3 < BL) blist[w3] = bstart(b) | 3u << 16;
      ++w3;
    }
    while (m4) {
      const int b = __builtin_ctz(m4);
      m4 &= m4 - 1;
      if (w4 < BL) blist[BL - 1 - w4] = bstart(b) | (bend(b) - bstart(b)) << 16;
      ++w4;
    }
  }
  __syncthreads();
  if (TRACE) ts[5] = stamp();
  const uint32_t nb3 = sh.scr[40], nb4 = sh.scr[42];
  if (nb3 + nb4 > BL) {   // (uniform) a skewed item
    fallback();
    return;
  }
  for (uint32_t i = tid; i < nb3; i += BR_T) {   // three records: a network
    const uint32_t bs = blist[i] & 0xFFFFu;
    uint64_t x = sh.rec[bs], y = sh.rec[bs + 1], z = sh.rec[bs + 2];
    auto cas = [](uint64_t& a, uint64_t& c2) {
      const uint64_t lo2 = a < c2 ? a : c2, hi2 = a < c2 ? c2 : a;
      a = lo2;
      c2 = hi2;
    };
    cas(x, y);
    cas(y, z);
    cas(x, y);
    sh.rec[bs] = x;
    sh.rec[bs + 1] = y;
    sh.rec[bs + 2] = z;
    const bool exy = kx(x) == kx(y), eyz = kx(y) == kx(z);
    if (exy || eyz) add_run(exy ? bs : bs + 1, exy && eyz ? 3u : 2u);
  }
  for (uint32_t i = tid; i < nb4; i += BR_T) {   // four or more
    const uint32_t e = blist[BL - 1 - i], bs = e & 0xFFFFu, c = e >> 16;
    if (c <= 8) {
      uint64_t r[8], kr[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // unconditional (past the plane's end: the lists' words); pads rank last
        const uint64_t v = sh.rec[bs + q];
        r[q] = (uint32_t)q < c ? v : ~0ull;
        kr[q] = kx(v);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        uint32_t rank = 0, eqn = 0, eqb = 0;
#pragma unroll
        for (int o = 0; o < 8; ++o) {
          if (o == q) continue;
          const bool lt = r[o] < r[q], e2 = (uint32_t)o < c && kr[o] == kr[q];
          rank += lt ? 1u : 0u;
          eqn += e2 ? 1u : 0u;
          eqb += e2 && lt ? 1u : 0u;
        }
        if ((uint32_t)q < c) {
          sh.rec[bs + rank] = r[q];
          if (eqn && !eqb) add_run(bs + rank, eqn + 1);
        }
      }
      continue;
    }
    const uint32_t be = bs + c;
    for (uint32_t p = bs + 1; p < be; ++p) {
      const uint64_t v = sh.rec[p];
      uint32_t q = p;
      while (q > bs) {
        const uint64_t u = sh.rec[q - 1];
        if (u < v) break;
        sh.rec[q] = u;
        --q;
      }
      sh.rec[q] = v;
    }
    uint32_t rs = bs;
    uint64_t kprev = kx(sh.rec[bs]);
    for (uint32_t p = bs + 1; p <= be; ++p) {
      const uint64_t kp = p < be ? kx(sh.rec[p]) : ~0ull;   // (keys < 2^64 >> xsh: ~0 ends the last run)
      if (kp != kprev) {
        if (p - rs >= 2) add_run(rs, p - rs);
        rs = p;
        kprev = kp;
      }
    }
  }
  if (nrun > 2) sh.scr[41] = 1u;   // (any thread: the flag is read after the next barrier)
  const uint32_t tinc = dpp_incl_sum(ltie);
  if (lane == 63) sh.scr[wv] = tinc;
  __syncthreads();
  if (TRACE) ts[6] = stamp();
  if (sh.scr[41]) {   // (uniform) a thread with more than two tie runs: the LSD passes list them
    fallback();
    return;
  }
  uint32_t tcar = 0, ntie = 0;
#pragma unroll
  for (int w = 0; w < BR_T / 64; ++w) {
    const uint32_t t = sh.scr[w];
    tcar += (uint32_t)w < wv ? t : 0u;
    ntie += t;
  }
  unsigned long long tbase = 0;
  if (tid == 0 && ntie) tbase = atomicAdd(tie_n, (unsigned long long)ntie);
  // ---- 5. SA / BWT in sorted order straight from the plane
  // u64 positions (slices of texts past 2^32): the position is the record's low pbits = 32 + phb bits
  const uint64_t posm = (1ull << pbits) - 1;
  const uint32_t pmask = (1u << pb) - 1;
  auto bwt_of = [&](uint64_t r) -> uint32_t {
    const uint32_t pv = (uint32_t)(r >> pbits) & pmask;
    return (r & posm) == 0 && term >= 0 ? (uint32_t)term : (uint32_t)tab[pv];
  };
  if (vec) {
    const uint32_t ng = (cnt + al + 3) >> 2;
    const uint32_t tlo = reinterpret_cast<const uint32_t*>(tab)[0], thi = reinterpret_cast<const uint32_t*>(tab)[1];
    for (uint32_t q = tid; q < ng; q += BR_T) {
      const uint4 ra = reinterpret_cast<const uint4*>(sh.rec)[2 * q];
      const uint4 rb = reinterpret_cast<const uint4*>(sh.rec)[2 * q + 1];
      const uint32_t lo4[4] = {ra.x, ra.z, rb.x, rb.z}, hi4[4] = {ra.y, ra.w, rb.y, rb.w};
      uint64_t pos[4];
      uint32_t sel = 0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t r = ((uint64_t)hi4[j] << 32) | lo4[j];
        pos[j] = r & posm;
        sel |= ((uint32_t)(r >> pbits) & pmask) << (8 * j);
      }
      uint32_t bw = __builtin_amdgcn_perm(thi, tlo, sel);
      if (term >= 0) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (pos[j] == 0) bw = (bw & ~(0xFFu << (8 * j))) | ((uint32_t)term << (8 * j));
      }
      const uint32_t g = 4u * q;
      if (g >= al && g + 4 <= cnt + al) {   // a whole group: aligned vector stores
        if constexpr (sizeof(V) == 4) {
          *reinterpret_cast<uint4*>(sa + start + (g - al)) =
              make_uint4((uint32_t)pos[0], (uint32_t)pos[1], (uint32_t)pos[2], (uint32_t)pos[3]);
        } else {
          uint4* const d4 = reinterpret_cast<uint4*>(sa + start + (g - al));
          d4[0] = make_uint4((uint32_t)pos[0], (uint32_t)(pos[0] >> 32), (uint32_t)pos[1], (uint32_t)(pos[1] >> 32));
          d4[1] = make_uint4((uint32_t)pos[2], (uint32_t)(pos[2] >> 32), (uint32_t)pos[3], (uint32_t)(pos[3] >> 32));
        }
        *reinterpret_cast<uint32_t*>(bwt + start + (g - al)) = bw;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const uint32_t r = g + j;
          if (r >= al && r < cnt + al) {
            sa[start + r - al] = (V)pos[j];
            bwt[start + r - al] = (uint8_t)(bw >> (8 * j));
          }
        }
      }
    }
  } else {
    for (uint32_t r = tid; r < cnt; r += BR_T) {
      const uint64_t x = sh.rec[r];
      sa[start + r] = (V)(x & posm);
      bwt[start + r] = (uint8_t)bwt_of(x);
    }
  }
  if (ntie) {   // (uniform) each thread's tie runs: a group's records consecutive, head first
    if (tid == 0) {
      sh.scr[8] = (uint32_t)tbase;
      sh.scr[9] = (uint32_t)(tbase >> 32);
    }
    __syncthreads();
    if (ltie) {
      uint64_t tb = ((uint64_t)sh.scr[9] << 32 | sh.scr[8]) + tcar + tinc - ltie;
      auto put = [&](uint32_t f, uint32_t len) {
        for (uint32_t j = 0; j < len; ++j) {
          tie_k[tb + j] = ((uint64_t)(start + f + j - sto) << 1) | (j == 0 ? 1u : 0u);
          tie_v[tb + j] = (V)(sh.rec[f + j] & posm);
        }
        tb += len;
      };
      if (nrun > 0) put(run0 & 0xFFFFu, run0 >> 16);
      if (nrun > 1) put(run1 & 0xFFFFu, run1 >> 16);
    }
  }
  if (TRACE) {
    ts[7] = stamp();
    if (tid == 0)
      for (int i = 0; i < 8; ++i) trace[(uint64_t)blockIdx.x * 8 + i] = ts[i];
  }
}

}  // namespace

// Launches the LDS sorts of the plan's work items over the bucket-grouped (keys, vals) or packed
// records (pk); writes sa / bwt in sorted order and appends the tied suffixes to ix.ties_*; returns
// the tie count.
template <typename V>
uint64_t sort_bucket_items(Index& ix, const BucketPlan& plan, const uint64_t* keys, const uint32_t* vals, uint64_t m,
                           int pb, int sb, int hb, uint64_t symbias, V* sa, uint8_t* bwt,
                           const PackedRecs* pk) {
  hipStream_t s = ix.stream;
  if (pk && (hb || symbias)) throw ApiError{-1, "packed records: no key-plane position bits or sym bias"};
  if (pk && sizeof(V) == 4 && (pk->g.phb || pk->uhb)) throw ApiError{-1, "packed records: u64 positions need a u64 SA"};
  // the LSD item sorts read full keys: packed items are unpacked to (kfull, vfull) first (with the
  // position's high bits below the key for u64 positions)
  const uint64_t* lkeys = pk ? pk->kfull : keys;
  const uint32_t* lvals = pk ? pk->vfull : vals;
  const int lhb = pk ? pk->uhb : hb;
  const uint8_t* d_inv = ix.small.as<uint8_t>() + 3072;
  ix.ties_k.ensure(m * 8 + 16);
  ix.ties_v.ensure(m * sizeof(V) + 16);
  ix.ties_n.ensure(16);
  HK_HIP(hipMemsetAsync(ix.ties_n.p, 0, 8, s));
  const uint64_t nn = plan.items_n.size(), nw = plan.items_w.size();
  ix.bk_items.ensure((nn + nw) * sizeof(uint2) + 16);
  if (nn + nw) {
    // pinned staging: the copy is queued behind the partition passes without holding the host (the
    // ~37 us DMA of ~1 MB of items still runs between pass B and the sort).  The same copy on the
    // auxiliary stream, under pass B, was slower: passes A and B lost 0.1-0.15 ms each beside it.
    // The previous call's copy is complete (this function ends with a stream synchronize).
    ix.items_host.ensure((nn + nw) * sizeof(uint2));
    uint2* const hi = ix.items_host.as<uint2>();
    if (nn) memcpy(hi, plan.items_n.data(), nn * sizeof(uint2));
    if (nw) memcpy(hi + nn, plan.items_w.data(), nw * sizeof(uint2));
    HK_HIP(hipMemcpyAsync(ix.bk_items.p, hi, (nn + nw) * sizeof(uint2), hipMemcpyHostToDevice, s));
  }
  {
    TimedLaunch t(ix.timer, "sa_bucket_sort", (double)(m - plan.big_total) * (pk ? 8 + 4 + 1 : 8 + 4 + 4 + 1));
    // HKCSA_BS_TRACE=1: the phase-stamped build of the fast sort (diagnostic; identical results, tested)
    const bool trace = getenv("HKCSA_BS_TRACE") != nullptr;
    const unsigned grid_n = (unsigned)nn, grid_w = (unsigned)nw;
    DevBuf tbuf;
    if (nn) {
      if (trace) {
        tbuf.ensure(nn * 64 + 64);
        HK_HIP(hipMemsetAsync(tbuf.p, 0, nn * 64, s));
      }
      ix.bk_fb.ensure(nn * sizeof(uint2) + 16);
      unsigned int* fbn = reinterpret_cast<unsigned int*>(ix.small.as<uint8_t>() + 4352);   // small+4352: fallback count
      HK_HIP(hipMemsetAsync(fbn, 0, 4, s));
      bool used_rec = false;
      auto launch = [&](auto ttag, auto itag, auto trtag) {
        constexpr int T = decltype(ttag)::value;
        constexpr int I = decltype(itag)::value;
        constexpr bool TR = decltype(trtag)::value;
        if constexpr (T == 512) {
          // the record-plane sort: sigma <= 8 codes and room for (low key <= 17 bits) << xsh; u64 positions
          // as the record's low 32 + phb bits.  HKCSA_BS_REC=0 (read per call) keeps the fast path, for A/B.
          const char* rec_env = getenv("HKCSA_BS_REC");
          const bool rec_off = rec_env && rec_env[0] == '0';
          const int xsh = pk ? pk->g.pbits + pk->g.pb2 : 0;
          const bool pos_ok = pk && (pk->g.phb == 0 || (sizeof(V) == 8 && pk->g.pbits == 32 + pk->g.phb));
          if (pk && !rec_off && xsh + 17 <= 64 && pk->g.pb2 <= 3 && pos_ok && plan.cap <= (uint64_t)BR_CAP) {
            auto go = [&](auto kern) {
              kern<<<grid_n, BR_T, 0, s>>>(keys, ix.bk_items.as<uint2>(), d_inv, sa, bwt, ix.ties_k.as<uint64_t>(),
                                           ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(),
                                           ix.bk_fb.as<uint2>(), fbn, pk->g, trace ? tbuf.as<uint64_t>() : nullptr);
            };
            if (xsh >= 32) trace ? go(k_bucket_sort_rec<V, true, true>) : go(k_bucket_sort_rec<V, false, true>);
            else trace ? go(k_bucket_sort_rec<V, true, false>) : go(k_bucket_sort_rec<V, false, false>);
            used_rec = true;
            return;
          }
        }
        if (pk && pk->g.pbits + pk->g.pb2 >= 32) {   // sym fields in the records' high words
          k_bucket_sort_fast<V, TR, T, I, true, true><<<grid_n, T, 0, s>>>(
              keys, pk->vfull, ix.bk_items.as<uint2>(), pb, sb, hb, symbias, d_inv, sa, bwt,
              ix.ties_k.as<uint64_t>(), ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(), ix.bk_fb.as<uint2>(),
              fbn, TR ? tbuf.as<uint64_t>() : nullptr, pk->g);
          return;
        }
        if (pk) {
          k_bucket_sort_fast<V, TR, T, I, true><<<grid_n, T, 0, s>>>(
              keys, pk->vfull, ix.bk_items.as<uint2>(), pb, sb, hb, symbias, d_inv, sa, bwt,
              ix.ties_k.as<uint64_t>(), ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(), ix.bk_fb.as<uint2>(),
              fbn, TR ? tbuf.as<uint64_t>() : nullptr, pk->g);
          return;
        }
        k_bucket_sort_fast<V, TR, T, I><<<grid_n, T, 0, s>>>(
            keys, vals, ix.bk_items.as<uint2>(), pb, sb, hb, symbias, d_inv, sa, bwt, ix.ties_k.as<uint64_t>(),
            ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(), ix.bk_fb.as<uint2>(), fbn,
            TR ? tbuf.as<uint64_t>() : nullptr, PkGeom{});
      };
      using T512 = std::integral_constant<int, 512>;
      using T1024 = std::integral_constant<int, 1024>;
      using I18 = std::integral_constant<int, 18>;
      using TrOn = std::integral_constant<bool, true>;
      using TrOff = std::integral_constant<bool, false>;
      // (1024 threads of 9 suffixes for the half items, two workgroups per CU at 64 VGPRs, spilled and
      // ran 2x slower: 10.5 vs 5.3 ms at 1 GiB)
      if (plan.cap <= (uint64_t)512 * BS_I) {
        if (trace) launch(T512{}, I18{}, TrOn{}); else launch(T512{}, I18{}, TrOff{});
      } else {
        launch(T1024{}, I18{}, TrOff{});   // (the phase stamps: 512-thread items only; the 1024-thread build spilled)
      }
      HK_HIP(hipGetLastError());
      if (trace) {
        std::vector<uint64_t> h(nn * 8);
        HK_HIP(hipMemcpyAsync(h.data(), tbuf.p, h.size() * 8, hipMemcpyDeviceToHost, s));
        HK_HIP(hipStreamSynchronize(s));
        double acc[7] = {0, 0, 0, 0, 0, 0, 0};
        for (size_t w = 0; w < nn; ++w)
          for (int i = 0; i < 7; ++i) acc[i] += (double)(h[w * 8 + i + 1] - h[w * 8 + i]);
        // (fast sort: load+prologue, hist, scan, scatter, small bins, listed bins, stage+out; record-plane
        // sort: load+prologue, hist, scan, scatter, pairs + lists, 3+ bins, output + ties)
        fprintf(stderr, "[bucket_sort trace] %s sort, %zu WGs, mean cycles per phase: %.0f %.0f %.0f %.0f %.0f %.0f %.0f\n",
                used_rec ? "record-plane" : "fast", (size_t)nn, acc[0] / nn, acc[1] / nn, acc[2] / nn, acc[3] / nn, acc[4] / nn, acc[5] / nn, acc[6] / nn);
      }
      // the fallback count and the tie count in one round trip (pinned slots); the tie count is read
      // again below only when fallback items ran
      uint64_t* const rbh = ix.rb();
      rbh[1] = 0;
      HK_HIP(hipMemcpyAsync(rbh + 1, fbn, 4, hipMemcpyDeviceToHost, s));
      HK_HIP(hipMemcpyAsync(rbh, ix.ties_n.p, 8, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
      const unsigned int nfb = (unsigned int)rbh[1];
      ix.info[8] += nfb;   // items sorted by the LSD passes (a bin over BF_MAXBIN, or wide local keys)
      if (!nfb && !nw) return rbh[0];
      if (nfb) {
        if (pk) unpack_items(ix, *pk, keys, ix.bk_fb.as<uint2>(), nfb);
        k_bucket_sort<false, false, V><<<nfb, BS_T, 0, s>>>(
            lkeys, lvals, ix.bk_fb.as<uint2>(), pb, sb, lhb, symbias, d_inv, sa, bwt, ix.ties_k.as<uint64_t>(),
            ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(), nullptr);
      }
    }
    if (nw) {
      if (pk) unpack_items(ix, *pk, keys, ix.bk_items.as<uint2>() + nn, (uint32_t)nw);
      k_bucket_sort<true, false, V><<<grid_w, BS_T, 0, s>>>(
          lkeys, lvals, ix.bk_items.as<uint2>() + nn, pb, sb, lhb, symbias, d_inv, sa, bwt, ix.ties_k.as<uint64_t>(),
          ix.ties_v.as<V>(), ix.ties_n.as<unsigned long long>(), nullptr);
    }
    HK_HIP(hipGetLastError());
  }
  uint64_t* const h = ix.rb();
  HK_HIP(hipMemcpyAsync(h, ix.ties_n.p, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  return h[0];
}

template uint64_t sort_bucket_items<uint32_t>(Index&, const BucketPlan&, const uint64_t*, const uint32_t*, uint64_t,
                                              int, int, int, uint64_t, uint32_t*, uint8_t*, const PackedRecs*);
template uint64_t sort_bucket_items<uint64_t>(Index&, const BucketPlan&, const uint64_t*, const uint32_t*, uint64_t,
                                              int, int, int, uint64_t, uint64_t*, uint8_t*, const PackedRecs*);

}  // namespace hk
