// hk_shard.hip — suffix-array construction sharded over the GPUs of one node.
//
// Every rank holds the same T' (≤ 288 GB HBM each makes replication cheap) and owns one
// contiguous range of the FINAL suffix array.  Two partition schemes, chosen from the alphabet
// (identically on every rank):
//
// Keyed coarse scheme (whole-symbol keyed radix 2^lb: DNA, binary, 16 or 256 symbols):
//   1. each rank counts, exactly, the coarse bucket (the top 16 bits of the keyed sym field = the
//      first 16 / lb symbols) of every suffix of its block; ONE RCCL all-reduce of the 65536 counts
//      gives every rank the exact global histogram, hence identical splitters C_r and exact slice
//      bounds (no second counting pass);
//   2. each rank builds its slice with the single-GPU pipeline fused with the selection
//      (hk_bucket.hip §1c): a pre-pass over T' counts the slice's bins, pass A scans T', keeps the
//      slice's suffixes and scatters packed records by digit, then pass B, the LDS bucket sorts and
//      the tie refinement.
// Partition-key scheme (any other alphabet):
//   1. each rank histograms the 14-bit radix-(sigma+1) key prefix of every 64th position of its
//      block; an RCCL all-reduce gives the sampled global histogram and the splitter buckets;
//   2. each rank counts, over its block, the suffixes below every splitter (a register-only byte
//      pre-test against the splitters' prefix images); a second all-reduce of N+1 counts gives
//      the exact slice bounds [lo, hi) of every rank;
//   3. each rank scans all of T' and keeps the suffixes whose bucket it owns (count + scan +
//      write, reading T' twice, writing only its ~n/N pairs);
//   4. it sorts its slice by the q-symbol key and refines tied groups by sorting on
//      (dense group ordinal, next symbols of the suffix) read straight from the replicated text.
// Both: an RCCL all-gather of per-rank status records checks that the slices tile [0, n); groups
// still tied after the chunk rounds finish by prefix doubling with an ISA rank exchange.
// Positions are 64-bit when n ≥ 2^32 (the 4 GiB + 1 config).

#include <rccl/rccl.h>

#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <string>
#include <type_traits>

#include "hk_index.hpp"
#include "hk_keys.hpp"

namespace hk {
namespace {

constexpr int SH_BUCKET_BITS = 14;
constexpr int SH_BUCKETS = 1 << SH_BUCKET_BITS;
constexpr int SH_KBUCKETS = 65536;   // keyed coarse scheme: the top 16 sym bits (hkcsa_shard_buckets())
constexpr int PS_TILE = 4096;
constexpr int SH_SAMPLE = 64;   // histogram sample stride (splitters need balance, not exact counts)

struct ShardComm {  // one RCCL communicator per process (one process per GPU)
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = -1;
  uint8_t id[128];
};

// bucket of a key: its top SH_BUCKET_BITS bits (key >> bsh) under partition_geometry (pb = 0, so
// bucket in [blo, bhi) <=> the q-symbol prefix value lies in [Mlo, Mhi), see sel_geom).
struct BucketGeom {
  uint64_t R, Rck, Rlast;
  int q, pb, ck, bsh;
};

__device__ __forceinline__ uint64_t key_global(const uint8_t* __restrict__ t, uint64_t n, const uint16_t* L,
                                               uint64_t p, uint64_t R, int q, int pb) {
  uint64_t key = 0;
  for (int j = 0; j < q; ++j) key = key * R + (p + j < n ? L[t[p + j]] : 0u);
  return (key << pb) | (pb ? L[t[p == 0 ? n - 1 : p - 1]] : 0u);
}

// sampled histogram: positions p in [lo, hi) with p % SH_SAMPLE == 0
__global__ __launch_bounds__(256) void k_shard_hist(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                    uint64_t hi, const uint16_t* __restrict__ lut, BucketGeom g,
                                                    unsigned long long* __restrict__ hist) {
  __shared__ uint32_t H[SH_BUCKETS];
  __shared__ uint16_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256) H[i] = 0;
  __syncthreads();
  const uint64_t j0 = (lo + SH_SAMPLE - 1) / SH_SAMPLE, j1 = (hi + SH_SAMPLE - 1) / SH_SAMPLE;
  for (uint64_t j = j0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; j < j1; j += (uint64_t)gridDim.x * 256) {
    // the first 32 symbols from two 16-byte loads (p is a multiple of 16; T' has 64 pad bytes)
    const uint64_t p = j * SH_SAMPLE;
    const uint4 a = *reinterpret_cast<const uint4*>(t + p);
    const uint4 b = *reinterpret_cast<const uint4*>(t + p + 16);
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint64_t key = 0;
#pragma unroll
    for (int i = 0; i < 32; ++i)
      if (i < g.q) key = key * g.R + (p + i < n ? L[(w[i >> 2] >> (8 * (i & 3))) & 255u] : 0u);
    for (int i = 32; i < g.q; ++i) key = key * g.R + (p + i < n ? L[t[p + i]] : 0u);
    atomicAdd(&H[key >> g.bsh], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256)
    if (H[i]) atomicAdd(&hist[i], (unsigned long long)H[i]);
}

// Exact slice sizes: below[r] += #{p in [lo, hi) : bucket(p) < B_r} for the splitters.  Same
// byte pre-test as the selection (see below): with A_r = floor(M_r / W) the prefix holding the
// splitter, P < A_r is below, P > A_r is not, P == A_r (or a window past the end) takes the
// full key.  Thresholds are byte images: "below" <=> window <= ID_r.
struct BelowImg {
  uint64_t ID, IA;
  uint32_t flags;   // 1: some prefix is below (ID valid), 2: IA valid
  uint32_t B;       // splitter bucket
};
constexpr int SH_MAX_RANKS = 64;

__global__ __launch_bounds__(256) void k_shard_below(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                     uint64_t hi, const uint16_t* __restrict__ lut, BucketGeom g,
                                                     int h, uint64_t topmask, int nopre,
                                                     const BelowImg* __restrict__ img, int nthr,
                                                     unsigned long long* __restrict__ below) {
  __shared__ uint16_t L[256];
  __shared__ BelowImg I[SH_MAX_RANKS];
  __shared__ uint32_t cnt[SH_MAX_RANKS];
  L[threadIdx.x] = lut[threadIdx.x];
  if ((int)threadIdx.x < nthr) {
    I[threadIdx.x] = img[threadIdx.x];
    cnt[threadIdx.x] = 0;
  }
  __syncthreads();
  const uint64_t g0 = lo / 16, g1 = (hi + 15) / 16;
  for (uint64_t gi = g0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; gi < g1; gi += (uint64_t)gridDim.x * 256) {
    const uint64_t p0 = gi * 16;
    uint32_t valid = 0xFFFFu;
    if (p0 < lo) valid &= 0xFFFFu << (lo - p0);
    if (p0 + 16 > hi) valid &= (1u << (hi - p0)) - 1u;
    const uint4 a = *reinterpret_cast<const uint4*>(t + p0);
    const uint4 b = *reinterpret_cast<const uint4*>(t + p0 + 16);
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
    uint64_t be[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int j = k >> 2, sh = k & 3;
      const uint32_t d0 = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
      const uint32_t d1 = __builtin_amdgcn_alignbyte(w[j + 2], w[j + 1], sh);
      be[k] = (((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1)) & topmask;
    }
    uint32_t amb = 0;
    if (nopre) amb = valid;
    else if (p0 + 16 + h > n) {
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (p0 + k + h > n) amb |= 1u << k;
      amb &= valid;
    }
    for (int r = 0; r < nthr; ++r) {   // a position equal to any splitter prefix takes the full key
      const BelowImg im = I[r];
      if (!(im.flags & 2u)) continue;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (be[k] == im.IA) amb |= 1u << k;
    }
    amb &= valid;
    for (int r = 0; r < nthr; ++r) {
      const BelowImg im = I[r];
      if (!(im.flags & 1u)) continue;
      uint32_t bl = 0;
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (be[k] <= im.ID) bl |= 1u << k;
      bl &= valid & ~amb;
      if (bl) atomicAdd(&cnt[r], (uint32_t)__popc(bl));
    }
    while (amb) {   // rare: splitter prefixes and the last h positions
      const int k = __ffs(amb) - 1;
      amb &= amb - 1;
      const uint32_t bk = (uint32_t)(key_global(t, n, L, p0 + k, g.R, g.q, g.pb) >> g.bsh);
      for (int r = 0; r < nthr; ++r)
        if (bk < I[r].B) atomicAdd(&cnt[r], 1u);
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < nthr && cnt[threadIdx.x]) atomicAdd(&below[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// Every rank scans all of T' and keeps the suffixes whose bucket lies in [blo, bhi).
//
// Pre-test on raw bytes (no LDS, no code lookup): the first h symbols of a suffix, as a radix-R
// prefix P, bound its key to [P·W, (P+1)·W), W = R^(q-h); with A / B the prefixes holding the
// range ends, P in (A, B) is inside the rank's range, P outside [A, B] is not, and P == A or B
// needs the full key.  The code map is strictly increasing, so comparing prefixes equals
// comparing the h raw bytes big-endian against byte images of the thresholds (SelGeom, host):
// each thread holds 32 text bytes in registers and tests its 16 consecutive positions with a
// few shifts, byte swaps and 64-bit compares.  Positions whose h bytes run past T' take the
// full-key path too.
//
// Block b owns the contiguous tiles [b*tpb, (b+1)*tpb): a count pass (registers only, one
// reduction per block), an exclusive scan of the block counts, and a write pass that stages the
// tile's codes in LDS, lists the selected offsets in LDS and builds their keys densely, so the
// key / position stores are coalesced and no global atomics are needed.
struct SelGeom {
  uint64_t TL, TH, TA, TB, topmask;
  int h;
  uint32_t flags;
};
constexpr uint32_t SEL_NOPRE = 1, SEL_EMPTY = 2, SEL_HAS_A = 4, SEL_HAS_B = 8;


// selection bits of the 16 positions p0 .. p0+15 (bit k: p0 + k) from their 32 text bytes a, b
__device__ __forceinline__ uint32_t select16w(const uint4& a, const uint4& b, const uint8_t* __restrict__ t,
                                              uint64_t n, uint64_t p0, const uint16_t* L, const BucketGeom& g,
                                              const SelGeom& sg, uint32_t blo, uint32_t bhi) {
  if (p0 >= n) return 0;
  const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
  // Branch-free per position (short-circuit && / || on per-lane values compiled to exec-mask
  // juggling that made this loop scalar-ALU bound): in range <=> be - TL <= TH - TL (unsigned);
  // an absent TA / TB is replaced by one that is present or by ~0, which at worst sends an
  // all-0xFF window down the exact path.
  const uint64_t span = sg.TH - sg.TL;
  const uint64_t TB = (sg.flags & SEL_HAS_B) ? sg.TB : ~0ull;
  const uint64_t TA = (sg.flags & SEL_HAS_A) ? sg.TA : TB;
  uint32_t acc = 0, amb = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int j = k >> 2, sh = k & 3;
    const uint32_t d0 = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
    const uint32_t d1 = __builtin_amdgcn_alignbyte(w[j + 2], w[j + 1], sh);
    const uint64_t be = (((uint64_t)__builtin_bswap32(d0) << 32) | __builtin_bswap32(d1)) & sg.topmask;
    acc |= (be - sg.TL <= span) ? (1u << k) : 0u;
    amb |= ((be == TA) | (be == TB)) ? (1u << k) : 0u;
  }
  if (sg.flags & SEL_EMPTY) acc = 0;
  if (sg.flags & SEL_NOPRE) amb = 0xFFFFu;
  if (p0 + 16 + sg.h > n) {   // windows running past T': the exact path
#pragma unroll
    for (int k = 0; k < 16; ++k) amb |= (p0 + k + sg.h > n) ? (1u << k) : 0u;
  }
  amb &= (p0 + 16 <= n) ? 0xFFFFu : ((1u << (n - p0)) - 1u);
  acc &= ~amb;
  while (amb) {   // rare: boundary prefixes and the last h positions
    const int k = __ffs(amb) - 1;
    amb &= amb - 1;
    const uint32_t bk = (uint32_t)(key_global(t, n, L, p0 + k, g.R, g.q, g.pb) >> g.bsh);
    if (bk >= blo && bk < bhi) acc |= 1u << k;
  }
  if (p0 + 16 > n) acc &= (1u << (n - p0)) - 1u;
  return acc;
}


__global__ __launch_bounds__(256) void k_select_count(const uint8_t* __restrict__ t, uint64_t n, uint64_t tpb,
                                                      const uint16_t* __restrict__ lut, BucketGeom g, SelGeom sg,
                                                      uint32_t blo, uint32_t bhi, uint64_t* __restrict__ block_cnt,
                                                      uint16_t* __restrict__ masks) {
  __shared__ uint16_t L[256];
  __shared__ uint64_t red[4];
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const uint64_t tiles = (n + PS_TILE - 1) / PS_TILE;
  const uint64_t t0 = (uint64_t)blockIdx.x * tpb;
  const uint64_t t1 = t0 + tpb < tiles ? t0 + tpb : tiles;
  uint64_t cnt = 0;
  // four tiles per round: their eight 16-byte loads are in flight together
  constexpr int U = 4;
  for (uint64_t ti = t0; ti < t1; ti += U) {
    uint4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t p0 = (ti + u) * PS_TILE + 16 * threadIdx.x;
      if (ti + u < t1 && p0 < n) {
        a[u] = *reinterpret_cast<const uint4*>(t + p0);
        b[u] = *reinterpret_cast<const uint4*>(t + p0 + 16);
      } else {
        a[u] = b[u] = make_uint4(0, 0, 0, 0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (ti + u >= t1) break;
      const uint32_t sel = select16w(a[u], b[u], t, n, (ti + u) * PS_TILE + 16 * threadIdx.x, L, g, sg, blo, bhi);
      masks[(ti + u) * 256 + threadIdx.x] = (uint16_t)sel;   // the write pass reads these instead of re-testing
      cnt += __popc(sel);
    }
  }
  cnt = wave_sum(cnt);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = cnt;
  __syncthreads();
  if (threadIdx.x == 0) block_cnt[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// Keys of the selected suffixes in the keyed layout of the single-GPU bucket build (see
// key_geometry_keyed): [bin][sym][dense code of T'[p-1], pb bits][position bits 32.., hb bits],
// the bin field only for multiplicative bins.  With hb > 0 (V = u32) the low 32 position bits go
// to vals and the high bits sit below the key, outside the sorted bit range; k_split_join
// reassembles them.  Keys come from the tile's keyed codes staged in LDS (measured faster than
// building each selected key from global text words, even at 1/8 selection density).
// kmm[0..1] collect the exact min / max sym (checked against the slice bounds), hist0 the
// histogram of the bins' low byte (the first LSD pass).
// MODE 0 (dense slices): the tile is staged as keyed codes.  MODE 1 (sparse slices): staged as raw
// text words, only the selected suffixes' bytes go through the code table.  MODE 2 (sparse, keyed
// radix 2^lb with lb | 32): raw words, then one pass packs the tile's codes MSB-first into lb-bit
// fields and every key is a q*lb-bit window of that stream (three LDS words, no per-symbol loop).
template <typename V, int MODE, int LB = 0>
__global__ __launch_bounds__(256) void k_select_write(const uint8_t* __restrict__ t, uint64_t n, uint64_t tpb,
                                                      const uint16_t* __restrict__ masks,
                                                      const uint16_t* __restrict__ lutk,
                                                      const uint16_t* __restrict__ lutp,
                                                      const uint16_t* __restrict__ k2d,
                                                      const uint64_t* __restrict__ skey, KeyedArgs ka,
                                                      const uint64_t* __restrict__ block_off,
                                                      uint64_t* __restrict__ keys, V* __restrict__ vals, int hb,
                                                      SliceBins sbn, unsigned long long* __restrict__ kmm,
                                                      unsigned long long* __restrict__ hist0) {
  constexpr bool RAW = MODE >= 1;
  // raw words: bytes [base - 4, base + PS_TILE + 108), enough for the last packed word at lb = 1
  constexpr int NW = (PS_TILE + 112) / 4;
  constexpr int NSYM = PS_TILE + 68;           // packed symbols: positions base - 1 .. base + PS_TILE + 66
  constexpr int NPK = NSYM / 4 + 4;            // packed words for lb <= 8
  __shared__ uint16_t c[RAW ? 1 : PS_TILE + kCodePad];
  __shared__ uint32_t W[RAW ? NW : 1];
  __shared__ uint32_t PK[MODE == 2 ? NPK : 1];
  __shared__ uint16_t K2D[MODE == 2 ? 256 : 1];
  __shared__ uint16_t list[PS_TILE];
  __shared__ uint16_t LK[256], LP[256];
  __shared__ uint64_t SK[64];
  __shared__ uint32_t red[4];
  __shared__ uint32_t H0[256];
  LK[threadIdx.x] = lutk[threadIdx.x];
  LP[threadIdx.x] = lutp[threadIdx.x];
  H0[threadIdx.x] = 0;
  if (MODE == 2) K2D[threadIdx.x] = k2d[threadIdx.x];
  if (threadIdx.x < 64 && ka.s_start + threadIdx.x < n) SK[threadIdx.x] = skey[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int pbe = ka.pb + hb;
  const int lb = LB ? LB : ka.lb, per = MODE == 2 ? 32 / lb : 1, kbits = ka.q * lb;
  const uint64_t tiles = (n + PS_TILE - 1) / PS_TILE;
  const uint64_t t0 = (uint64_t)blockIdx.x * tpb;
  const uint64_t t1 = t0 + tpb < tiles ? t0 + tpb : tiles;
  uint64_t run = block_off[blockIdx.x];
  uint64_t kmin = ~0ull, kmax = 0;
  // software pipelining: the next tile's mask and text words are loaded while this tile is built
  constexpr int RPER = (NW + 255) / 256;
  uint32_t nsel = 0, pw[RPER];
  TextWords<PS_TILE, 256> tw;
  auto prefetch = [&](uint64_t ti) {
    nsel = masks[ti * 256 + threadIdx.x];
    if (RAW) {
#pragma unroll
      for (int k = 0; k < RPER; ++k) {
        const int i = threadIdx.x + 256 * k;
        const int64_t a = (int64_t)(ti * PS_TILE) - 4 + 4 * i;
        pw[k] = (i < NW && a >= 0 && (uint64_t)a < n) ? *reinterpret_cast<const uint32_t*>(t + a) : 0u;
      }
    } else {
      load_text_words<PS_TILE, 256>(tw, t, n, ti * PS_TILE);
    }
  };
  if (t0 < t1) prefetch(t0);
  for (uint64_t ti = t0; ti < t1; ++ti) {
    const uint64_t base = ti * PS_TILE;
    uint32_t sel = nsel;
    uint32_t cw[RPER];
#pragma unroll
    for (int k = 0; k < RPER; ++k) cw[k] = pw[k];
    const TextWords<PS_TILE, 256> ctw = tw;
    if (ti + 1 < t1) prefetch(ti + 1);
    const uint32_t cnt = __popc(sel);
    const uint32_t inc = wave_incl_sum<uint32_t>(cnt);
    if (lane == 63) red[w] = inc;
    const uint32_t any = __syncthreads_or(sel != 0);
    if (!any) continue;   // block-uniform: nothing of this tile is ours
    uint32_t o = inc - cnt;
    uint32_t tot = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < w) o += red[i];
      tot += red[i];
    }
    while (sel) {
      const int k = __ffs(sel) - 1;
      sel &= sel - 1;
      list[o++] = (uint16_t)(16 * threadIdx.x + k);
    }
    if (RAW) {
#pragma unroll
      for (int k = 0; k < RPER; ++k)
        if (threadIdx.x + 256 * k < (unsigned)NW) W[threadIdx.x + 256 * k] = cw[k];
    } else {
      store_text_codes<PS_TILE, 256>(c, LK, ctw, n, base);
    }
    __syncthreads();
    if (MODE == 2) {
      // symbol s (position base - 1 + s) is byte s + 3 of W; word wd packs symbols [wd*per, +per)
      const uint8_t* WB = reinterpret_cast<const uint8_t*>(W);
      for (int wd = threadIdx.x; wd * per < NSYM; wd += 256) {
        uint32_t word = 0;
        if (LB) {   // compile-time lb: unrolled
          constexpr int PER = LB ? 32 / LB : 1;
#pragma unroll
          for (int u = 0; u < PER; ++u) word = (word << LB) | (LK[WB[wd * PER + u + 3]] & 255u);
        } else {
          for (int u = 0; u < per; ++u) word = (word << lb) | (LK[WB[wd * per + u + 3]] & 255u);
        }
        PK[wd] = word;
      }
      __syncthreads();
    }
    for (uint32_t i = threadIdx.x; i < tot; i += 256) {
      const int off = list[i];
      const uint64_t p = base + off;
      uint64_t sym;
      uint32_t pcode;   // dense code of T'[p-1]
      if (MODE == 2) {
        if (p >= ka.s_start) {
          sym = SK[p - ka.s_start];
        } else {
          const uint32_t bit = (uint32_t)(off + 1) * lb, w0 = bit >> 5, o = bit & 31u;
          const uint64_t hi = ((uint64_t)PK[w0] << 32) | PK[w0 + 1];
          const uint64_t win = o ? (hi << o) | (PK[w0 + 2] >> (32 - o)) : hi;
          sym = kbits >= 64 ? win : win >> (64 - kbits);
        }
        // T'[p-1] is a keyed byte except for p = 0 (the terminal before it)
        const uint32_t pbit = (uint32_t)off * lb;
        const uint32_t kc = (PK[pbit >> 5] >> (32 - lb - (pbit & 31u))) & ((1u << lb) - 1u);
        pcode = p == 0 ? LP[t[n - 1]] : K2D[kc];
      } else if (RAW) {
        sym = p >= ka.s_start ? SK[p - ka.s_start] : keyed_sym_words(W, (uint32_t)off + 4, ka, LK);
        pcode = LP[p == 0 ? t[n - 1] : (W[(off + 3) >> 2] >> (8 * ((off + 3) & 3))) & 255u];
      } else {
        sym = keyed_sym(c, off, p, ka, SK);
        pcode = LP[c[off] >> 8];
      }
      kmin = sym < kmin ? sym : kmin;
      kmax = sym > kmax ? sym : kmax;
      uint64_t key = (sym << pbe) | ((uint64_t)pcode << hb);
      if (hb) key |= p >> 32;
      if (sbn.D > 0) {
        const uint64_t x = sym - sbn.kmin;
        const uint32_t bin = sbn.mul ? (uint32_t)__umul64hi(x, sbn.mul) : (uint32_t)(x >> sbn.bsh);
        if (sbn.mul) key |= (uint64_t)bin << sbn.binpos;
        atomicAdd(&H0[bin & 255u], 1u);
      }
      keys[run + i] = key;
      vals[run + i] = (V)p;
    }
    run += tot;
    __syncthreads();   // list / staging / red are rewritten by the next tile
  }
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t a = __shfl_xor(kmin, d), b = __shfl_xor(kmax, d);
    kmin = a < kmin ? a : kmin;
    kmax = b > kmax ? b : kmax;
  }
  if (lane == 0 && kmin <= kmax) {
    atomicMin(&kmm[0], (unsigned long long)kmin);
    atomicMax(&kmm[1], (unsigned long long)kmax);
  }
  __syncthreads();
  if (H0[threadIdx.x]) atomicAdd(&hist0[threadIdx.x], (unsigned long long)H0[threadIdx.x]);
}

__global__ __launch_bounds__(256) void k_split_join(uint64_t* __restrict__ keys, const uint32_t* __restrict__ lo32,
                                                    uint64_t m, int hb, uint64_t* __restrict__ sa) {
  const uint64_t mask = (1ull << hb) - 1;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256) {
    const uint64_t k = keys[i];
    sa[i] = ((k & mask) << 32) | lo32[i];
    keys[i] = k >> hb;
  }
}

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

void ncclcheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw ApiError{-8, std::string(what) + ": " + ncclGetErrorString(r)};
}

// Partition geometry: the prefix key of the splitters.  No prev field (pb = 0: a bucket has to be
// a range of the suffix order, which a prev field below a short key would split) and as many
// symbols as fit in 64 bits, so the top SH_BUCKET_BITS bits split the prefixes as finely as
// possible.  oracle/hkcsa_oracle.c partition_geometry restates it.
KeyGeom partition_geometry(Index& ix) {
  KeyGeom g = key_geometry(ix, false);
  g.pb = 0;
  g.q = 1;
  while (g.q < 64 && mixed_radix_bits(g.R, g.q + 1) <= 64) ++g.q;
  g.sym_bits = mixed_radix_bits(g.R, g.q);
  g.key_bits = g.sym_bits;
  return g;
}

int bucket_shift(const KeyGeom& kg) {
  const int sh = kg.key_bits - SH_BUCKET_BITS;
  return sh < 0 ? 0 : sh;
}

BucketGeom bucket_geom(const KeyGeom& kg) {
  const KeyChunks kc = key_chunks(kg.R, kg.q);
  return BucketGeom{kg.R, kc.Rck, kc.Rlast, kg.q, kg.pb, kc.ck, bucket_shift(kg)};
}

// Byte images of h-symbol prefixes.  Prefixes of in-text positions have digits 1..R-1 only
// (0 = past the end), and digit d is byte inv[d], increasing in d — so comparing zero-free
// prefixes equals comparing their h raw bytes big-endian.
struct PrefixImages {
  const KeyGeom& kg;
  uint64_t R = 2, Rh = 2;
  int h = 0;
  bool usable = false;      // false: every position takes the full key
  unsigned __int128 W = 1;  // R^(q-h)
  uint64_t topmask = 0;

  PrefixImages(const KeyGeom& k, const BucketGeom& g) : kg(k), R(k.R) {
    h = 1;
    Rh = R;
    while (Rh < (1ull << 16) && h < 8) {
      Rh *= R;
      ++h;
    }
    usable = g.bsh >= g.pb && kg.q > h;
    for (int i = h; i < kg.q; ++i) W *= R;
    topmask = ~0ull << (8 * (8 - h));
  }
  void digits(uint64_t P, int* d) const {
    for (int i = h - 1; i >= 0; --i) { d[i] = (int)(P % R); P /= R; }
  }
  bool zero_free(uint64_t P) const {
    int d[8];
    digits(P, d);
    for (int i = 0; i < h; ++i) if (!d[i]) return false;
    return true;
  }
  uint64_t image(uint64_t P) const {   // big-endian byte image, top-aligned in 64 bits
    int d[8];
    digits(P, d);
    uint64_t v = 0;
    for (int i = 0; i < h; ++i) v = (v << 8) | kg.inv[d[i]];
    return v << (8 * (8 - h));
  }
  uint64_t up0(uint64_t P) const {     // smallest zero-free value >= P (Rh when none)
    while (P < Rh && !zero_free(P)) {
      int d[8];
      digits(P, d);
      int i = 0;
      while (d[i]) ++i;
      for (int k = i; k < h; ++k) d[k] = 1;
      uint64_t v = 0;
      for (int k = 0; k < h; ++k) v = v * R + (uint64_t)d[k];
      P = v;
    }
    return P;
  }
  int64_t down0(int64_t P) const {     // largest zero-free value <= P (-1 when none)
    while (P >= 0 && !zero_free((uint64_t)P)) {
      int d[8];
      digits((uint64_t)P, d);
      int i = 0;
      while (d[i]) ++i;
      uint64_t pre = 0;
      for (int k = 0; k < i; ++k) pre = pre * R + (uint64_t)d[k];
      uint64_t scale = 1;
      for (int k = i; k < h; ++k) scale *= R;
      P = (int64_t)(pre * scale) - 1;
    }
    return P;
  }
  // the prefix holding mixed value M (clamped to Rh)
  uint64_t prefix_of(unsigned __int128 M) const {
    const unsigned __int128 A = M / W;
    return A < Rh ? (uint64_t)A : Rh;
  }
  unsigned __int128 mixed_of_bucket(uint64_t B, int bsh, int pb) const {
    return ((unsigned __int128)B << bsh) >> pb;
  }
};

// Selection of buckets [blo, bhi): accept iff TL <= window <= TH, full key on TA / TB.
SelGeom sel_geom(const KeyGeom& kg, const BucketGeom& g, uint32_t blo, uint32_t bhi) {
  SelGeom sg{};
  const PrefixImages pi(kg, g);
  if (!pi.usable || bhi <= blo) {
    sg.flags = SEL_NOPRE;
    return sg;
  }
  const uint64_t a = pi.prefix_of(pi.mixed_of_bucket(blo, g.bsh, g.pb));
  const uint64_t bb = pi.prefix_of(pi.mixed_of_bucket(bhi, g.bsh, g.pb) - 1);
  sg.h = pi.h;
  sg.topmask = pi.topmask;
  const uint64_t lo = pi.up0(a < pi.Rh ? a + 1 : pi.Rh);
  const int64_t hi = pi.down0((int64_t)(bb < pi.Rh ? bb : pi.Rh) - 1);
  if (lo >= pi.Rh || hi < 0 || (int64_t)lo > hi) {
    sg.flags |= SEL_EMPTY;
  } else {
    sg.TL = pi.image(lo);
    sg.TH = pi.image((uint64_t)hi);
  }
  if (a < pi.Rh && pi.zero_free(a)) { sg.flags |= SEL_HAS_A; sg.TA = pi.image(a); }
  if (bb < pi.Rh && pi.zero_free(bb)) { sg.flags |= SEL_HAS_B; sg.TB = pi.image(bb); }
  return sg;
}

// "bucket < B": P < A below, P == A full key, else not below (A = prefix holding B's first key)
BelowImg below_img(const PrefixImages& pi, const BucketGeom& g, uint32_t B) {
  BelowImg im{};
  im.B = B;
  if (!pi.usable) return im;
  const uint64_t a = pi.prefix_of(pi.mixed_of_bucket(B, g.bsh, g.pb));
  const int64_t d = pi.down0((int64_t)a - 1);
  if (d >= 0) {
    im.flags |= 1u;
    im.ID = pi.image((uint64_t)d);
  }
  if (a < pi.Rh && pi.zero_free(a)) {
    im.flags |= 2u;
    im.IA = pi.image(a);
  }
  return im;
}

// splitter buckets B_0 = 0 < ... < B_N = nb from a global histogram of nb bins: B_r = the smallest B
// with cum[B] >= floor(total * r / N).  aligned (keyed scheme): when N divides nb and the equal-width
// splitters B_r = r * nb / N leave no slice 2 % above total / N, those are taken instead (iid text: a
// slice of exactly 2^k coarse buckets gets 2^17 bins, where a balanced 2^k + 1 would get half as many).
// hkcsa/shard.py split_buckets restates this rule.
std::vector<uint32_t> splitters(const uint64_t* ghist, int nranks, int nb = SH_BUCKETS, bool aligned = false) {
  std::vector<uint64_t> cum(nb + 1, 0);
  for (int i = 0; i < nb; ++i) cum[i + 1] = cum[i] + ghist[i];
  const uint64_t tot = cum[nb];
  std::vector<uint32_t> B(nranks + 1);
  if (aligned && nb % nranks == 0) {
    bool ok = true;
    const uint64_t cap = tot / (uint64_t)nranks + tot / (uint64_t)nranks / 50;
    for (int r = 0; r < nranks && ok; ++r)
      ok = cum[(uint64_t)nb * (r + 1) / nranks] - cum[(uint64_t)nb * r / nranks] <= cap;
    if (ok) {
      for (int r = 0; r <= nranks; ++r) B[r] = (uint32_t)((uint64_t)nb * r / nranks);
      return B;
    }
  }
  for (int r = 0; r <= nranks; ++r) {
    if (r == 0) { B[r] = 0; continue; }
    if (r == nranks) { B[r] = (uint32_t)nb; continue; }
    const uint64_t target = (uint64_t)((__uint128_t)tot * (uint64_t)r / (uint64_t)nranks);
    uint32_t lo = 0, hi = (uint32_t)nb;
    while (lo < hi) {  // smallest B with cum[B] >= target
      const uint32_t mid = (lo + hi) / 2;
      if (cum[mid] >= target) hi = mid; else lo = mid + 1;
    }
    B[r] = lo;
  }
  return B;
}

// rank r's block of T' for the per-rank histograms: 16-aligned starts (the last block ends at n)
std::pair<uint64_t, uint64_t> block_of(uint64_t n, int nranks, int rank) {
  const uint64_t b0 = rank ? ((uint64_t)((__uint128_t)n * (uint64_t)rank / (uint64_t)nranks) & ~15ull) : 0;
  const uint64_t b1 =
      rank + 1 < nranks ? ((uint64_t)((__uint128_t)n * (uint64_t)(rank + 1) / (uint64_t)nranks) & ~15ull) : n;
  return {b0, b1};
}

// Bounds of the keyed sym fields of the suffixes whose partition bucket lies in [blo, bhi), from
// the partition keys alone.  A partition key spells a string: digit d >= 1 is byte inv[d], digit 0
// ends it.  Every suffix of the range is >= the string of the range's first key and <= that of its
// last.  Digit of byte b in keyed radix: kdig[b] (the keyed bytes below b; its keyed code when b is
// keyed); the string stops after a non-keyed byte (the unique terminal: a short suffix, whose
// boundary key is exactly that prefix followed by zeros) or at its end.  The lower bound fills the
// remaining digits with 0, the upper bound with Rk - 1; both are monotone in the string, so the
// slice's sym fields lie in [lo, hi].
std::pair<uint64_t, uint64_t> slice_sym_bounds(const KeyGeom& pg, int bsh_p, uint32_t blo, uint32_t bhi,
                                               const KeyGeom& kk) {
  unsigned __int128 Rq = 1;
  for (int i = 0; i < pg.q; ++i) Rq *= pg.R;
  auto bound = [&](unsigned __int128 pkey, bool upper) -> uint64_t {
    if (pkey > Rq - 1) pkey = Rq - 1;   // the last bucket's top key may lie past R^q - 1
    std::vector<int> d(pg.q);
    for (int i = pg.q - 1; i >= 0; --i) {
      d[i] = (int)(pkey % pg.R);
      pkey /= pg.R;
    }
    unsigned __int128 v = 0;
    int i = 0;
    while (i < kk.q && i < pg.q && d[i] != 0) {
      const uint8_t b = pg.inv[d[i]];
      v = v * kk.Rk + kk.kdig[b];
      ++i;
      if (!kk.kflag[b]) break;
    }
    for (; i < kk.q; ++i) v = v * kk.Rk + (upper ? kk.Rk - 1 : 0);
    const unsigned __int128 mx = kk.sym_bits >= 64 ? ~(uint64_t)0 : ((((unsigned __int128)1) << kk.sym_bits) - 1);
    return (uint64_t)(v < mx ? v : mx);
  };
  const uint64_t lo = bound((unsigned __int128)blo << bsh_p, false);
  const uint64_t hi = bound((((unsigned __int128)bhi) << bsh_p) - 1, true);
  return {lo, hi};
}

template <typename V>
void shard_build_t(Index& ix, const uint64_t* ghist, const uint64_t* gbelow, int nranks, int rank) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  const KeyGeom kg = partition_geometry(ix);   // selection geometry (same as phases 1-2)
  // splitters: rank r owns buckets [B[r], B[r+1]); its SA slice is [below(B[r]), below(B[r+1]))
  const std::vector<uint32_t> B = splitters(ghist, nranks);
  if (gbelow[0] != 0 || gbelow[nranks] != n) throw ApiError{-7, "global splitter counts do not cover n"};
  for (int r = 0; r < nranks; ++r)
    if (gbelow[r] > gbelow[r + 1]) throw ApiError{-7, "global splitter counts are not monotone"};
  const uint32_t blo = B[rank], bhi = B[rank + 1];
  ix.shard_lo = gbelow[rank];
  ix.shard_hi = gbelow[rank + 1];
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  ix.info.assign(9, 0);
  ix.dbl = Index::DblState{};
  ix.sharded = true;
  ix.sa_pos64 = sizeof(V) == 8;
  ix.have_sa = ix.have_bwt = ix.have_wt = false;
  ix.sa.ensure(m * sizeof(V) + 16);
  ix.bwt.ensure(m + 64);
  if (!m) {
    ix.have_sa = ix.have_bwt = true;
    return;
  }
  // 64-bit positions: sort u32 low halves with the high bits parked below the key (20 instead of
  // 24 bytes per pair and pass); NO_SPLIT sorts whole u64 values on the global path
  const bool whole = sizeof(V) == 8 && (ix.flags & kFlagNoSplit);
  int hb = 0;
  if (sizeof(V) == 8 && !whole) {
    hb = 1;
    while (((n - 1) >> 32) >> hb) ++hb;
  }
  // sort geometry: the keyed layout of the single-GPU bucket build, hb bits reserved
  const KeyGeom kk = key_geometry_keyed(ix, hb);
  ix.info[3] = (uint64_t)kk.q;
  upload_geometry(ix, kk);
  const uint8_t* small = ix.small.as<uint8_t>();
  const KeyChunks kch = key_chunks(kk.Rk, kk.q);
  KeyedArgs ka{kk.Rk, kch.Rck, kch.Rlast, kk.s_start, kk.q, kch.ck, kk.pb, 0};
  {
    // keyed radix 2^lb with whole codes per 32-bit word and the sym field exactly q*lb bits:
    // keys are bit windows of a packed code stream (k_select_write MODE 2)
    const int lb = (kk.Rk & (kk.Rk - 1)) == 0 ? __builtin_ctzll(kk.Rk) : 0;
    if (lb && 32 % lb == 0 && kk.sym_bits == lb * kk.q) ka.lb = lb;
  }
  const BucketGeom bg = bucket_geom(kg);
  // bucket bins of the slice from its sym bounds (known before any key is built)
  const auto kb = slice_sym_bounds(kg, bg.bsh, blo, bhi, kk);
  const bool global = whole || (ix.flags & kFlagGlobalSort);
  SliceBins sbn = global ? SliceBins{} : slice_bins(m, kk, hb, kb.first, kb.second, ix.flags & kFlagMulBins);
  uint64_t got = 0;
  uint64_t kmm[2] = {~0ull, 0};
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(m * 8 + 16);
    ix.vals[i].ensure(m * sizeof(V) + 16);
  }
  uint64_t* d_h0 = reinterpret_cast<uint64_t*>(ix.small.as<uint8_t>() + 5120);
  HK_HIP(hipMemsetAsync(d_h0, 0, 256 * 8, s));
  {
    const uint64_t tiles = ceil_div(n, (uint64_t)PS_TILE);
    const uint64_t G = tiles < 8192 ? tiles : 8192;
    const uint64_t tpb = ceil_div(tiles, G);
    const unsigned grid = (unsigned)ceil_div(tiles, tpb);
    ix.tile_d.ensure((grid + 1) * 8 + 16);
    ix.sel.ensure(tiles * 256 * 2 + 16);   // selection masks, one u16 per 16 positions
    uint64_t* bc = ix.tile_d.as<uint64_t>();
    unsigned long long* d_kmm = reinterpret_cast<unsigned long long*>(bc + grid + 1);
    HK_HIP(hipMemcpyAsync(d_kmm, kmm, 16, hipMemcpyHostToDevice, s));
    const uint16_t* lut = reinterpret_cast<const uint16_t*>(small + 2048);
    const uint16_t* lutk = reinterpret_cast<const uint16_t*>(small + 2560);
    const uint16_t* lutp = reinterpret_cast<const uint16_t*>(small + 4608);
    const uint64_t* skey = reinterpret_cast<const uint64_t*>(small + 3584);
    const SelGeom sg = sel_geom(kg, bg, blo, bhi);
    {
      TimedLaunch t(ix.timer, "shard_select_count", (double)n);
      k_select_count<<<grid, 256, 0, s>>>(ix.text.as<uint8_t>(), n, tpb, lut, bg, sg, blo, bhi, bc,
                                          ix.sel.as<uint16_t>());
      HK_HIP(hipGetLastError());
    }
    scan_exclusive_u64(ix.sw, bc, bc, grid, true, s);
    {
      TimedLaunch t(ix.timer, "shard_pack_select", (double)n + (double)m * (8 + sizeof(V)));
      unsigned long long* h0 = reinterpret_cast<unsigned long long*>(d_h0);
      // sparse slices stage raw words (only the selected suffixes' bytes are converted), packed
      // lb-bit codes when the keyed radix is 2^lb with lb | 32
      const bool sparse = m * 3 < n;
      const int mode = ka.lb ? 2 : (sparse ? 1 : 0);
      const uint16_t* mk = ix.sel.as<uint16_t>();
      const uint16_t* k2d = reinterpret_cast<const uint16_t*>(small + 7456);
      uint64_t* k0 = ix.keys[0].as<uint64_t>();
      auto launch = [&](auto vtag, auto modetag, void* v) {
        using VT = decltype(vtag);
        constexpr int MD = decltype(modetag)::value;
        if (MD == 2 && ka.lb == 2)   // DNA: the packing loop unrolled
          k_select_write<VT, MD, 2><<<grid, 256, 0, s>>>(
              ix.text.as<uint8_t>(), n, tpb, mk, lutk, lutp, k2d, skey, ka, bc, k0, reinterpret_cast<VT*>(v), hb,
              sbn, d_kmm, h0);
        else
          k_select_write<VT, MD><<<grid, 256, 0, s>>>(
              ix.text.as<uint8_t>(), n, tpb, mk, lutk, lutp, k2d, skey, ka, bc, k0, reinterpret_cast<VT*>(v), hb,
              sbn, d_kmm, h0);
      };
      using M0 = std::integral_constant<int, 0>;
      using M1 = std::integral_constant<int, 1>;
      using M2 = std::integral_constant<int, 2>;
      void* v0 = ix.vals[0].p;
      if (hb) {
        if (mode == 2) launch(uint32_t{}, M2{}, v0);
        else if (mode == 1) launch(uint32_t{}, M1{}, v0);
        else launch(uint32_t{}, M0{}, v0);
      } else {
        if (mode == 2) launch(V{}, M2{}, v0);
        else if (mode == 1) launch(V{}, M1{}, v0);
        else launch(V{}, M0{}, v0);
      }
      HK_HIP(hipGetLastError());
    }
    HK_HIP(hipMemcpyAsync(&got, bc + grid, 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipMemcpyAsync(kmm, d_kmm, 16, hipMemcpyDeviceToHost, s));
  }
  HK_HIP(hipStreamSynchronize(s));
  if (got != m) throw ApiError{-7, "shard selection count mismatch"};
  if (kmm[0] > kmm[1]) throw ApiError{-7, "shard selection produced no keys"};
  static const bool dbg = getenv("HKCSA_SHARD_DEBUG") != nullptr;   // diagnostic: slice geometry
  if (dbg)
    fprintf(stderr, "[shard] rank %d/%d m=%llu q=%d sb=%d pb=%d hb=%d sym [%llx, %llx] bounds [%llx, %llx]\n", rank,
            nranks, (unsigned long long)m, kk.q, kk.sym_bits, kk.pb, hb, (unsigned long long)kmm[0],
            (unsigned long long)kmm[1], (unsigned long long)kb.first, (unsigned long long)kb.second);
  if (kmm[0] < kb.first || kmm[1] > kb.second) throw ApiError{-7, "slice sym fields outside their bounds"};
  // LDS bucket sorts over the slice's bins, unless a bucket is too big for them
  if (!global && bucket_sort_slice<V>(ix, kk, m, hb, sbn, d_h0)) {
    HK_HIP(hipStreamSynchronize(s));
    ix.have_sa = ix.have_bwt = !ix.dbl.pending;   // pending: the rank exchange finishes the slice
    return;
  }
  ix.info[7] = 1;
  const int pbe = kk.pb + hb;
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  int slot;
  if (hb) {
    uint32_t* vq[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
    slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vq, 0, m, pbe, pbe + kk.sym_bits, false, s);
    TimedLaunch t(ix.timer, "shard_split_join", (double)m * (8 + 4 + 8 + 8));
    k_split_join<<<grid_for(m, 256, 16384), 256, 0, s>>>(kp[slot], vq[slot], m, hb, ix.sa.as<uint64_t>());
    HK_HIP(hipGetLastError());
  } else {
    V* vp[2] = {ix.vals[0].as<V>(), ix.vals[1].as<V>()};
    slot = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vp, 0, m, kk.pb, kk.pb + kk.sym_bits, false, s);
    std::swap(ix.sa, ix.vals[slot]);
    ix.vals[slot].ensure(m * sizeof(V) + 16);
  }
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  refine_after_sort<V>(ix, kk, slot, m, false);
  HK_HIP(hipStreamSynchronize(s));
  ix.have_sa = ix.have_bwt = !ix.dbl.pending;   // BWT of the slice (bwt[j] for SA[lo + j])
}

// Keyed coarse scheme: rank r owns the coarse buckets [C_r, C_{r+1}) (splitters of the exact global
// histogram) and its SA slice is [cum(C_r), cum(C_{r+1})).  gbelow (hkcsa_shard_build's global counts)
// must agree with the histogram.
template <typename V>
void shard_build_keyed(Index& ix, const uint64_t* ghist, const uint64_t* gbelow, int nranks, int rank) {
  const uint64_t n = ix.n;
  const std::vector<uint32_t> B = splitters(ghist, nranks, SH_KBUCKETS, true);
  std::vector<uint64_t> cum(SH_KBUCKETS + 1, 0);
  for (int c = 0; c < SH_KBUCKETS; ++c) cum[c + 1] = cum[c] + ghist[c];
  if (cum[SH_KBUCKETS] != n) throw ApiError{-7, "keyed coarse histogram does not count every suffix"};
  for (int r = 0; r <= nranks; ++r)
    if (gbelow[r] != cum[B[r]]) throw ApiError{-7, "global splitter counts disagree with the coarse histogram"};
  ix.shard_lo = cum[B[rank]];
  ix.shard_hi = cum[B[rank + 1]];
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  ix.info.assign(9, 0);
  ix.dbl = Index::DblState{};
  ix.sharded = true;
  ix.sa_pos64 = sizeof(V) == 8;
  ix.have_sa = ix.have_bwt = ix.have_wt = false;
  ix.sa.ensure(m * sizeof(V) + 16);
  ix.bwt.ensure(m + 64);
  if (!m) {
    ix.have_sa = ix.have_bwt = true;
    return;
  }
  build_slice_keyed<V>(ix, B[rank], B[rank + 1], m);
  HK_HIP(hipStreamSynchronize(ix.stream));
  ix.have_sa = ix.have_bwt = !ix.dbl.pending;   // pending: the rank exchange finishes the slice
}

}  // namespace

bool shard_keyed(Index& ix) { return shard_keyed_lb(ix) > 0; }

// Slot indices inside a slice are 32-bit (tie lists, refinement / doubling rows, big-bucket rows), so a
// slice must hold fewer than 2^32 - 1 suffixes.  Slices end on coarse-bucket boundaries: one coarse
// bucket larger than that (a run of one symbol, or a few-symbol period, in a text of n > 2^32) cannot be
// cut, and the build refuses it instead of wrapping the slots.
void check_slice_sizes(const uint64_t* below, int k) {
  for (int r = 0; r < k; ++r)
    if (below[r + 1] - below[r] >= 0xFFFFFFFFull)
      throw ApiError{-6, "a slice would hold 2^32 - 1 or more suffixes: one coarse bucket (first 16 key bits) "
                         "of the text is too large to split across slices"};
}

std::vector<uint64_t> slice_bounds(const uint64_t* hist, int nbins, int k) {
  const std::vector<uint32_t> B = splitters(hist, k, nbins, true);
  std::vector<uint64_t> below(k + 1, 0);
  uint64_t acc = 0;
  uint32_t c = 0;
  for (int r = 0; r <= k; ++r) {
    while (c < B[r]) acc += hist[c++];
    below[r] = acc;
  }
  check_slice_sizes(below.data(), k);
  return below;
}

void shard_histogram(Index& ix, int nranks, int rank, uint64_t* d_hist) {
  if (shard_keyed(ix)) {   // exact coarse histogram of the 16-aligned block
    const auto b = block_of(ix.n, nranks, rank);
    shard_coarse_hist(ix, b.first, b.second, d_hist);
    return;
  }
  KeyGeom kg = partition_geometry(ix);
  hipStream_t s = ix.stream;
  const uint64_t lo = (uint64_t)((__uint128_t)ix.n * (uint64_t)rank / (uint64_t)nranks);
  const uint64_t hi = (uint64_t)((__uint128_t)ix.n * (uint64_t)(rank + 1) / (uint64_t)nranks);
  upload_geometry(ix, kg);
  HK_HIP(hipMemsetAsync(d_hist, 0, SH_KBUCKETS * 8, s));
  if (hi > lo) {
    TimedLaunch t(ix.timer, "shard_hist", (double)(hi - lo) / SH_SAMPLE * (kg.q + 1));
    k_shard_hist<<<grid_for((hi - lo) / SH_SAMPLE + 1, 256, 512), 256, 0, s>>>(
        ix.text.as<uint8_t>(), ix.n, lo, hi, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048),
        bucket_geom(kg), reinterpret_cast<unsigned long long*>(d_hist));
    HK_HIP(hipGetLastError());
  }
}

void shard_counts(Index& ix, const uint64_t* h_global_hist, int nranks, int rank, uint64_t* d_below) {
  if (nranks > SH_MAX_RANKS) throw ApiError{-2, "at most 64 ranks"};
  if (shard_keyed(ix)) {   // the block's exact coarse counts, summed below every splitter
    const std::vector<uint32_t> B = splitters(h_global_hist, nranks, SH_KBUCKETS, true);
    const auto b = block_of(ix.n, nranks, rank);
    DevBuf d;
    d.ensure(SH_KBUCKETS * 8);
    shard_coarse_hist(ix, b.first, b.second, d.as<uint64_t>());
    std::vector<uint64_t> bh(SH_KBUCKETS), below(nranks + 1, 0);
    HK_HIP(hipMemcpyAsync(bh.data(), d.p, SH_KBUCKETS * 8, hipMemcpyDeviceToHost, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));
    uint64_t acc = 0;
    uint32_t c = 0;
    for (int r = 0; r <= nranks; ++r) {
      while (c < B[r]) acc += bh[c++];
      below[r] = acc;
    }
    HK_HIP(hipMemcpyAsync(d_below, below.data(), (nranks + 1) * 8, hipMemcpyHostToDevice, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));
    return;
  }
  KeyGeom kg = partition_geometry(ix);
  hipStream_t s = ix.stream;
  const uint64_t lo = (uint64_t)((__uint128_t)ix.n * (uint64_t)rank / (uint64_t)nranks);
  const uint64_t hi = (uint64_t)((__uint128_t)ix.n * (uint64_t)(rank + 1) / (uint64_t)nranks);
  upload_geometry(ix, kg);
  const BucketGeom g = bucket_geom(kg);
  const PrefixImages pi(kg, g);
  const std::vector<uint32_t> B = splitters(h_global_hist, nranks);
  std::vector<BelowImg> img(nranks + 1);
  for (int r = 0; r <= nranks; ++r) img[r] = below_img(pi, g, B[r]);
  ix.tile_d.ensure(sizeof(BelowImg) * (nranks + 1) + 64);
  HK_HIP(hipMemcpyAsync(ix.tile_d.p, img.data(), sizeof(BelowImg) * (nranks + 1), hipMemcpyHostToDevice, s));
  HK_HIP(hipMemsetAsync(d_below, 0, 8 * (nranks + 1), s));
  if (hi > lo) {
    TimedLaunch t(ix.timer, "shard_below", (double)(hi - lo));
    k_shard_below<<<grid_for((hi - lo) / 16 + 2, 256, 4096), 256, 0, s>>>(
        ix.text.as<uint8_t>(), ix.n, lo, hi, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048), g,
        pi.h, pi.topmask, pi.usable ? 0 : 1, ix.tile_d.as<BelowImg>(), nranks + 1,
        reinterpret_cast<unsigned long long*>(d_below));
    HK_HIP(hipGetLastError());
  }
  HK_HIP(hipStreamSynchronize(s));   // img staging buffer reuse
}

void shard_build(Index& ix, const uint64_t* h_global_hist, const uint64_t* h_global_below, int nranks, int rank) {
  if (h_global_below[rank + 1] >= h_global_below[rank]) check_slice_sizes(h_global_below + rank, 1);
  const bool keyed = shard_keyed(ix);
  if (ix.n > 0xFFFFFFFEull || (ix.flags & kFlagPos64)) {
    if (keyed) shard_build_keyed<uint64_t>(ix, h_global_hist, h_global_below, nranks, rank);
    else shard_build_t<uint64_t>(ix, h_global_hist, h_global_below, nranks, rank);
  } else {
    if (keyed) shard_build_keyed<uint32_t>(ix, h_global_hist, h_global_below, nranks, rank);
    else shard_build_t<uint32_t>(ix, h_global_hist, h_global_below, nranks, rank);
  }
}

// ---------------------------------------------------------------- one GPU, several slices
// The suffix array of a text too long for 32-bit positions (n >= 2^32 - 1: configs[4]'s 4 GiB + 1 on
// one MI355X; the reference's build_suffix_array has no size limit, csa/suffix_array.py:131-134), or of
// any text under kFlagSlices: the sharded slice pipeline runs k times on this device, slice r writing
// straight into its rows of one full SA and BWT (the slice's ix.sa / ix.bwt are views of them).  The
// slice bounds come from one partition histogram of the whole text (keyed scheme: the exact coarse
// histogram and balanced / equal-width splitters; else the sampled key histogram and exact counts
// below the splitters).  Groups still tied after a slice's chunk rounds wait; once every slice is
// placed, one ISA from the full SA drives prefix doubling over every pending slice, each round at
// K = the smallest common-prefix length of any of them (the sharded rank exchange's rule) with the ISA
// updated in place - on one device there is nothing to exchange.
int slices_for(const Index& ix) {
  if (ix.n < 0xFFFFFFFFull) return 4;   // kFlagSlices at a 32-bit size (parity tests)
  const uint64_t k = (ix.n + (1ull << 29)) >> 30;   // ~2^30 suffixes per slice: the 1 GiB pipeline
  return (int)std::max<uint64_t>(2, std::min<uint64_t>(64, k));
}

namespace {
struct PendingSlice {   // a slice whose tied groups wait for the full ISA
  uint64_t lo = 0, hi = 0;
  Index::DblState dbl;
  DevBuf act[2][3], head_slot;
};
void swap_pending(Index& ix, PendingSlice& p) {
  std::swap(ix.dbl, p.dbl);
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 3; ++j) std::swap(ix.act[i][j], p.act[i][j]);
  std::swap(ix.head_slot, p.head_slot);
}
}  // namespace

void build_sa_slices(Index& ix, int k) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  if (k < 1 || k > SH_MAX_RANKS) throw ApiError{-1, "slices: 1 to 64 slices"};
  ix.have_alpha = false;   // every build recomputes the byte histogram / C (utils/utils.py:16-24)
  compute_alphabet(ix);
  ix.have_sa = ix.have_bwt = ix.have_wt = false;
  ix.dbl = Index::DblState{};
  const bool w64 = n > 0xFFFFFFFEull || (ix.flags & kFlagPos64);   // shard_build's position width
  const size_t V = w64 ? 8 : 4;
  // the full arrays (the previous build's, when the handle holds them)
  DevBuf full_sa, full_bwt;
  if (ix.sa.owned) std::swap(full_sa, ix.sa);
  if (ix.bwt.owned) std::swap(full_bwt, ix.bwt);
  ix.sa.release();
  ix.bwt.release();
  full_sa.ensure(n * V + 16);
  full_bwt.ensure(n + 64);
  if (n <= 1) {   // (kFlagSlices on a one-symbol text)
    HK_HIP(hipMemsetAsync(full_sa.p, 0, V, s));
    HK_HIP(hipMemcpyAsync(full_bwt.p, ix.text.p, n, hipMemcpyDeviceToDevice, s));
    HK_HIP(hipStreamSynchronize(s));
    ix.sa = std::move(full_sa);
    ix.bwt = std::move(full_bwt);
    ix.sharded = false;
    ix.sa_pos64 = w64;
    ix.info.assign(9, 0);
    ix.have_sa = ix.have_bwt = true;
    return;
  }
  struct LocalGuard {   // the sharded state and the row views never outlive the call
    Index& ix;
    ~LocalGuard() {
      ix.slices_local = false;
      ix.sharded = false;
      for (DevBuf* b : {&ix.sa, &ix.bwt, &ix.vals[0], &ix.vals[1], &ix.keys[0], &ix.keys[1]})
        if (!b->owned) b->release();
      ix.fused.reset();
    }
  } guard{ix};
  ix.slices_local = true;
  // ---- slice bounds
  const bool keyed = shard_keyed(ix);
  std::vector<uint64_t> gh(SH_KBUCKETS, 0), below(k + 1, 0);
  std::vector<uint32_t> B;   // keyed: the coarse splitters
  {
    DevBuf d;
    d.ensure((SH_KBUCKETS + 1) * 8 + 64);
    shard_histogram(ix, 1, 0, d.as<uint64_t>());
    HK_HIP(hipMemcpyAsync(gh.data(), d.p, SH_KBUCKETS * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    if (keyed) {
      B = splitters(gh.data(), k, SH_KBUCKETS, true);
      below = slice_bounds(gh.data(), SH_KBUCKETS, k);
    } else {
      std::vector<uint64_t> part(k + 1);
      for (int r = 0; r < k; ++r) {   // each block's counts below every splitter, summed
        shard_counts(ix, gh.data(), k, r, d.as<uint64_t>());
        HK_HIP(hipMemcpyAsync(part.data(), d.p, (k + 1) * 8, hipMemcpyDeviceToHost, s));
        HK_HIP(hipStreamSynchronize(s));
        for (int j = 0; j <= k; ++j) below[j] += part[j];
      }
    }
  }
  if (below[0] != 0 || below[k] != n) throw ApiError{-7, "slices: the partition does not cover the text"};
  check_slice_sizes(below.data(), k);
  // ---- the slices, one after another
  std::vector<uint64_t> info(9, 0), ties;
  std::vector<PendingSlice> pend;
  auto point = [&](uint64_t lo, uint64_t hi) {   // the slice's SA / BWT rows of the full arrays
    ix.sa.view(full_sa.as<uint8_t>() + lo * V, (hi - lo) * V + 16);
    ix.bwt.view(full_bwt.as<uint8_t>() + lo, hi - lo + 64);
    ix.shard_lo = lo;
    ix.shard_hi = hi;
  };
  constexpr int kFuse = 4;   // slices per fused pass A (one scan of T' for the group)
  for (int r = 0; r < k; ++r) {
    if (keyed && r % kFuse == 0) slices_fuse(ix, B, below, r, std::min(k, r + kFuse), w64);
    const uint64_t lo = below[r], hi = below[r + 1];
    point(lo, hi);
    void* const rows = ix.sa.p;
    shard_build(ix, gh.data(), below.data(), k, r);
    if (ix.shard_lo != lo || ix.shard_hi != hi) throw ApiError{-7, "slices: a slice left its bounds"};
    if (ix.sa.p != rows) {   // a global-path slice adopted a value buffer as its SA: move the rows over
      HK_HIP(hipMemcpyAsync(rows, ix.sa.p, (hi - lo) * V, hipMemcpyDeviceToDevice, s));
      for (int i = 0; i < 2; ++i)
        if (!ix.vals[i].owned) ix.vals[i] = std::move(ix.sa);
    }
    for (int i = 0; i < 2; ++i) {   // no view may stay behind as the next slice's scratch
      if (!ix.vals[i].owned) ix.vals[i].release();
      if (!ix.keys[i].owned) ix.keys[i].release();
    }
    for (int j : {0, 1, 4, 5, 6}) info[j] += ix.info[j];
    info[2] = std::max(info[2], ix.info[2]);
    info[3] = std::max(info[3], ix.info[3]);
    info[7] |= ix.info[7];
    info[8] += ix.info[8];
    for (size_t j = 9; j < ix.info.size(); ++j) {
      if (ties.size() < j - 8) ties.push_back(0);
      ties[j - 9] += ix.info[j];
    }
    if (ix.dbl.pending) {
      pend.emplace_back();
      PendingSlice& p = pend.back();
      p.lo = lo;
      p.hi = hi;
      swap_pending(ix, p);
      // while parked only the active lists and head slots matter: the round's output lists are
      // re-allocated at the list's size when its doubling starts (dbl_round_t)
      for (DevBuf& b : p.act[p.dbl.cur ^ 1]) b.release();
    }
  }
  ix.fused.reset();   // (the last group's records)
  // ---- prefix doubling over the slices still tied (repetitive texts)
  if (!pend.empty()) {
    ix.sa_pos64 = w64;
    dbl_ensure_isa(ix);
    dbl_isa_segment(ix, full_sa.p, n, 0);   // isa[SA[j]] = j over the full (provisional) SA
    for (auto& p : pend) {   // tied suffixes: their group head's slot
      swap_pending(ix, p);
      point(p.lo, p.hi);
      dbl_emit_groups(ix);
      swap_pending(ix, p);
    }
    ix.info.assign(9, 0);
    for (int round = 0;; ++round) {
      if (round > 64) throw ApiError{-7, "slices: prefix doubling did not converge"};
      uint64_t K = ~0ull;
      for (auto& p : pend)
        if (p.dbl.A) K = std::min(K, p.dbl.h);
      if (K == ~0ull) break;
      for (auto& p : pend) {
        if (!p.dbl.A) continue;
        swap_pending(ix, p);
        point(p.lo, p.hi);
        dbl_round(ix, K);
        swap_pending(ix, p);
      }
      info[2] += 1ull << 32;
    }
  }
  HK_HIP(hipStreamSynchronize(s));
  ix.sa = std::move(full_sa);
  ix.bwt = std::move(full_bwt);
  ix.sharded = false;
  ix.slices_local = false;
  ix.shard_lo = 0;
  ix.shard_hi = n;
  ix.sa_pos64 = w64;
  ix.dbl = Index::DblState{};
  ix.info = info;
  ix.info.insert(ix.info.end(), ties.begin(), ties.end());
  ix.have_sa = ix.have_bwt = true;
}

int shard_buckets() { return SH_KBUCKETS; }
int shard_sample() { return SH_SAMPLE; }

void shard_get_bwt(Index& ix, uint64_t a, uint64_t b, uint8_t* out) {
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  if (!(a <= b && b <= m)) throw ApiError{-4, "shard BWT range out of bounds"};
  if (a == b) return;
  HK_HIP(hipMemcpyAsync(out, ix.bwt.as<uint8_t>() + a, b - a, hipMemcpyDeviceToHost, ix.stream));
  HK_HIP(hipStreamSynchronize(ix.stream));
}

void shard_get_sa(Index& ix, uint64_t a, uint64_t b, uint64_t* out) {
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  if (!(a <= b && b <= m)) throw ApiError{-4, "shard SA range out of bounds"};
  if (a == b) return;
  hipStream_t s = ix.stream;
  if (ix.sa_pos64) {
    HK_HIP(hipMemcpyAsync(out, ix.sa.as<uint64_t>() + a, (b - a) * 8, hipMemcpyDeviceToHost, s));
  } else {
    sa_to_host_u64(ix, a, b - a, out);   // widened on the GPU in chunks, straight into `out`
  }
  HK_HIP(hipStreamSynchronize(s));
}

static ShardComm g_comm;  // one communicator per process (one process per GPU)

namespace {

void comm_abort() {
  if (g_comm.comm) (void)ncclCommAbort(g_comm.comm);
  g_comm.comm = nullptr;
  g_comm.nranks = 0;
  g_comm.rank = -1;
}

// an RCCL call that fails tears the communicator down (peers see their own collective fail)
void nccl_do(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) {
    const std::string msg = std::string(what) + ": " + ncclGetErrorString(r);
    comm_abort();
    throw ApiError{-8, msg};
  }
}

// Per-rank record exchanged after every local step.  A local failure is reported through it, so
// every rank leaves the collective sequence at the same point instead of blocking in a collective.
struct RankStatus {
  uint64_t lo, hi, A, h, npairs, err;
};
static_assert(sizeof(RankStatus) == 48, "RankStatus layout");

std::vector<RankStatus> gather_status(Index& ix, const RankStatus& mine, DevBuf& buf) {
  const int N = g_comm.nranks;
  hipStream_t s = ix.stream;
  buf.ensure(sizeof(RankStatus) * N + 64);
  RankStatus* d = buf.as<RankStatus>();
  HK_HIP(hipMemcpyAsync(d + g_comm.rank, &mine, sizeof(RankStatus), hipMemcpyHostToDevice, s));
  {
    TimedLaunch t(ix.timer, "rccl_allgather_status", (double)N * sizeof(RankStatus));
    nccl_do(ncclAllGather(d + g_comm.rank, d, sizeof(RankStatus), ncclUint8, g_comm.comm, s), "ncclAllGather");
  }
  std::vector<RankStatus> all(N);
  HK_HIP(hipMemcpyAsync(all.data(), d, sizeof(RankStatus) * N, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  for (int r = 0; r < N; ++r)
    if (all[r].err) {
      if (r == g_comm.rank) continue;
      throw ApiError{-8, "sharded build failed on rank " + std::to_string(r) + " (error " +
                             std::to_string((int64_t)all[r].err) + ")"};
    }
  return all;
}

// Runs f; a failure becomes an error code in the status record (and the message is kept).
template <typename F>
uint64_t local_step(F&& f, std::string& emsg, int& ecode) {
  try {
    f();
    return 0;
  } catch (const ApiError& e) {
    emsg = e.msg;
    ecode = e.code;
  } catch (const HipError& e) {
    emsg = std::string("HIP error ") + hipGetErrorString(e.code) + " in " + e.where;
    ecode = -2;
    (void)hipGetLastError();
  }
  return (uint64_t)(int64_t)ecode;
}

constexpr uint64_t kIsaChunk = 1ull << 26;    // SA entries per rank per all-gather of the ISA build
constexpr uint64_t kPairChunk = 1ull << 24;   // (position, ISA) pairs per rank per all-gather

// In-place all-gather of per-rank ragged device arrays, CH elements of esz bytes per rank per call:
// for each chunk, rank r's elements [off, off + cnt_r) land in gb[r*CH .. ) and visit(r, ptr, cnt,
// off) consumes them.
template <typename Visit>
void ragged_allgather(Index& ix, const uint8_t* mine, const std::vector<uint64_t>& cnt, size_t esz, uint64_t CH,
                      DevBuf& gb, const char* timer, Visit&& visit) {
  const int N = g_comm.nranks, me = g_comm.rank;
  hipStream_t s = ix.stream;
  uint64_t mx = 0;
  for (uint64_t c : cnt) mx = std::max(mx, c);
  if (!mx) return;
  CH = std::min(CH, mx);
  gb.ensure((size_t)N * CH * esz + 64);
  uint8_t* base = gb.as<uint8_t>();
  for (uint64_t off = 0; off < mx; off += CH) {
    const uint64_t my = cnt[me] > off ? std::min(CH, cnt[me] - off) : 0;
    if (my) HK_HIP(hipMemcpyAsync(base + (size_t)me * CH * esz, mine + off * esz, my * esz, hipMemcpyDeviceToDevice, s));
    {
      TimedLaunch t(ix.timer, timer, (double)N * CH * esz);
      nccl_do(ncclAllGather(base + (size_t)me * CH * esz, base, CH * esz, ncclUint8, g_comm.comm, s),
              "ncclAllGather");
    }
    for (int r = 0; r < N; ++r) {
      const uint64_t c = cnt[r] > off ? std::min(CH, cnt[r] - off) : 0;
      if (c) visit(r, base + (size_t)r * CH * esz, c, off);
    }
  }
}

// Prefix doubling of the slices' tied suffixes with the rank exchange:
// every rank keeps a replica of the global ISA, built from an all-gather of the SA slices and
// refreshed after each round by an all-gather of the (position, ISA) pairs of the suffixes that
// round re-ranked.  K = the smallest common-prefix length of any group still tied anywhere.
// agreed: set while the error being thrown is known to every rank (a status exchange reported it)
void shard_doubling_rounds(Index& ix, std::vector<RankStatus> st, DevBuf& sbuf, DevBuf& gb, bool& agreed) {
  const int N = g_comm.nranks, me = g_comm.rank;
  const size_t V = ix.sa_pos64 ? 8 : 4;
  {
    std::vector<uint64_t> cnt(N);
    for (int r = 0; r < N; ++r) cnt[r] = st[r].hi - st[r].lo;
    ragged_allgather(ix, ix.sa.as<uint8_t>(), cnt, V, kIsaChunk, gb, "rccl_allgather_sa",
                     [&](int r, const uint8_t* p, uint64_t c, uint64_t off) {
                       dbl_isa_segment(ix, p, c, st[r].lo + off);
                     });
  }
  for (int round = 0;; ++round) {
    if (round > 64) throw ApiError{-7, "sharded prefix doubling did not converge"};
    {
      std::vector<uint64_t> cnt(N);
      for (int r = 0; r < N; ++r) cnt[r] = st[r].npairs;
      ragged_allgather(ix, ix.upd.as<uint8_t>(), cnt, 16, kPairChunk, gb, "rccl_allgather_pairs",
                       [&](int, const uint8_t* p, uint64_t c, uint64_t) {
                         dbl_apply_pairs(ix, reinterpret_cast<const uint64_t*>(p), c);
                       });
    }
    uint64_t K = ~0ull;
    for (int r = 0; r < N; ++r)
      if (st[r].A) K = std::min(K, st[r].h);
    std::string emsg;
    int ecode = 0;
    const uint64_t err = local_step([&] {
      if (ix.dbl.A) dbl_round(ix, K);
      else ix.dbl.npairs = 0;
      HK_HIP(hipStreamSynchronize(ix.stream));
    }, emsg, ecode);
    const RankStatus mine{ix.shard_lo, ix.shard_hi, err ? 0 : ix.dbl.A, ix.dbl.h, err ? 0 : ix.dbl.npairs, err};
    agreed = true;   // a peer's failure is thrown by gather_status itself, after the exchange
    st = gather_status(ix, mine, sbuf);
    if (err) throw ApiError{ecode, emsg};
    agreed = false;
    uint64_t tot = 0;
    for (int r = 0; r < N; ++r) tot += st[r].A;
    if (!tot) break;
  }
  (void)me;
  ix.dbl.pending = false;
  ix.have_sa = ix.have_bwt = true;
}


// The allocations a rank can fail on (the ISA replica, the gather staging) run first, under local_step,
// and one status exchange makes every rank leave together before any all-gather; a failure after that
// (a launch inside a gather's visit) aborts the communicator so that peers see their collective fail.
void shard_doubling(Index& ix, std::vector<RankStatus> st, DevBuf& sbuf) {
  const int N = g_comm.nranks, me = g_comm.rank;
  const size_t V = ix.sa_pos64 ? 8 : 4;
  DevBuf gb;
  {
    uint64_t mx = 1;
    for (int r = 0; r < N; ++r) mx = std::max(mx, st[r].hi - st[r].lo);
    std::string emsg;
    int ecode = 0;
    const uint64_t err = local_step([&] {
      dbl_ensure_isa(ix);
      gb.ensure(std::max((size_t)N * std::min(kIsaChunk, mx) * V, (size_t)N * kPairChunk * 16) + 64);
    }, emsg, ecode);
    const RankStatus mine{ix.shard_lo, ix.shard_hi, st[me].A, st[me].h, st[me].npairs, err};
    st = gather_status(ix, mine, sbuf);
    if (err) throw ApiError{ecode, emsg};
  }
  bool agreed = false;
  try {
    shard_doubling_rounds(ix, st, sbuf, gb, agreed);
  } catch (...) {
    if (!agreed) comm_abort();
    throw;
  }
}

}  // namespace

void build_sa_sharded(Index& ix, const uint8_t id[128], int nranks, int rank) {
  hipStream_t s = ix.stream;
  if (!g_comm.comm || g_comm.nranks != nranks || g_comm.rank != rank || memcmp(g_comm.id, id, 128) != 0) {
    if (g_comm.comm) (void)ncclCommDestroy(g_comm.comm);
    g_comm.comm = nullptr;
    ncclUniqueId uid;
    static_assert(sizeof(uid.internal) == 128, "unexpected RCCL unique id size");
    memcpy(uid.internal, id, 128);
    ncclcheck(ncclCommInitRank(&g_comm.comm, nranks, uid, rank), "ncclCommInitRank");
    g_comm.nranks = nranks;
    g_comm.rank = rank;
    memcpy(g_comm.id, id, 128);
  }
  std::string emsg;
  int ecode = 0;
  DevBuf hist;
  hist.ensure((SH_KBUCKETS + 1) * 8 + 64);
  // phase 0: every build recomputes the byte histogram / C (utils/utils.py:16-24): each rank counts
  // its 16-aligned block of T' and an all-reduce sums them (+ a failure slot), so no rank reads
  // all of T' for it
  uint64_t err = local_step([&] {
    const auto b = block_of(ix.n, nranks, rank);
    byte_hist_range(ix, b.first, b.second, hist.as<unsigned long long>());
  }, emsg, ecode);
  {
    const uint64_t e1 = err ? 1 : 0;
    HK_HIP(hipMemcpyAsync(hist.as<uint64_t>() + 256, &e1, 8, hipMemcpyHostToDevice, s));
    TimedLaunch t(ix.timer, "rccl_allreduce_bytes", 257.0 * 8);
    nccl_do(ncclAllReduce(hist.p, hist.p, 257, ncclUint64, ncclSum, g_comm.comm, s), "ncclAllReduce");
  }
  {
    std::vector<uint64_t> bh(257);
    HK_HIP(hipMemcpyAsync(bh.data(), hist.p, 257 * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    if (err) throw ApiError{ecode, emsg};
    if (bh[256]) throw ApiError{-8, "sharded build failed on a peer rank (byte histogram)"};
    set_alphabet(ix, bh.data());
  }
  // phase 1: partition histogram (keyed scheme: exact coarse counts of the block; else the sampled
  // partition-key histogram); the extra bin carries failures (summed)
  bool keyed = false;
  err = local_step([&] {
    keyed = shard_keyed(ix);
    shard_histogram(ix, nranks, rank, hist.as<uint64_t>());
  }, emsg, ecode);
  // every rank reduces the same count whatever its scheme decision (a failed rank could not know it);
  // the partition-key scheme leaves the bins past SH_BUCKETS zero
  const int nbh = SH_KBUCKETS;
  {
    const uint64_t e1 = err ? 1 : 0;
    HK_HIP(hipMemcpyAsync(hist.as<uint64_t>() + nbh, &e1, 8, hipMemcpyHostToDevice, s));
    TimedLaunch t(ix.timer, "rccl_allreduce_hist", (double)nbh * 8);
    nccl_do(ncclAllReduce(hist.p, hist.p, nbh + 1, ncclUint64, ncclSum, g_comm.comm, s), "ncclAllReduce");
  }
  std::vector<uint64_t> h(SH_KBUCKETS + 1, 0);
  HK_HIP(hipMemcpyAsync(h.data(), hist.p, (nbh + 1) * 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (err) throw ApiError{ecode, emsg};
  if (h[nbh]) throw ApiError{-8, "sharded build failed on a peer rank (histogram)"};
  std::vector<uint64_t> below(nranks + 2, 0);
  if (keyed) {
    // exact counts: the slice bounds follow from the histogram itself (no second collective)
    const std::vector<uint32_t> B = splitters(h.data(), nranks, SH_KBUCKETS, true);
    uint64_t acc = 0;
    uint32_t c = 0;
    for (int r = 0; r <= nranks; ++r) {
      while (c < B[r]) acc += h[c++];
      below[r] = acc;
    }
  } else {
    // phase 2: exact slice sizes: per-rank counts below every splitter, summed (+ failure slot)
    err = local_step([&] { shard_counts(ix, h.data(), nranks, rank, hist.as<uint64_t>()); }, emsg, ecode);
    {
      const uint64_t e1 = err ? 1 : 0;
      HK_HIP(hipMemcpyAsync(hist.as<uint64_t>() + nranks + 1, &e1, 8, hipMemcpyHostToDevice, s));
      TimedLaunch t(ix.timer, "rccl_allreduce_counts", (double)(nranks + 2) * 8);
      nccl_do(ncclAllReduce(hist.p, hist.p, nranks + 2, ncclUint64, ncclSum, g_comm.comm, s), "ncclAllReduce");
    }
    HK_HIP(hipMemcpyAsync(below.data(), hist.p, (nranks + 2) * 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    if (err) throw ApiError{ecode, emsg};
    if (below[nranks + 1]) throw ApiError{-8, "sharded build failed on a peer rank (slice counts)"};
  }
  // phase 3: the slice sort; then every rank's bounds / tied count are exchanged
  err = local_step([&] { shard_build(ix, h.data(), below.data(), nranks, rank); }, emsg, ecode);
  DevBuf sbuf;
  const RankStatus mine{ix.shard_lo, ix.shard_hi, err ? 0 : ix.dbl.A, ix.dbl.h, err ? 0 : ix.dbl.npairs, err};
  const std::vector<RankStatus> st = gather_status(ix, mine, sbuf);
  if (err) throw ApiError{ecode, emsg};
  uint64_t expect = 0, tied = 0;
  for (int r = 0; r < nranks; ++r) {
    if (st[r].lo != expect) throw ApiError{-8, "shard slices do not tile the suffix array"};
    expect = st[r].hi;
    tied += st[r].A;
  }
  if (expect != ix.n) throw ApiError{-8, "shard slices do not cover the suffix array"};
  ix.shard_bounds.resize((size_t)nranks + 1);
  for (int r = 0; r < nranks; ++r) ix.shard_bounds[r] = st[r].lo;
  ix.shard_bounds[nranks] = ix.n;
  // phase 4 (repetitive texts only): prefix doubling with the ISA rank exchange
  if (tied) shard_doubling(ix, st, sbuf);
}

// Replicas for batched queries: all-gather every rank's SA slice and BWT rows, so
// each rank holds the full SA + BWT (and then builds its own wavelet tree).
void shard_replicate(Index& ix) {
  if (!ix.sharded || !ix.have_sa) throw ApiError{-3, "replicate: no sharded suffix array"};
  if (!g_comm.comm || (int)ix.shard_bounds.size() != g_comm.nranks + 1)
    throw ApiError{-3, "replicate: no communicator of the sharded build"};
  const int N = g_comm.nranks;
  const uint64_t n = ix.n;
  const size_t V = ix.sa_pos64 ? 8 : 4;
  hipStream_t s = ix.stream;
  std::vector<uint64_t> cnt(N);
  uint64_t mx = 1;
  for (int r = 0; r < N; ++r) {
    cnt[r] = ix.shard_bounds[r + 1] - ix.shard_bounds[r];
    mx = std::max(mx, cnt[r]);
  }
  DevBuf full_sa, full_bwt, gb, sbuf;
  // the allocations first, then one status exchange: every rank leaves together if any failed
  {
    std::string emsg;
    int ecode = 0;
    const uint64_t err = local_step([&] {
      full_sa.ensure(n * V + 16);
      full_bwt.ensure(n + 64);
      gb.ensure((size_t)N * std::max(std::min(kIsaChunk, mx) * V, std::min(kIsaChunk * 8, mx)) + 64);
    }, emsg, ecode);
    const RankStatus mine{ix.shard_lo, ix.shard_hi, 0, 0, 0, err};
    (void)gather_status(ix, mine, sbuf);
    if (err) throw ApiError{ecode, emsg};
  }
  try {
    ragged_allgather(ix, ix.sa.as<uint8_t>(), cnt, V, kIsaChunk, gb, "rccl_allgather_sa",
                     [&](int r, const uint8_t* p, uint64_t c, uint64_t off) {
                       HK_HIP(hipMemcpyAsync(full_sa.as<uint8_t>() + (ix.shard_bounds[r] + off) * V, p, c * V,
                                             hipMemcpyDeviceToDevice, s));
                     });
    ragged_allgather(ix, ix.bwt.as<uint8_t>(), cnt, 1, kIsaChunk * 8, gb, "rccl_allgather_bwt",
                     [&](int r, const uint8_t* p, uint64_t c, uint64_t off) {
                       HK_HIP(hipMemcpyAsync(full_bwt.as<uint8_t>() + ix.shard_bounds[r] + off, p, c,
                                             hipMemcpyDeviceToDevice, s));
                     });
    HK_HIP(hipStreamSynchronize(s));
  } catch (...) {
    comm_abort();   // a peer may be waiting in the next all-gather
    throw;
  }
  std::swap(ix.sa, full_sa);
  std::swap(ix.bwt, full_bwt);
  ix.sharded = false;
  ix.shard_lo = 0;
  ix.shard_hi = n;
  ix.have_sa = ix.have_bwt = true;
  ix.have_wt = false;
}

namespace {
// adopted replica check: every entry < n and seen once (a bitmap, one atomic OR each; n entries, so
// no duplicate means a permutation) and bwt[i] == T'[sa[i] - 1] (wrapping, csa/bwt.py:8-11); flags:
// bit 0 out of range / duplicate, bit 1 BWT mismatch
template <typename V>
__global__ __launch_bounds__(256) void k_adopt_check(const V* __restrict__ sa, const uint8_t* __restrict__ bwt,
                                                     const uint8_t* __restrict__ t, uint64_t n,
                                                     uint32_t* __restrict__ seen, unsigned int* __restrict__ flag) {
  uint32_t f = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t p = sa[i];
    if (p >= n) {
      f |= 1u;
      continue;
    }
    const uint32_t bit = 1u << (p & 31);
    if (atomicOr(&seen[p >> 5], bit) & bit) f |= 1u;
    if (bwt[i] != t[p ? p - 1 : n - 1]) f |= 2u;
  }
  if (f) atomicOr(flag, f);
}
}  // namespace

// Host-assembled replica (hosts running their own collectives): the full SA and BWT, checked on the
// GPU (a permutation of [0, n) whose BWT rows match the text) before it replaces the slice.
void shard_adopt(Index& ix, const uint64_t* h_sa, const uint8_t* h_bwt) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  if (!ix.sharded) throw ApiError{-3, "adopt: the handle holds no sharded build"};
  const bool w64 = ix.sa_pos64 || n > 0xFFFFFFFFull;
  DevBuf full_sa, full_bwt;
  full_sa.ensure(n * (w64 ? 8 : 4) + 16);
  full_bwt.ensure(n + 64);
  if (w64) {
    HK_HIP(hipMemcpyAsync(full_sa.p, h_sa, n * 8, hipMemcpyHostToDevice, s));
  } else {
    std::vector<uint32_t> t(n);
    for (uint64_t i = 0; i < n; ++i) {   // (narrowed here: an entry >= n must not wrap into range)
      if (h_sa[i] >= n) throw ApiError{-4, "adopt: suffix array entry out of range"};
      t[i] = (uint32_t)h_sa[i];
    }
    HK_HIP(hipMemcpyAsync(full_sa.p, t.data(), n * 4, hipMemcpyHostToDevice, s));
    HK_HIP(hipStreamSynchronize(s));
  }
  HK_HIP(hipMemcpyAsync(full_bwt.p, h_bwt, n, hipMemcpyHostToDevice, s));
  {
    DevBuf seen;
    seen.ensure((n / 32 + 1) * 4 + 16);
    HK_HIP(hipMemsetAsync(seen.p, 0, (n / 32 + 1) * 4 + 16, s));
    unsigned int* d_flag = reinterpret_cast<unsigned int*>(seen.as<uint8_t>() + (n / 32 + 1) * 4);
    if (w64)
      k_adopt_check<uint64_t><<<grid_for(n, 256, 8192), 256, 0, s>>>(full_sa.as<uint64_t>(), full_bwt.as<uint8_t>(),
                                                                      ix.text.as<uint8_t>(), n, seen.as<uint32_t>(),
                                                                      d_flag);
    else
      k_adopt_check<uint32_t><<<grid_for(n, 256, 8192), 256, 0, s>>>(full_sa.as<uint32_t>(), full_bwt.as<uint8_t>(),
                                                                      ix.text.as<uint8_t>(), n, seen.as<uint32_t>(),
                                                                      d_flag);
    HK_HIP(hipGetLastError());
    unsigned int flag = 0;
    HK_HIP(hipMemcpyAsync(&flag, d_flag, 4, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    if (flag & 1u) throw ApiError{-4, "adopt: the suffix array is not a permutation of [0, n)"};
    if (flag & 2u) throw ApiError{-4, "adopt: BWT rows do not match T'[SA - 1]"};
  }
  std::swap(ix.sa, full_sa);
  std::swap(ix.bwt, full_bwt);
  ix.sa_pos64 = w64;
  ix.sharded = false;
  ix.shard_lo = 0;
  ix.shard_hi = n;
  ix.dbl = Index::DblState{};
  ix.have_sa = ix.have_bwt = true;
  ix.have_wt = false;
}

// ---------------------------------------------------------------- host-driven rank exchange
void shard_status(Index& ix, uint64_t st[4]) {
  if (!ix.sharded) throw ApiError{-3, "index is not sharded"};
  st[0] = ix.shard_lo;
  st[1] = ix.shard_hi;
  st[2] = ix.dbl.A;
  st[3] = ix.dbl.h;
}

void shard_isa_segment_host(Index& ix, const uint64_t* h_sa, uint64_t count, uint64_t lo) {
  if (!ix.sharded || !ix.dbl.pending) throw ApiError{-3, "no pending sharded prefix doubling"};
  if (lo > ix.n || count > ix.n - lo) throw ApiError{-4, "ISA segment out of range"};
  if (!count) return;
  dbl_ensure_isa(ix);
  DevBuf tmp;
  const size_t V = ix.sa_pos64 ? 8 : 4;
  tmp.ensure(count * V + 16);
  if (ix.sa_pos64) {
    HK_HIP(hipMemcpyAsync(tmp.p, h_sa, count * 8, hipMemcpyHostToDevice, ix.stream));
  } else {
    std::vector<uint32_t> t(count);
    for (uint64_t i = 0; i < count; ++i) {
      if (h_sa[i] >= ix.n) throw ApiError{-4, "ISA segment entry out of range"};
      t[i] = (uint32_t)h_sa[i];
    }
    HK_HIP(hipMemcpyAsync(tmp.p, t.data(), count * 4, hipMemcpyHostToDevice, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));
  }
  dbl_isa_segment(ix, tmp.p, count, lo);
  HK_HIP(hipStreamSynchronize(ix.stream));
}

uint64_t shard_updates(Index& ix, uint64_t* h_pairs, uint64_t cap) {
  if (!ix.sharded) throw ApiError{-3, "index is not sharded"};
  const uint64_t c = ix.dbl.npairs;
  if (h_pairs && c) {
    if (cap < c) throw ApiError{-4, "pair buffer too small"};
    HK_HIP(hipMemcpyAsync(h_pairs, ix.upd.p, c * 16, hipMemcpyDeviceToHost, ix.stream));
    HK_HIP(hipStreamSynchronize(ix.stream));
  }
  return c;
}

void shard_apply_host(Index& ix, const uint64_t* h_pairs, uint64_t count) {
  if (!ix.sharded || !ix.dbl.pending) throw ApiError{-3, "no pending sharded prefix doubling"};
  if (!count) return;
  for (uint64_t i = 0; i < count; ++i)
    if (h_pairs[2 * i] >= ix.n || h_pairs[2 * i + 1] >= ix.n) throw ApiError{-4, "ISA pair out of range"};
  dbl_ensure_isa(ix);
  DevBuf tmp;
  tmp.ensure(count * 16 + 16);
  HK_HIP(hipMemcpyAsync(tmp.p, h_pairs, count * 16, hipMemcpyHostToDevice, ix.stream));
  dbl_apply_pairs(ix, tmp.as<uint64_t>(), count);
  HK_HIP(hipStreamSynchronize(ix.stream));
}

void shard_round(Index& ix, uint64_t K) {
  if (!ix.sharded) throw ApiError{-3, "index is not sharded"};
  if (!ix.dbl.pending || !ix.dbl.A) {   // final (or never tied): nothing to sort, no pairs to re-send
    ix.dbl.npairs = 0;
    return;
  }
  if (!ix.isa.p) throw ApiError{-3, "ISA replica not loaded (hkcsa_shard_isa_segment)"};
  if (ix.dbl.A) dbl_round(ix, K);
  else ix.dbl.npairs = 0;
  HK_HIP(hipStreamSynchronize(ix.stream));
  if (!ix.dbl.A) ix.have_sa = ix.have_bwt = true;   // this slice is final (peers may still need its pairs)
}

// the last round of every rank: the host calls hkcsa_shard_round until all ranks report A = 0;
// a rank's slice is final as soon as its own A is 0
void comm_unique_id(uint8_t id[128]) {
  ncclUniqueId uid;
  ncclcheck(ncclGetUniqueId(&uid), "ncclGetUniqueId");
  memcpy(id, uid.internal, 128);
}

}  // namespace hk
