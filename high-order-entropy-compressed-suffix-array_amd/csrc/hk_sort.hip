// hk_sort.hip — scans and the onesweep LSD radix sort (gfx950).
//
// The radix pass is the roofline kernel of the suffix-array build (SURVEY.md §8d:
// algorithmic bytes 2*N*(K+V) per 8-bit pass).  One launch per digit:
//   * every workgroup takes a tile id from an atomic counter (so all lower tiles have
//     started: the lookback below always makes progress),
//   * ranks its 8192 keys per wave with an LDS match-mask table (a lane ORs its bit into its
//     digit's mask, reads back the lanes sharing the digit; a per-wave LDS histogram carries
//     counts across the wave's 16 items, stable order),
//   * publishes its 256 digit counts as 8-byte {epoch|flag|count} granules written and
//     polled with relaxed agent-scope (sc1) accesses — the granule IS the flag, so no
//     fences are needed (MI355X_MICROARCH.md §visibility, R2 granules),
//   * looks back over predecessor tiles for its exclusive digit prefix (decoupled lookback),
//   * stages keys then values through LDS in sorted order and writes them out so that
//     consecutive lanes write consecutive addresses of one digit run.
// Digit offsets come from one upfront histogram kernel over all digit positions.

#include <cstdlib>

#include "hk_sort.hpp"

namespace hk {

// =============================================================== scans
namespace {

constexpr int SC_T = 256;
constexpr int SC_I = 16;
constexpr int SC_TILE = SC_T * SC_I;

struct OpSum {
  static __device__ __forceinline__ uint64_t id() { return 0; }
  static __device__ __forceinline__ uint64_t f(uint64_t a, uint64_t b) { return a + b; }
};
struct OpMax {
  static __device__ __forceinline__ uint64_t id() { return 0; }
  static __device__ __forceinline__ uint64_t f(uint64_t a, uint64_t b) { return a > b ? a : b; }
};

template <typename Op>
__device__ __forceinline__ uint64_t block_reduce(uint64_t v, uint64_t* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = Op::f(v, __shfl_xor(v, o, 64));
  if (lane == 0) red[w] = v;
  __syncthreads();
  uint64_t r = Op::id();
  for (int i = 0; i < SC_T / 64; ++i) r = Op::f(r, red[i]);
  return r;
}

// exclusive block scan of one value per thread; returns exclusive prefix, *total = block total
template <typename Op>
__device__ __forceinline__ uint64_t block_excl_scan(uint64_t v, uint64_t* red, uint64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc = Op::f(inc, t);
  }
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint64_t carry = Op::id(), tot = Op::id();
  for (int i = 0; i < SC_T / 64; ++i) {
    if (i < w) carry = Op::f(carry, red[i]);
    tot = Op::f(tot, red[i]);
  }
  uint64_t exc = __shfl_up(inc, 1, 64);
  if (lane == 0) exc = Op::id();
  *total = tot;
  return Op::f(carry, exc);
}

template <typename Tin, typename Op>
__global__ __launch_bounds__(SC_T) void k_scan_reduce(const Tin* __restrict__ in, uint64_t n,
                                                      uint64_t* __restrict__ part) {
  __shared__ uint64_t red[SC_T / 64];
  const uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
  uint64_t acc = Op::id();
#pragma unroll
  for (int i = 0; i < SC_I; ++i) {
    uint64_t j = base + (uint64_t)i * SC_T + threadIdx.x;
    if (j < n) acc = Op::f(acc, (uint64_t)in[j]);
  }
  uint64_t r = block_reduce<Op>(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = r;
}

template <typename Tin, typename Op>
__global__ __launch_bounds__(SC_T) void k_scan_down(const Tin* in, uint64_t* out, uint64_t n,
                                                    const uint64_t* __restrict__ part_excl,
                                                    int write_total) {
  __shared__ uint64_t tile[SC_TILE];
  __shared__ uint64_t red[SC_T / 64];
  const uint64_t base = (uint64_t)blockIdx.x * SC_TILE;
  const uint64_t carry_in = part_excl ? part_excl[blockIdx.x] : Op::id();
#pragma unroll
  for (int i = 0; i < SC_I; ++i) {
    uint64_t j = base + (uint64_t)i * SC_T + threadIdx.x;
    tile[i * SC_T + threadIdx.x] = j < n ? (uint64_t)in[j] : Op::id();
  }
  __syncthreads();
  uint64_t loc[SC_I];
  uint64_t run = Op::id();
#pragma unroll
  for (int i = 0; i < SC_I; ++i) {
    loc[i] = run;
    run = Op::f(run, tile[threadIdx.x * SC_I + i]);
  }
  uint64_t total;
  uint64_t pre = block_excl_scan<Op>(run, red, &total);
  pre = Op::f(carry_in, pre);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SC_I; ++i) tile[threadIdx.x * SC_I + i] = Op::f(pre, loc[i]);
  __syncthreads();
#pragma unroll
  for (int i = 0; i < SC_I; ++i) {
    uint64_t j = base + (uint64_t)i * SC_T + threadIdx.x;
    if (j < n) out[j] = tile[i * SC_T + threadIdx.x];
  }
  if (write_total && blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) out[n] = Op::f(carry_in, total);
}

template <typename Tin, typename Op>
void scan_impl(uint64_t* scratch, const Tin* in, uint64_t* out, uint64_t n, bool write_total,
               hipStream_t s) {
  if (n == 0) {
    if (write_total) HK_HIP(hipMemsetAsync(out, 0, sizeof(uint64_t), s));
    return;
  }
  const uint64_t nb = ceil_div(n, SC_TILE);
  uint64_t* part = nullptr;
  if (nb > 1) {
    part = scratch;
    k_scan_reduce<Tin, Op><<<(unsigned)nb, SC_T, 0, s>>>(in, n, part);
    HK_HIP(hipGetLastError());
    scan_impl<uint64_t, Op>(scratch + nb + 1, part, part, nb, false, s);
  }
  k_scan_down<Tin, Op><<<(unsigned)nb, SC_T, 0, s>>>(in, out, n, part, write_total ? 1 : 0);
  HK_HIP(hipGetLastError());
}

uint64_t scan_scratch_words(uint64_t n) {
  uint64_t w = 16;
  while (n > SC_TILE) {
    n = ceil_div(n, SC_TILE);
    w += n + 1;
  }
  return w;
}

}  // namespace

void scan_exclusive_u64(SortWork& w, const uint64_t* in, uint64_t* out, uint64_t count,
                        bool write_total, hipStream_t s) {
  w.scan_tmp.ensure(scan_scratch_words(count) * 8);
  scan_impl<uint64_t, OpSum>(w.scan_tmp.as<uint64_t>(), in, out, count, write_total, s);
}
void scan_exclusive_u32_to_u64(SortWork& w, const uint32_t* in, uint64_t* out, uint64_t count,
                               bool write_total, hipStream_t s) {
  w.scan_tmp.ensure(scan_scratch_words(count) * 8);
  scan_impl<uint32_t, OpSum>(w.scan_tmp.as<uint64_t>(), in, out, count, write_total, s);
}
void scan_exclusive_max_u64(SortWork& w, const uint64_t* in, uint64_t* out, uint64_t count,
                            hipStream_t s) {
  w.scan_tmp.ensure(scan_scratch_words(count) * 8);
  scan_impl<uint64_t, OpMax>(w.scan_tmp.as<uint64_t>(), in, out, count, false, s);
}

// ========================================================== radix sort
namespace {

constexpr int HG_T = 512;
constexpr int HG_PER_BLOCK = HG_T * 16;

// digit histograms for `np` consecutive 8-bit digits starting at bit `lo`
__global__ __launch_bounds__(HG_T) void k_digit_hist(const uint64_t* __restrict__ keys, uint64_t n,
                                                     int lo, int np,
                                                     unsigned long long* __restrict__ hist, uint64_t kbias = 0) {
  __shared__ uint32_t h[8][256];
  for (int i = threadIdx.x; i < 8 * 256; i += HG_T) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t stride = (uint64_t)gridDim.x * HG_T * 2;
  for (uint64_t j = ((uint64_t)blockIdx.x * HG_T + threadIdx.x) * 2; j < n; j += stride) {
    uint64_t a, b;
    bool two = j + 1 < n;
    if (two) {
      const ulonglong2 kk = *reinterpret_cast<const ulonglong2*>(keys + j);
      a = kk.x - kbias;
      b = kk.y - kbias;
    } else {
      a = keys[j] - kbias;
      b = 0;
    }
    for (int p = 0; p < np; ++p) {
      const int sh = lo + 8 * p;
      atomicAdd(&h[p][(a >> sh) & 255], 1u);
      if (two) atomicAdd(&h[p][(b >> sh) & 255], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < np * 256; i += HG_T) {
    uint32_t c = (&h[0][0])[i];
    if (c) atomicAdd(&hist[i], (unsigned long long)c);
  }
}

// exclusive scan of each 256-bin histogram: one wave... one block of 256 threads per digit
__global__ __launch_bounds__(256) void k_hist_offsets(const uint64_t* __restrict__ hist,
                                                      uint64_t* __restrict__ offs) {
  __shared__ uint64_t red[4];
  const int p = blockIdx.x, d = threadIdx.x;
  const uint64_t v = hist[p * 256 + d];
  const int lane = d & 63, w = d >> 6;
  uint64_t inc = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint64_t carry = 0;
  for (int i = 0; i < w; ++i) carry += red[i];
  offs[p * 256 + d] = carry + inc - v;
}

constexpr int OS_T = 512;
constexpr int OS_I = 16;
constexpr int OS_TILE = OS_T * OS_I;   // 8192 pairs per tile (production variant)
constexpr uint64_t kSmallSort = 1ull << 24;   // below this, sorts use the 256-thread tile variant
constexpr uint64_t ST_VAL_MASK = (1ull << 46) - 1;
constexpr uint64_t ST_AGG = 1, ST_INC = 2;
constexpr uint32_t SPIN_LIMIT = 1u << 22;

__device__ __forceinline__ uint64_t st_pack(uint32_t epoch, uint64_t flag, uint64_t v) {
  return ((uint64_t)epoch << 48) | (flag << 46) | v;
}

template <typename V, int T, int I>
struct OsShared {
  union {
    uint64_t keys[T * I];
    V vals[T * I];
    uint16_t codes[T * I + kCodePad];   // text-keyed first pass: the tile's text codes
    struct {                            // ... radix 2^lb: codes packed MSB-first, and raw bytes
      uint32_t pk[(T * I + 64) / 4 + 4];
      uint8_t raw[T * I + 64];
    } ft;
  } stage;
  uint32_t prev0;                // text-keyed first pass: T'[tile base - 1]
  uint16_t L[256], LP[256];      // text-keyed first pass: keyed / dense code tables
  uint64_t SK[72];               // ... and the short suffixes' boundary keys
  uint32_t whist[T / 64][256];   // per-wave digit counts, then per-wave exclusive prefix
  uint32_t tstart[256];          // tile-local exclusive digit start
  uint64_t gbase[256];           // global destination base minus tstart
  uint32_t nhist[256];           // histogram of the NEXT pass's digit over this tile
  uint32_t wsum[4];
  uint32_t tile;
};

// Decoupled lookback for digit d of tile `tile`: sums predecessor counts until an inclusive
// prefix is found.  Up to LB_WIN predecessor granules are loaded at once (independent sc1 loads),
// so a chain of k not-yet-inclusive predecessors costs ~k/LB_WIN memory round trips, not k.
template <int LB_WIN>
__device__ __forceinline__ uint64_t lookback(const uint64_t* status, uint32_t tile, uint32_t d, uint32_t epoch,
                                             uint32_t* err) {
  uint64_t excl = 0;
  int64_t t = (int64_t)tile - 1;
  uint32_t spins = 0;
  while (t >= 0) {
    uint64_t g[LB_WIN];
#pragma unroll
    for (int i = 0; i < LB_WIN; ++i) g[i] = (t - i >= 0) ? ld_agent(status + (uint64_t)(t - i) * 256 + d) : 0;
    int consumed = 0;
    bool done = false, stalled = false;
#pragma unroll
    for (int i = 0; i < LB_WIN; ++i) {
      if (done || stalled || t - i < 0) continue;
      const uint64_t flag = (g[i] >> 46) & 3u;
      if ((uint32_t)(g[i] >> 48) != epoch || flag == 0) {
        stalled = true;
        continue;
      }
      excl += g[i] & ST_VAL_MASK;
      ++consumed;
      if (flag == ST_INC) done = true;
    }
    if (done) break;
    t -= consumed;
    if (stalled) {
      if (++spins > SPIN_LIMIT) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
  }
  return excl;
}

// MODE 0 = decoupled lookback (single kernel per pass).
// MODE 4 = downsweep of the reduce-then-scan pass: the tile's global digit offsets come from a
//          precomputed table tpre[tile * 256 + d] (no in-kernel hand-off); `goff` is that table.
// Diagnostic ablations (wrong results, in-bounds writes):
//   1 = no decoupled lookback (tile prefix taken as 0)
//   2 = no lookback and no LDS staging (scatter straight from registers)
//   3 = lookback with tile id = workgroup id (no tile counter)
// Order of work per tile: load keys -> wave ranking -> tile digit scan -> keys into LDS in sorted
// order -> value loads issued -> lookback (its latency overlaps the value loads) -> keys out ->
// values into LDS -> values out.
// FT: the pass reads the text instead of keys and builds each suffix's keyed key in registers from
// the tile's text codes staged in LDS (the first pass of the bucket build; values are positions).
template <typename V, int T, int I, int MODE, int LBW = 4, bool FT = false, int LB = 0>
__global__ __launch_bounds__(T, T >= 512 ? 4 : 3) void k_onesweep(
    const uint64_t* __restrict__ kin, const V* __restrict__ vin, uint64_t* __restrict__ kout,
    V* __restrict__ vout, uint64_t n, uint32_t shift, const uint64_t* __restrict__ goff,
    uint64_t* status, uint32_t* tile_counter, uint32_t epoch, uint32_t* err, int iota, int next_shift,
    unsigned long long* __restrict__ hpart, TextKeySrc src = TextKeySrc{}, uint64_t kbias = 0) {
  constexpr int W = T / 64;
  constexpr int TILE = T * I;
  constexpr int WSPAN = I * 64;
  __shared__ OsShared<V, T, I> sh;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;

  for (uint32_t i = tid; i < W * 256; i += T) (&sh.whist[0][0])[i] = 0;
  if (tid < 256) sh.nhist[tid] = 0;
  if (MODE != 3 && MODE != 4 && tid == 0) sh.tile = atomicAdd(tile_counter, 1u);
  __syncthreads();
  // MODE 3: tile id = workgroup id (relies on in-order workgroup dispatch; spins stay bounded)
  const uint32_t tile = (MODE == 3 || MODE == 4) ? blockIdx.x : sh.tile;
  const uint64_t tbase = (uint64_t)tile * TILE;
  const uint64_t wbase = tbase + (uint64_t)wv * WSPAN;

  uint64_t key[I];
  if constexpr (FT) {
    if (tid < 256) {
      sh.L[tid] = src.lutk[tid];
      sh.LP[tid] = src.lutp[tid];
    }
    if (tid < 72) sh.SK[tid] = src.skey[tid];
    __syncthreads();
    text_keys<T, I, LB>(key, src, n, tbase, wbase, lane, sh.stage.codes, sh.stage.ft.pk, sh.stage.ft.raw, &sh.prev0,
                    sh.L, sh.LP, sh.SK);
  } else {
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const uint64_t j = wbase + (uint64_t)k * 64 + lane;
      key[k] = j < n ? kin[j] : ~0ull;
    }
  }

  // ---- rank within the wave (stable: item-major, then lane).  The lanes sharing a digit come from
  // a per-wave match-mask table in the (still unused) staging area: each lane ORs its bit into its
  // digit's mask and reads the mask back; the group's lowest lane advances the wave's count and
  // clears the mask (LDS ops in wave order) — no per-bit ballots.
  uint64_t* const mtab = reinterpret_cast<uint64_t*>(&sh.stage);
  if (FT) __syncthreads();   // the staging area held the tile's text
  for (uint32_t i = tid; i < (uint32_t)W * 256; i += T) mtab[i] = 0;
  __syncthreads();
  uint64_t* const mt = mtab + wv * 256;
  uint32_t rk[I];
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const uint64_t j = wbase + (uint64_t)k * 64 + lane;
    const bool valid = j < n;
    const uint32_t d = (uint32_t)((key[k] - kbias) >> shift) & 255u;
    if (valid) __hip_atomic_fetch_or(mt + d, 1ull << lane, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint64_t m = __hip_atomic_load(mt + d, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    const uint32_t below = mbcnt(m);
    const uint32_t prior = sh.whist[wv][d];
    if (valid && below == 0) {
      __hip_atomic_store(mt + d, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      sh.whist[wv][d] = prior + (uint32_t)__popcll(m);
    }
    rk[k] = ((prior + below) & 0xFFFFu) | (d << 16);
  }
  __syncthreads();

  // ---- per-digit tile count, per-wave exclusive prefix, tile-local digit starts
  uint32_t tcount = 0;
  if (tid < 256) {
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < W; ++w) {
      const uint32_t c = sh.whist[w][tid];
      sh.whist[w][tid] = run;
      run += c;
    }
    tcount = run;
    uint32_t inc = run;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t t = __shfl_up(inc, o, 64);
      if (lane >= (uint32_t)o) inc += t;
    }
    if (lane == 63) sh.wsum[wv] = inc;
    sh.tstart[tid] = inc - run;  // wave-local exclusive, fixed below
  }
  __syncthreads();
  if (tid < 256) {
    uint32_t carry = 0;
    for (uint32_t w = 0; w < wv; ++w) carry += sh.wsum[w];
    sh.tstart[tid] += carry;
    if (MODE == 0 || MODE == 3) {  // publish this tile's counts as early as possible
      st_agent(status + (uint64_t)tile * 256 + tid, st_pack(epoch, tile == 0 ? ST_INC : ST_AGG, tcount));
    }
  }
  __syncthreads();

  if (MODE == 2) {  // ablation: scatter straight from registers
    if (tid < 256) {
      uint64_t go = goff[tid];
      if (go + TILE > n) go = n > (uint64_t)TILE ? n - TILE : 0;
      sh.gbase[tid] = go;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const uint64_t j = wbase + (uint64_t)k * 64 + lane;
      const uint32_t d = rk[k] >> 16;
      const uint32_t lr = sh.whist[wv][d] + (rk[k] & 0xFFFFu);
      if (j < n) {
        const uint64_t dst = sh.gbase[d] + lr;
        kout[dst] = key[k];
        vout[dst] = iota ? (V)j : vin[j];
      }
    }
    return;
  }

  // ---- keys into LDS in sorted order (rk becomes the tile-local rank)
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const uint64_t j = wbase + (uint64_t)k * 64 + lane;
    const uint32_t d = rk[k] >> 16;
    rk[k] = sh.tstart[d] + sh.whist[wv][d] + (rk[k] & 0xFFFFu);
    if (j < n) sh.stage.keys[rk[k]] = key[k];
  }
  // ---- value loads in flight across the lookback
  V val[I];
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const uint64_t j = wbase + (uint64_t)k * 64 + lane;
    val[k] = iota ? (V)j : (j < n ? vin[j] : (V)0);
  }
  const uint32_t tile_n = (uint32_t)((n - tbase) < (uint64_t)TILE ? (n - tbase) : TILE);
  if (next_shift >= 0) {
    // the next pass's digit histogram (the key multiset is the same in every pass); with 512
    // threads the upper 256 count it from the staged keys while the lower 256 look back
    __syncthreads();
    if (T < 512 || tid >= 256) {
      const uint32_t t0 = T < 512 ? tid : tid - 256, tn = T < 512 ? T : T - 256;
      for (uint32_t s2 = t0; s2 < tile_n; s2 += tn)
        atomicAdd(&sh.nhist[(uint32_t)((sh.stage.keys[s2] - kbias) >> next_shift) & 255u], 1u);
    }
  }
  if (tid < 256) {
    const uint32_t d = tid;
    uint64_t excl = 0;
    if ((MODE == 0 || MODE == 3) && tile > 0) {
      excl = lookback<LBW>(status, tile, d, epoch, err);
      st_agent(status + (uint64_t)tile * 256 + d, st_pack(epoch, ST_INC, excl + tcount));
    }
    uint64_t go = MODE == 4 ? goff[(uint64_t)tile * 256 + d] : goff[d];
    if ((MODE == 1 || MODE == 2) && go + TILE > n) go = n > (uint64_t)TILE ? n - TILE : 0;  // ablations in bounds
    sh.gbase[d] = go + excl - sh.tstart[d];
  }
  __syncthreads();
  if (next_shift >= 0 && tid < 256) {
    const uint32_t c = sh.nhist[tid];
    if (c) atomicAdd(&hpart[(uint64_t)(tile & 63) * 256 + tid], (unsigned long long)c);
  }

  uint32_t dg[(I + 3) / 4] = {};   // digits of the staged slots, 4 per register
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const uint32_t s = (uint32_t)i * T + tid;
    if (s < tile_n) {
      const uint64_t kk = sh.stage.keys[s];
      const uint32_t d = (uint32_t)((kk - kbias) >> shift) & 255u;
      dg[i >> 2] |= d << (8 * (i & 3));
      kout[sh.gbase[d] + s] = kk;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < I; ++k) {
    const uint64_t j = wbase + (uint64_t)k * 64 + lane;
    if (j < n) sh.stage.vals[rk[k]] = val[k];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < I; ++i) {
    const uint32_t s = (uint32_t)i * T + tid;
    if (s < tile_n) vout[sh.gbase[(dg[i >> 2] >> (8 * (i & 3))) & 255u] + s] = sh.stage.vals[s];
  }
}

// hist[d] = sum of the 64 partial histograms written by a pass
__global__ __launch_bounds__(256) void k_hist_reduce(const unsigned long long* __restrict__ hpart,
                                                     uint64_t* __restrict__ hist) {
  uint64_t a = 0;
  for (int p = 0; p < 64; ++p) a += hpart[p * 256 + threadIdx.x];
  hist[threadIdx.x] = a;
}

// bandwidth reference for the pass shape: read (key, value), write them back shifted by one tile
template <typename V>
__global__ __launch_bounds__(256) void k_copy_pairs(const uint64_t* __restrict__ kin, const V* __restrict__ vin,
                                                    uint64_t* __restrict__ kout, V* __restrict__ vout, uint64_t n) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256) {
    kout[j] = kin[j];
    vout[j] = vin[j];
  }
}

template <typename V>
__global__ void k_iota(V* v, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = (V)i;
}

}  // namespace

template <typename V>
void fill_iota(V* v, uint64_t n, hipStream_t s) {
  if (!n) return;
  unsigned g = (unsigned)std::min<uint64_t>(ceil_div(n, 256), 8192);
  k_iota<V><<<g, 256, 0, s>>>(v, n);
  HK_HIP(hipGetLastError());
}

template <typename V>
int radix_sort_pairs(SortWork& w, KernelTimer& tm, uint64_t* k[2], V* v[2], int in_slot, uint64_t n, int bit_lo,
                     int bit_hi, bool vals_iota, hipStream_t s, const uint64_t* d_hist0, const TextKeySrc* src,
                     uint64_t kbias) {
  w.passes_run = 0;
  w.passes_skipped = 0;
  int cur = in_slot;
  if (n == 0 || bit_hi <= bit_lo) {
    if (vals_iota) fill_iota<V>(v[cur], n, s);
    return cur;
  }
  const int np = (bit_hi - bit_lo + 7) / 8;
  if (np > 8) throw ApiError{-1, "radix_sort_pairs: more than 64 key bits"};
  // large sorts: 1024 (key passes) or 512 (text-keyed first pass) threads x 16 keys per tile;
  // small sorts (refinement of tied suffixes): 256 x 16, its own kernel symbol and timer name
  const bool small = n < kSmallSort;
  // large key passes: 1024 x 16 tiles (pass 2 of the 1 GiB build 6.79 -> 6.61 ms against 512 x 16); the
  // text-keyed first pass keeps 512-thread tiles (its key building is heavier per tile)
  const uint64_t tile_elems = small ? 256 * OS_I : OS_TILE;
  const uint64_t big_elems = 1024 * OS_I;
  const uint64_t tiles = ceil_div(n, tile_elems);
  if (tiles > 0xFFFFFFFFull) throw ApiError{-6, "radix_sort_pairs: too many tiles"};
  // the lookback status holds 256 granules per tile of the smallest tile this sort launches (1024 x 8 for
  // the key passes of u64 values)
  const uint64_t st_tiles = small || sizeof(V) == 4 ? tiles : ceil_div(n, (uint64_t)1024 * OS_I / 2);

  w.hist.ensure(9 * 256 * 8);
  w.offs.ensure(8 * 256 * 8);
  w.hpart.ensure(64 * 256 * 8);
  w.counters.ensure(64 * 4);
  w.err.ensure(16);
  if (st_tiles > w.status_tiles || !w.status.p) {
    w.status.ensure(st_tiles * 256 * 8);
    HK_HIP(hipMemsetAsync(w.status.p, 0, st_tiles * 256 * 8, s));
    w.status_tiles = st_tiles;
    w.epoch = 0;
  }
  HK_HIP(hipMemsetAsync(w.counters.p, 0, 64 * 4, s));
  HK_HIP(hipMemsetAsync(w.err.p, 0, 4, s));
  uint64_t* hist = w.hist.as<uint64_t>();

  // histogram of one digit straight from the keys in buffer `cur` (first digit, or after a skip)
  auto digit_hist = [&](int p) {
    HK_HIP(hipMemsetAsync(hist + p * 256, 0, 256 * 8, s));
    TimedLaunch t(tm, "radix_hist", (double)n * 8);
    unsigned g = (unsigned)std::min<uint64_t>(ceil_div(n, HG_PER_BLOCK), 2048);
    k_digit_hist<<<g, HG_T, 0, s>>>(k[cur], n, bit_lo + 8 * p, 1,
                                    reinterpret_cast<unsigned long long*>(hist + p * 256), kbias);
    HK_HIP(hipGetLastError());
  };
  if (src && (!d_hist0 || !vals_iota)) throw ApiError{-1, "radix_sort_pairs: text keys need hist0 and iota values"};
  // every digit's histogram and offsets from one read of the keys, then every pass back to back: small
  // sorts (refinement rounds) with no host round trip (no single-digit pass is skipped: a skipped small
  // pass saves less than the readback that finds it), large sorts with one read-back of all digits.
  // (The large passes used to count the next digit over their tile while looking back: on natural text's
  // skewed digits that cost ~0.36 ms a pass, English-like 15.7 -> 13.1 ms of passes for +0.8 ms here.)
  const bool upfront = !d_hist0;
  if (upfront) {
    HK_HIP(hipMemsetAsync(hist, 0, (uint64_t)np * 256 * 8, s));
    {
      TimedLaunch t(tm, "radix_hist", (double)n * 8);
      unsigned g = (unsigned)std::min<uint64_t>(ceil_div(n, HG_PER_BLOCK), 2048);
      k_digit_hist<<<g, HG_T, 0, s>>>(k[cur], n, bit_lo, np, reinterpret_cast<unsigned long long*>(hist), kbias);
      HK_HIP(hipGetLastError());
    }
    k_hist_offsets<<<np, 256, 0, s>>>(hist, w.offs.as<uint64_t>());
    HK_HIP(hipGetLastError());
    if (!small) {   // large sorts: one read-back finds every single-bucket (skipped) pass
      HK_HIP(hipMemcpyAsync(w.h_hist, hist, (uint64_t)np * 256 * 8, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
    }
  } else if (d_hist0) {
    HK_HIP(hipMemcpyAsync(hist, d_hist0, 256 * 8, hipMemcpyDeviceToDevice, s));
  } else {
    digit_hist(0);
  }

  bool iota_pending = vals_iota;
  for (int p = 0; p < np; ++p) {
    // the digit's histogram is complete here: offsets + single-bucket (skippable) check
    if (!upfront) {
      k_hist_offsets<<<1, 256, 0, s>>>(hist + p * 256, w.offs.as<uint64_t>() + p * 256);
      HK_HIP(hipGetLastError());
      HK_HIP(hipMemcpyAsync(w.h_hist + p * 256, hist + p * 256, 256 * 8, hipMemcpyDeviceToHost, s));
      HK_HIP(hipStreamSynchronize(s));
    }
    bool trivial = false;
    for (int d = 0; d < 256 && (!upfront || !small); ++d)
      if (w.h_hist[p * 256 + d] == n) trivial = true;
    const bool from_text = src && p == 0;   // builds the keys: never skipped
    if (from_text) trivial = false;
    const bool has_next = p + 1 < np && !upfront;   // upfront: no next-digit histogram in the pass
    if (trivial) {
      w.passes_skipped++;
      if (has_next) digit_hist(p + 1);
      continue;
    }
    if (w.epoch >= 0xFFFF) {
      HK_HIP(hipMemsetAsync(w.status.p, 0, w.status_tiles * 256 * 8, s));
      w.epoch = 0;
    }
    w.epoch++;
    if (has_next) HK_HIP(hipMemsetAsync(w.hpart.p, 0, 64 * 256 * 8, s));
    const int nxt = cur ^ 1;
    {
      // algorithmic bytes: read key + value, write key + value; the text-keyed pass reads 1 B of text
      // and no value
      const double ab = from_text ? (double)n * (1 + 8 + sizeof(V)) : (double)n * 2.0 * (8 + sizeof(V));
      TimedLaunch t(tm, from_text ? (small ? "radix_onesweep_text_small" : "radix_onesweep_text")
                                  : (small ? "radix_onesweep_small" : "radix_onesweep"), ab);
      if (from_text) {
        if (small)
          k_onesweep<V, 256, OS_I, 0, 4, true><<<(unsigned)tiles, 256, 0, s>>>(
              nullptr, nullptr, k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p), w.offs.as<uint64_t>() + p * 256,
              w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch, w.err.as<uint32_t>(), 1,
              has_next ? bit_lo + 8 * (p + 1) : -1, w.hpart.as<unsigned long long>(), *src);
        else if (src->g.lb == 2)   // DNA: packing fully unrolled
          k_onesweep<V, OS_T, OS_I, 0, 4, true, 2><<<(unsigned)tiles, OS_T, 0, s>>>(
              nullptr, nullptr, k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p), w.offs.as<uint64_t>() + p * 256,
              w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch, w.err.as<uint32_t>(), 1,
              has_next ? bit_lo + 8 * (p + 1) : -1, w.hpart.as<unsigned long long>(), *src);
        else
          k_onesweep<V, OS_T, OS_I, 0, 4, true><<<(unsigned)tiles, OS_T, 0, s>>>(
              nullptr, nullptr, k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p), w.offs.as<uint64_t>() + p * 256,
              w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch, w.err.as<uint32_t>(), 1,
              has_next ? bit_lo + 8 * (p + 1) : -1, w.hpart.as<unsigned long long>(), *src);
      } else if (small)
        k_onesweep<V, 256, OS_I, 0><<<(unsigned)tiles, 256, 0, s>>>(
            k[cur], iota_pending ? nullptr : v[cur], k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p),
            w.offs.as<uint64_t>() + p * 256, w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch,
            w.err.as<uint32_t>(), iota_pending ? 1 : 0, has_next ? bit_lo + 8 * (p + 1) : -1,
            w.hpart.as<unsigned long long>(), TextKeySrc{}, kbias);
      else if constexpr (sizeof(V) == 8)   // u64 values: 1024 x 8 tiles (1024 x 16 spills 52 B/lane)
        k_onesweep<V, 1024, OS_I / 2, 0><<<(unsigned)ceil_div(n, big_elems / 2), 1024, 0, s>>>(
            k[cur], iota_pending ? nullptr : v[cur], k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p),
            w.offs.as<uint64_t>() + p * 256, w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch,
            w.err.as<uint32_t>(), iota_pending ? 1 : 0, has_next ? bit_lo + 8 * (p + 1) : -1,
            w.hpart.as<unsigned long long>(), TextKeySrc{}, kbias);
      else
        k_onesweep<V, 1024, OS_I, 0><<<(unsigned)ceil_div(n, big_elems), 1024, 0, s>>>(
            k[cur], iota_pending ? nullptr : v[cur], k[nxt], v[nxt], n, (uint32_t)(bit_lo + 8 * p),
            w.offs.as<uint64_t>() + p * 256, w.status.as<uint64_t>(), w.counters.as<uint32_t>() + p, w.epoch,
            w.err.as<uint32_t>(), iota_pending ? 1 : 0, has_next ? bit_lo + 8 * (p + 1) : -1,
            w.hpart.as<unsigned long long>(), TextKeySrc{}, kbias);
      HK_HIP(hipGetLastError());
    }
    if (has_next) {
      k_hist_reduce<<<1, 256, 0, s>>>(w.hpart.as<unsigned long long>(), hist + (p + 1) * 256);
      HK_HIP(hipGetLastError());
    }
    iota_pending = false;
    cur = nxt;
    w.passes_run++;
  }
  if (iota_pending) fill_iota<V>(v[cur], n, s);
  w.herr.ensure(16);
  uint32_t* const he = static_cast<uint32_t*>(w.herr.p);
  HK_HIP(hipMemcpyAsync(he, w.err.p, 4, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (*he) throw ApiError{-7, "radix sort lookback exceeded its spin bound"};
  return cur;
}

// ---------------------------------------------------------------- diagnostics
// Times `reps` radix passes of variant (threads x items, mode) over n DNA-text keys (u32 values)
// plus a plain pair copy of the same bytes; used to decide where a pass spends its time.
template <int T, int I, int MODE, int LBW = 4>
static double time_variant(SortWork& w, uint64_t* k[2], uint32_t* v[2], uint64_t n, int reps, int bit_lo,
                           const uint64_t* pristine, hipStream_t s) {
  // every variant starts from the same keys: the ablations scramble the multiset, and an exact
  // variant's scatter is only in bounds when the keys match the digit offsets
  HK_HIP(hipMemcpyAsync(k[0], pristine, n * 8, hipMemcpyDeviceToDevice, s));
  fill_iota<uint32_t>(v[0], n, s);
  const uint64_t tiles = ceil_div(n, (uint64_t)T * I);
  w.status.ensure(tiles * 256 * 8);
  if (tiles > w.status_tiles) w.status_tiles = tiles;
  HK_HIP(hipMemsetAsync(w.status.p, 0, tiles * 256 * 8, s));
  w.counters.ensure(64 * 4);
  w.err.ensure(16);
  hipEvent_t a, b;
  HK_HIP(hipEventCreate(&a));
  HK_HIP(hipEventCreate(&b));
  float total = 0;
  for (int r = 0; r < reps + 1; ++r) {
    HK_HIP(hipMemsetAsync(w.counters.p, 0, 4, s));
    HK_HIP(hipEventRecord(a, s));
    k_onesweep<uint32_t, T, I, MODE, LBW><<<(unsigned)tiles, T, 0, s>>>(
        k[r & 1], v[r & 1], k[(r + 1) & 1], v[(r + 1) & 1], n, (uint32_t)(bit_lo + 8 * (r % 7)),
        w.offs.as<uint64_t>() + (r % 7) * 256, w.status.as<uint64_t>(), w.counters.as<uint32_t>(),
        (uint32_t)(r + 1), w.err.as<uint32_t>(), 0, -1, nullptr);
    HK_HIP(hipGetLastError());
    HK_HIP(hipEventRecord(b, s));
    HK_HIP(hipEventSynchronize(b));
    float ms = 0;
    HK_HIP(hipEventElapsedTime(&ms, a, b));
    if (r) total += ms;  // first launch is warm-up
  }
  (void)hipEventDestroy(a);
  (void)hipEventDestroy(b);
  w.status_tiles = 0;  // epochs restarted; force a clean status on the next real sort
  w.epoch = 0;
  return total / reps;
}

void debug_radix_bench(SortWork& w, uint64_t* k[2], uint32_t* v[2], uint64_t n, int bit_lo, int reps,
                       double* out, int nout, hipStream_t s) {
  // digit offsets of the real keys, so that every variant scatters inside the arrays
  w.hist.ensure(8 * 256 * 8);
  w.offs.ensure(8 * 256 * 8);
  HK_HIP(hipMemsetAsync(w.hist.p, 0, 8 * 256 * 8, s));
  k_digit_hist<<<2048, HG_T, 0, s>>>(k[0], n, bit_lo, 7, w.hist.as<unsigned long long>());
  k_hist_offsets<<<7, 256, 0, s>>>(w.hist.as<uint64_t>(), w.offs.as<uint64_t>());
  HK_HIP(hipGetLastError());
  DevBuf pristine;
  pristine.ensure(n * 8);
  HK_HIP(hipMemcpyAsync(pristine.p, k[0], n * 8, hipMemcpyDeviceToDevice, s));
  const uint64_t* pk = pristine.as<uint64_t>();
  double r[8] = {0};
  r[0] = time_variant<512, 16, 0>(w, k, v, n, reps, bit_lo, pk, s);
  r[1] = time_variant<512, 16, 1>(w, k, v, n, reps, bit_lo, pk, s);
  r[2] = time_variant<1024, 16, 0, 4>(w, k, v, n, reps, bit_lo, pk, s);
  r[3] = time_variant<1024, 12, 0, 4>(w, k, v, n, reps, bit_lo, pk, s);
  r[4] = time_variant<512, 16, 0, 4>(w, k, v, n, reps, bit_lo, pk, s);
  r[5] = time_variant<1024, 16, 1, 4>(w, k, v, n, reps, bit_lo, pk, s);
  {
    hipEvent_t a, b;
    HK_HIP(hipEventCreate(&a));
    HK_HIP(hipEventCreate(&b));
    float total = 0;
    for (int q = 0; q < reps + 1; ++q) {
      HK_HIP(hipEventRecord(a, s));
      k_copy_pairs<uint32_t><<<8192, 256, 0, s>>>(k[q & 1], v[q & 1], k[(q + 1) & 1], v[(q + 1) & 1], n);
      HK_HIP(hipEventRecord(b, s));
      HK_HIP(hipEventSynchronize(b));
      float ms = 0;
      HK_HIP(hipEventElapsedTime(&ms, a, b));
      if (q) total += ms;
    }
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    r[6] = total / reps;
  }
  uint32_t herr = 0;
  HK_HIP(hipMemcpyAsync(&herr, w.err.p, 4, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  r[7] = herr;
  for (int i = 0; i < nout && i < 8; ++i) out[i] = r[i];
}

template int radix_sort_pairs<uint32_t>(SortWork&, KernelTimer&, uint64_t* k[2], uint32_t* v[2],
                                        int, uint64_t, int, int, bool, hipStream_t, const uint64_t*,
                                        const TextKeySrc*, uint64_t);
template int radix_sort_pairs<uint64_t>(SortWork&, KernelTimer&, uint64_t* k[2], uint64_t* v[2],
                                        int, uint64_t, int, int, bool, hipStream_t, const uint64_t*,
                                        const TextKeySrc*, uint64_t);
template void fill_iota<uint32_t>(uint32_t*, uint64_t, hipStream_t);
template void fill_iota<uint64_t>(uint64_t*, uint64_t, hipStream_t);

}  // namespace hk
