// hk_sa.hip — suffix array by GPU prefix doubling, BWT gather, alphabet/C array.
//
// Semantics follow the reference exactly (SURVEY.md §8 "Exact semantics"):
//   * SA of T' in Python str order (csa/suffix_array.py:131-134): symbols compare by byte
//     value, end-of-text is smaller than every symbol ('$' is an ordinary byte).
//   * BWT[j] = T'[SA[j]-1], wrapping to T'[n-1] (csa/bwt.py:3-13).
//   * C[c] = #{symbols < c} (utils/utils.py:16-24).
//
// Algorithm (MI355X-first, not a translation of anything in the reference):
//   1. pack the first q symbols of every suffix into a u64 key (b bits per dense code,
//      code 0 = end of text), so one LSD radix sort orders suffixes by q symbols;
//   2. head flags + max-scan give every suffix its group start ("h-rank") in the ISA;
//      singleton groups are final and leave the active list;
//   3. each doubling round sorts the active suffixes by (group, ISA[p+h]) and splits groups
//      until none remain — the classic prefix-doubling invariant, restricted to active suffixes.

#include "hk_index.hpp"

namespace hk {
namespace {

// --------------------------------------------------------------- helpers
constexpr int GR_T = 256;
constexpr int GR_I = 16;
constexpr int GR_TILE = GR_T * GR_I;

__device__ __forceinline__ uint64_t blk_excl_sum(uint64_t v, uint64_t* red, uint64_t* total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = wave_incl_sum<uint64_t>(v);
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint64_t carry = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < GR_T / 64; ++i) {
    if (i < w) carry += red[i];
    tot += red[i];
  }
  *total = tot;
  __syncthreads();
  return carry + inc - v;
}

__device__ __forceinline__ uint64_t blk_excl_max(uint64_t v, uint64_t* red) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t inc = wave_incl_max<uint64_t>(v);
  if (lane == 63) red[w] = inc;
  __syncthreads();
  uint64_t carry = 0;
#pragma unroll
  for (int i = 0; i < GR_T / 64; ++i)
    if (i < w) carry = carry > red[i] ? carry : red[i];
  uint64_t exc = __shfl_up(inc, 1, 64);
  if (lane == 0) exc = 0;
  __syncthreads();
  return carry > exc ? carry : exc;
}

// ---------------------------------------------------------- kernels
__global__ __launch_bounds__(256) void k_byte_hist(const uint8_t* __restrict__ t, uint64_t n,
                                                   unsigned long long* __restrict__ hist) {
  __shared__ uint32_t h[4][256];
  for (int i = threadIdx.x; i < 4 * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  uint32_t* mine = h[(threadIdx.x >> 6) & 3];
  const uint64_t nv = n / 16;
  const uint4* t4 = reinterpret_cast<const uint4*>(t);
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < nv; i += (uint64_t)gridDim.x * 256) {
    const uint4 v = t4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int b = 0; b < 4; ++b) atomicAdd(&mine[(w[q] >> (8 * b)) & 255], 1u);
  }
  if (blockIdx.x == 0)
    for (uint64_t i = nv * 16 + threadIdx.x; i < n; i += 256) atomicAdd(&mine[t[i]], 1u);
  __syncthreads();
  const uint32_t c = h[0][threadIdx.x] + h[1][threadIdx.x] + h[2][threadIdx.x] + h[3][threadIdx.x];
  if (c) atomicAdd(&hist[threadIdx.x], (unsigned long long)c);
}

// key[i-lo] = code(T[i]) .. code(T[i+q-1]) packed MSB-first, b bits each, code 0 past the end
constexpr int PK_TILE = 4096;
__global__ __launch_bounds__(256) void k_pack_keys(const uint8_t* __restrict__ t, uint64_t n,
                                                   uint64_t lo, uint64_t count,
                                                   const uint8_t* __restrict__ lut, int b, int q,
                                                   uint64_t* __restrict__ keys) {
  __shared__ uint8_t c[PK_TILE + 64];
  __shared__ uint8_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const uint64_t base = lo + (uint64_t)blockIdx.x * PK_TILE;
  for (int i = threadIdx.x; i < PK_TILE + q; i += 256) {
    const uint64_t p = base + i;
    c[i] = p < n ? L[t[p]] : 0;
  }
  __syncthreads();
  const uint64_t end = lo + count;
#pragma unroll 4
  for (int k = 0; k < PK_TILE / 256; ++k) {
    const int off = k * 256 + threadIdx.x;
    const uint64_t p = base + off;
    if (p < end) {
      uint64_t key = 0;
      for (int j = 0; j < q; ++j) key = (key << b) | c[off + j];
      keys[p - lo] = key;
    }
  }
}

// per tile: index (or J value) of the last group head, number of suffixes in non-singleton groups
template <bool HAS_J>
__global__ __launch_bounds__(GR_T) void k_group_stats(const uint64_t* __restrict__ keys,
                                                      const uint32_t* __restrict__ J, uint64_t A,
                                                      uint64_t* __restrict__ tile_last,
                                                      uint32_t* __restrict__ tile_act) {
  __shared__ uint64_t red[GR_T / 64];
  const uint64_t base = (uint64_t)blockIdx.x * GR_TILE + (uint64_t)threadIdx.x * GR_I;
  int64_t last = -1;
  uint32_t act = 0;
  if (base < A) {
    uint64_t prev = base > 0 ? keys[base - 1] : 0;
    uint64_t cur = keys[base];
#pragma unroll
    for (int i = 0; i < GR_I; ++i) {
      const uint64_t j = base + i;
      if (j >= A) break;
      const uint64_t nxt = j + 1 < A ? keys[j + 1] : 0;
      const bool h = (j == 0) || cur != prev;
      const bool hn = (j + 1 >= A) || nxt != cur;
      if (h) last = (int64_t)j;
      act += (h && hn) ? 0u : 1u;
      prev = cur;
      cur = nxt;
    }
  }
  // block max of `last` (as last+1, 0 = none) and sum of act
  uint64_t lv = (uint64_t)(last + 1);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    uint64_t t = __shfl_xor(lv, o, 64);
    lv = lv > t ? lv : t;
    act += __shfl_xor(act, o, 64);
  }
  __shared__ uint32_t redc[GR_T / 64];
  if ((threadIdx.x & 63) == 0) {
    red[threadIdx.x >> 6] = lv;
    redc[threadIdx.x >> 6] = act;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t m = 0;
    uint32_t c = 0;
    for (int i = 0; i < GR_T / 64; ++i) {
      m = m > red[i] ? m : red[i];
      c += redc[i];
    }
    uint64_t v = 0;
    if (m) v = HAS_J ? (uint64_t)J[m - 1] : (m - 1);
    tile_last[blockIdx.x] = v;
    tile_act[blockIdx.x] = c;
  }
}

// assign group starts, update ISA (and SA for doubling rounds), compact the active list
template <bool HAS_J>
__global__ __launch_bounds__(GR_T) void k_group_apply(
    const uint64_t* __restrict__ keys, const uint32_t* __restrict__ P, const uint32_t* __restrict__ J,
    uint64_t A, const uint64_t* __restrict__ carry_last, const uint64_t* __restrict__ act_off,
    uint32_t* __restrict__ isa, uint32_t* __restrict__ sa, uint32_t* __restrict__ oP,
    uint32_t* __restrict__ oJ, uint32_t* __restrict__ oG) {
  __shared__ uint64_t red[GR_T / 64];
  const uint64_t base = (uint64_t)blockIdx.x * GR_TILE + (uint64_t)threadIdx.x * GR_I;
  uint32_t hmask = 0, amask = 0;
  uint64_t tmax = 0;
  if (base < A) {
    uint64_t prev = base > 0 ? keys[base - 1] : 0;
    uint64_t cur = keys[base];
#pragma unroll
    for (int i = 0; i < GR_I; ++i) {
      const uint64_t j = base + i;
      if (j >= A) break;
      const uint64_t nxt = j + 1 < A ? keys[j + 1] : 0;
      const bool h = (j == 0) || cur != prev;
      const bool hn = (j + 1 >= A) || nxt != cur;
      if (h) {
        hmask |= 1u << i;
        tmax = HAS_J ? (uint64_t)J[j] : j;
      }
      if (!(h && hn)) amask |= 1u << i;
      prev = cur;
      cur = nxt;
    }
  }
  const uint64_t carry = carry_last[blockIdx.x];
  uint64_t gpre = blk_excl_max(tmax, red);
  gpre = gpre > carry ? gpre : carry;
  uint64_t tot;
  uint64_t o = blk_excl_sum((uint64_t)__popc(amask), red, &tot) + act_off[blockIdx.x];
  uint64_t g = gpre;
#pragma unroll
  for (int i = 0; i < GR_I; ++i) {
    const uint64_t j = base + i;
    if (j >= A) break;
    const uint32_t jv = HAS_J ? J[j] : (uint32_t)j;
    if (hmask & (1u << i)) g = jv;
    const uint32_t p = P[j];
    isa[p] = (uint32_t)g;
    if (HAS_J) sa[jv] = p;
    if (amask & (1u << i)) {
      oP[o] = p;
      oJ[o] = jv;
      oG[o] = (uint32_t)g;
      ++o;
    }
  }
}

// doubling round keys: (group start, ISA[p+h]+1 or 0 past the end), value = position
__global__ __launch_bounds__(256) void k_pair_keys(const uint32_t* __restrict__ P,
                                                   const uint32_t* __restrict__ G, uint64_t A,
                                                   const uint32_t* __restrict__ isa, uint64_t n,
                                                   uint64_t h, uint64_t* __restrict__ keys,
                                                   uint32_t* __restrict__ vals) {
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const uint32_t p = P[a];
    const uint64_t q = (uint64_t)p + h;
    const uint64_t s = q < n ? (uint64_t)isa[q] + 1 : 0;
    keys[a] = ((uint64_t)G[a] << 32) | s;
    vals[a] = p;
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

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

// one grouping step over A sorted keys. Returns the new active count.
uint64_t group_step(Index& ix, const uint64_t* keys, const uint32_t* P, const uint32_t* J, uint64_t A,
                    uint32_t* oP, uint32_t* oJ, uint32_t* oG) {
  hipStream_t s = ix.stream;
  const uint64_t nt = ceil_div(A, GR_TILE);
  ix.tile_a.ensure((nt + 1) * 8);
  ix.tile_b.ensure((nt + 1) * 4);
  ix.tile_c.ensure((nt + 1) * 8);
  ix.tile_d.ensure((nt + 2) * 8);
  uint64_t* tl = ix.tile_a.as<uint64_t>();
  uint32_t* ta = ix.tile_b.as<uint32_t>();
  uint64_t* cl = ix.tile_c.as<uint64_t>();
  uint64_t* ao = ix.tile_d.as<uint64_t>();
  {
    TimedLaunch t(ix.timer, "sa_group_stats", (double)A * 8);
    if (J) k_group_stats<true><<<(unsigned)nt, GR_T, 0, s>>>(keys, J, A, tl, ta);
    else k_group_stats<false><<<(unsigned)nt, GR_T, 0, s>>>(keys, J, A, tl, ta);
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_max_u64(ix.sw, tl, cl, nt, s);
  scan_exclusive_u32_to_u64(ix.sw, ta, ao, nt, true, s);
  {
    TimedLaunch t(ix.timer, "sa_group_apply", (double)A * (8 + 4 + 4 + 4 + (J ? 8 : 0)));
    if (J)
      k_group_apply<true><<<(unsigned)nt, GR_T, 0, s>>>(keys, P, J, A, cl, ao, ix.isa.as<uint32_t>(),
                                                        ix.sa.as<uint32_t>(), oP, oJ, oG);
    else
      k_group_apply<false><<<(unsigned)nt, GR_T, 0, s>>>(keys, P, J, A, cl, ao, ix.isa.as<uint32_t>(),
                                                         ix.sa.as<uint32_t>(), oP, oJ, oG);
    HK_HIP(hipGetLastError());
  }
  uint64_t na = 0;
  HK_HIP(hipMemcpyAsync(&na, ao + nt, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  return na;
}

}  // namespace

void pack_keys(const uint8_t* d_text, uint64_t n, uint64_t lo, uint64_t count, const uint8_t* d_lut,
               int b, int q, uint64_t* d_keys, hipStream_t s) {
  if (!count) return;
  const uint64_t g = ceil_div(count, PK_TILE);
  k_pack_keys<<<(unsigned)g, 256, 0, s>>>(d_text, n, lo, count, d_lut, b, q, d_keys);
  HK_HIP(hipGetLastError());
}

void synth_text(uint8_t* d_text, uint64_t n, const uint8_t* alphabet, int sigma, uint64_t seed,
                uint8_t terminator, hipStream_t s) {
  Alpha256 al{};
  for (int i = 0; i < sigma; ++i) al.s[i] = alphabet[i];
  k_synth<<<grid_for(n), 256, 0, s>>>(d_text, n, al, sigma, seed, terminator);
  HK_HIP(hipGetLastError());
}

void compute_alphabet(Index& ix) {
  if (ix.have_alpha) return;
  hipStream_t s = ix.stream;
  ix.small.ensure(4096);
  HK_HIP(hipMemsetAsync(ix.small.p, 0, 256 * 8, s));
  {
    TimedLaunch t(ix.timer, "byte_hist", (double)ix.n);
    k_byte_hist<<<grid_for(ix.n / 16 + 1, 256, 2048), 256, 0, s>>>(ix.text.as<uint8_t>(), ix.n,
                                                                   ix.small.as<unsigned long long>());
    HK_HIP(hipGetLastError());
  }
  HK_HIP(hipMemcpyAsync(ix.byte_hist, ix.small.p, 256 * 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
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

void build_sa(Index& ix) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  if (n >= 0xFFFFFFFFull) throw ApiError{-6, "single-GPU build supports n < 2^32 - 1"};
  compute_alphabet(ix);
  ix.info.assign(4, 0);
  ix.sharded = false;
  ix.sa_pos64 = false;
  ix.sa.ensure(n * 4 + 16);
  if (n <= 1) {
    HK_HIP(hipMemsetAsync(ix.sa.p, 0, 4, s));
    HK_HIP(hipStreamSynchronize(s));
    ix.have_sa = true;
    return;
  }
  // dense codes 1..sigma, 0 = end of text
  int b = 1;
  while ((1 << b) < ix.sigma + 1) ++b;
  int q = 64 / b;
  uint8_t lut[256];
  for (int c = 0; c < 256; ++c) lut[c] = ix.code_of[c] < 0 ? 0 : (uint8_t)(ix.code_of[c] + 1);
  ix.small.ensure(4096);
  uint8_t* d_lut = ix.small.as<uint8_t>() + 2048;
  HK_HIP(hipMemcpyAsync(d_lut, lut, 256, hipMemcpyHostToDevice, s));

  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(n * 8 + 16);
    ix.vals[i].ensure(n * 4 + 16);
  }
  ix.isa.ensure(n * 4 + 16);
  {
    TimedLaunch t(ix.timer, "sa_pack_keys", (double)n * 9);
    pack_keys(ix.text.as<uint8_t>(), n, 0, n, d_lut, b, q, ix.keys[0].as<uint64_t>(), s);
  }
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  uint32_t* vp[2] = {ix.vals[0].as<uint32_t>(), ix.vals[1].as<uint32_t>()};
  int slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, n, 0, q * b, true, s);
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  // the sorted values are the SA candidate order: adopt that buffer as SA
  std::swap(ix.sa, ix.vals[slot]);
  ix.vals[slot].ensure(n * 4 + 16);
  vp[slot] = ix.vals[slot].as<uint32_t>();
  for (int i = 0; i < 2; ++i)
    for (int k = 0; k < 3; ++k) ix.act[i][k].ensure(n * 4 + 16);

  uint64_t A = group_step(ix, kp[slot], ix.sa.as<uint32_t>(), nullptr, n, ix.act[0][0].as<uint32_t>(),
                          ix.act[0][1].as<uint32_t>(), ix.act[0][2].as<uint32_t>());
  ix.info.push_back(A);
  uint64_t h = (uint64_t)q;
  int rounds = 0;
  while (A > 0) {
    if (++rounds > 64) throw ApiError{-7, "prefix doubling did not converge"};
    uint32_t* P = ix.act[0][0].as<uint32_t>();
    uint32_t* J = ix.act[0][1].as<uint32_t>();
    uint32_t* G = ix.act[0][2].as<uint32_t>();
    {
      TimedLaunch t(ix.timer, "sa_pair_keys", (double)A * (4 + 4 + 4 + 8 + 4));
      k_pair_keys<<<grid_for(A), 256, 0, s>>>(P, G, A, ix.isa.as<uint32_t>(), n, h, kp[0], vp[0]);
      HK_HIP(hipGetLastError());
    }
    slot = radix_sort_pairs<uint32_t>(ix.sw, ix.timer, kp, vp, 0, A, 0, 64, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    A = group_step(ix, kp[slot], vp[slot], J, A, ix.act[1][0].as<uint32_t>(), ix.act[1][1].as<uint32_t>(),
                   ix.act[1][2].as<uint32_t>());
    ix.info.push_back(A);
    for (int k = 0; k < 3; ++k) std::swap(ix.act[0][k], ix.act[1][k]);
    h *= 2;
  }
  ix.info[2] = (uint64_t)rounds;
  ix.info[3] = (uint64_t)q;
  ix.have_sa = true;
}

void build_bwt(Index& ix) {
  if (!ix.have_sa) throw ApiError{-3, "build_bwt: suffix array not built"};
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
  }
  ix.isa.release();
  ix.tile_a.release();
  ix.tile_b.release();
  ix.tile_c.release();
  ix.tile_d.release();
  ix.sw.status.release();
  ix.sw.status_tiles = 0;
  ix.sw.scan_tmp.release();
}

}  // namespace hk
