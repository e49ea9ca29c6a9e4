// hk_shard.hip — suffix-array construction sharded over the GPUs of one node.
//
// Every rank holds the same T' (≤ 288 GB HBM each makes replication cheap) and owns one
// contiguous range of the FINAL suffix array:
//   1. each rank histograms the 14-bit key prefix of its block of positions; one RCCL
//      all-reduce gives the global histogram, so all ranks derive identical splitters
//      (bucket ranges) and their slice bounds [lo, hi) without further exchange;
//   2. each rank scans all of T' and keeps the suffixes whose bucket it owns (pack + select,
//      reading T' once, writing only its ~n/N pairs);
//   3. it radix-sorts its slice by the q-symbol key and refines tied groups by sorting on
//      (dense group ordinal, next symbols of the suffix) read straight from the replicated
//      text — no rank exchange is needed because every comparison stays inside one slice;
//   4. an RCCL all-gather of the slice bounds merges the per-rank ranges into the global SA
//      layout (and checks that they tile [0, n)).
// Positions are 64-bit when n ≥ 2^32 (the 4 GiB + 1 config).

#include <rccl/rccl.h>

#include <cstring>

#include "hk_index.hpp"

namespace hk {
namespace {

constexpr int SH_BUCKET_BITS = 14;
constexpr int SH_BUCKETS = 1 << SH_BUCKET_BITS;
constexpr int PS_TILE = 4096;

struct ShardComm {
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = -1;
  uint8_t id[128];
};

// keys are built from LDS-staged dense codes (see k_pack_keys in hk_sa.hip)
__device__ __forceinline__ uint64_t key_at(const uint8_t* c, int off, int b, int q) {
  uint64_t key = 0;
  for (int j = 0; j < q; ++j) key = (key << b) | c[off + j];
  return key;
}

__global__ __launch_bounds__(256) void k_shard_hist(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                    uint64_t hi, const uint8_t* __restrict__ lut, int b, int q,
                                                    int bsh, unsigned long long* __restrict__ hist) {
  __shared__ uint32_t H[SH_BUCKETS];
  __shared__ uint8_t c[PS_TILE + 64];
  __shared__ uint8_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256) H[i] = 0;
  __syncthreads();
  for (uint64_t base = lo + (uint64_t)blockIdx.x * PS_TILE; base < hi; base += (uint64_t)gridDim.x * PS_TILE) {
    for (int i = threadIdx.x; i < PS_TILE + q; i += 256) {
      const uint64_t p = base + i;
      c[i] = p < n ? L[t[p]] : 0;
    }
    __syncthreads();
    for (int k = 0; k < PS_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      if (base + off < hi) atomicAdd(&H[key_at(c, off, b, q) >> bsh], 1u);
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256)
    if (H[i]) atomicAdd(&hist[i], (unsigned long long)H[i]);
}

template <typename V>
__global__ __launch_bounds__(256) void k_pack_select(const uint8_t* __restrict__ t, uint64_t n,
                                                     const uint8_t* __restrict__ lut, int b, int q, int bsh,
                                                     uint32_t blo, uint32_t bhi, uint64_t* __restrict__ keys,
                                                     V* __restrict__ vals, unsigned long long* counter) {
  __shared__ uint8_t c[PS_TILE + 64];
  __shared__ uint8_t L[256];
  __shared__ uint32_t red[4];
  __shared__ unsigned long long gbase;
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t base = (uint64_t)blockIdx.x * PS_TILE; base < n; base += (uint64_t)gridDim.x * PS_TILE) {
    for (int i = threadIdx.x; i < PS_TILE + q; i += 256) {
      const uint64_t p = base + i;
      c[i] = p < n ? L[t[p]] : 0;
    }
    __syncthreads();
    uint64_t kk[PS_TILE / 256];
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < PS_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      kk[k] = key_at(c, off, b, q);
      const uint32_t bk = (uint32_t)(kk[k] >> bsh);
      if (base + off < n && bk >= blo && bk < bhi) sel |= 1u << k;
    }
    const uint32_t cnt = __popc(sel);
    const uint32_t inc = wave_incl_sum<uint32_t>(cnt);
    if (lane == 63) red[w] = inc;
    __syncthreads();
    uint32_t carry = 0, tot = 0;
    for (int i = 0; i < 4; ++i) {
      if (i < w) carry += red[i];
      tot += red[i];
    }
    if (threadIdx.x == 0) gbase = tot ? atomicAdd(counter, (unsigned long long)tot) : 0ull;
    __syncthreads();
    uint64_t o = gbase + carry + inc - cnt;
#pragma unroll
    for (int k = 0; k < PS_TILE / 256; ++k)
      if (sel & (1u << k)) {
        keys[o] = kk[k];
        vals[o] = (V)(base + k * 256 + threadIdx.x);
        ++o;
      }
    __syncthreads();
  }
}

constexpr int RF_T = 256, RF_I = 16, RF_TILE = RF_T * RF_I;

// per tile: suffixes in tied groups, and heads of tied groups
__global__ __launch_bounds__(RF_T) void k_refine_stats(const uint64_t* __restrict__ keys, uint64_t A,
                                                       uint32_t* __restrict__ tact, uint32_t* __restrict__ thead) {
  const uint64_t base = (uint64_t)blockIdx.x * RF_TILE + (uint64_t)threadIdx.x * RF_I;
  uint32_t act = 0, hd = 0;
  if (base < A) {
    uint64_t prev = base > 0 ? keys[base - 1] : 0, cur = keys[base];
    for (int i = 0; i < RF_I; ++i) {
      const uint64_t j = base + i;
      if (j >= A) break;
      const uint64_t nxt = j + 1 < A ? keys[j + 1] : 0;
      const bool h = j == 0 || cur != prev;
      const bool hn = j + 1 >= A || nxt != cur;
      if (!(h && hn)) {
        ++act;
        if (h) ++hd;
      }
      prev = cur;
      cur = nxt;
    }
  }
  act = wave_sum<uint32_t>(act);
  hd = wave_sum<uint32_t>(hd);
  __shared__ uint32_t ra[4], rh[4];
  if ((threadIdx.x & 63) == 0) {
    ra[threadIdx.x >> 6] = act;
    rh[threadIdx.x >> 6] = hd;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    tact[blockIdx.x] = ra[0] + ra[1] + ra[2] + ra[3];
    thead[blockIdx.x] = rh[0] + rh[1] + rh[2] + rh[3];
  }
}

// write the slice entry of every suffix; compact tied suffixes with their group ordinal
template <typename V>
__global__ __launch_bounds__(RF_T) void k_refine_apply(const uint64_t* __restrict__ keys, const V* __restrict__ P,
                                                       const uint32_t* __restrict__ J, uint64_t A,
                                                       const uint64_t* __restrict__ act_off,
                                                       const uint64_t* __restrict__ head_off, V* __restrict__ sa,
                                                       V* __restrict__ oP, uint32_t* __restrict__ oJ,
                                                       uint32_t* __restrict__ oG) {
  __shared__ uint32_t ra[4], rh[4];
  const uint64_t base = (uint64_t)blockIdx.x * RF_TILE + (uint64_t)threadIdx.x * RF_I;
  uint32_t hmask = 0, amask = 0;
  if (base < A) {
    uint64_t prev = base > 0 ? keys[base - 1] : 0, cur = keys[base];
    for (int i = 0; i < RF_I; ++i) {
      const uint64_t j = base + i;
      if (j >= A) break;
      const uint64_t nxt = j + 1 < A ? keys[j + 1] : 0;
      const bool h = j == 0 || cur != prev;
      const bool hn = j + 1 >= A || nxt != cur;
      if (!(h && hn)) {
        amask |= 1u << i;
        if (h) hmask |= 1u << i;
      }
      prev = cur;
      cur = nxt;
    }
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t ca = __popc(amask), ch = __popc(hmask);
  const uint32_t ia = wave_incl_sum<uint32_t>(ca), ih = wave_incl_sum<uint32_t>(ch);
  if (lane == 63) {
    ra[w] = ia;
    rh[w] = ih;
  }
  __syncthreads();
  uint64_t oa = act_off[blockIdx.x], oh = head_off[blockIdx.x];
  for (int i = 0; i < w; ++i) {
    oa += ra[i];
    oh += rh[i];
  }
  oa += ia - ca;
  oh += ih - ch;
  // group ordinal of a tied suffix = (# tied-group heads up to and including its own head) - 1
  uint64_t g = oh;  // heads before this thread's first item
  for (int i = 0; i < RF_I; ++i) {
    const uint64_t j = base + i;
    if (j >= A) break;
    const uint32_t jv = J ? J[j] : (uint32_t)j;
    const V p = P[j];
    sa[jv] = p;
    if (amask & (1u << i)) {
      if (hmask & (1u << i)) ++g;
      oP[oa] = p;
      oJ[oa] = jv;
      oG[oa] = (uint32_t)(g - 1);
      ++oa;
    }
  }
}

// refinement key: (group ordinal << (64-gbits)) | next qn symbols of the suffix from offset h
template <typename V>
__global__ __launch_bounds__(256) void k_refine_keys(const V* __restrict__ P, const uint32_t* __restrict__ G,
                                                     uint64_t A, const uint8_t* __restrict__ t, uint64_t n,
                                                     const uint8_t* __restrict__ lut, int b, int qn, int gbits,
                                                     uint64_t h, uint64_t* __restrict__ keys, V* __restrict__ vals) {
  __shared__ uint8_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  for (uint64_t a = (uint64_t)blockIdx.x * 256 + threadIdx.x; a < A; a += (uint64_t)gridDim.x * 256) {
    const V p = P[a];
    const uint64_t s = (uint64_t)p + h;
    uint64_t chunk = 0;
    for (int j = 0; j < qn; ++j) {
      const uint64_t x = s + j;
      chunk = (chunk << b) | (x < n ? L[t[x]] : 0u);
    }
    keys[a] = gbits ? (((uint64_t)G[a] << (64 - gbits)) | chunk) : chunk;
    vals[a] = p;
  }
}

template <typename V>
__global__ void k_widen(const V* __restrict__ in, uint64_t* __restrict__ out, uint64_t m) {
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < m; i += (uint64_t)gridDim.x * 256)
    out[i] = (uint64_t)in[i];
}

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

void ncclcheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw ApiError{-8, std::string(what) + ": " + ncclGetErrorString(r)};
}

struct KeyGeom {
  int b, q, bsh;
  uint8_t lut[256];
};

KeyGeom geometry(Index& ix) {
  compute_alphabet(ix);
  KeyGeom g{};
  g.b = 1;
  while ((1 << g.b) < ix.sigma + 1) ++g.b;
  g.q = 64 / g.b;
  g.bsh = g.q * g.b - SH_BUCKET_BITS;
  if (g.bsh < 0) g.bsh = 0;
  for (int c = 0; c < 256; ++c) g.lut[c] = ix.code_of[c] < 0 ? 0 : (uint8_t)(ix.code_of[c] + 1);
  return g;
}

template <typename V>
void refine_slice(Index& ix, const KeyGeom& kg, const uint8_t* d_lut, uint64_t m) {
  hipStream_t s = ix.stream;
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  V* vp[2] = {ix.vals[0].as<V>(), ix.vals[1].as<V>()};
  int slot = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vp, 0, m, 0, kg.q * kg.b, false, s);
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  const uint32_t* J = nullptr;
  uint64_t A = m;
  uint64_t h = (uint64_t)kg.q;
  int rounds = 0;
  int cur = 0;
  for (;;) {
    const uint64_t nt = ceil_div(A, RF_TILE);
    ix.tile_b.ensure((nt + 1) * 4);
    ix.tile_c.ensure((nt + 1) * 4);
    ix.tile_a.ensure((nt + 2) * 8);
    ix.tile_d.ensure((nt + 2) * 8);
    k_refine_stats<<<(unsigned)nt, RF_T, 0, s>>>(kp[slot], A, ix.tile_b.as<uint32_t>(), ix.tile_c.as<uint32_t>());
    HK_HIP(hipGetLastError());
    scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nt, true, s);
    scan_exclusive_u32_to_u64(ix.sw, ix.tile_c.as<uint32_t>(), ix.tile_d.as<uint64_t>(), nt, true, s);
    V* oP = ix.act[cur ^ 1][0].as<V>();
    uint32_t* oJ = ix.act[cur ^ 1][1].as<uint32_t>();
    uint32_t* oG = ix.act[cur ^ 1][2].as<uint32_t>();
    k_refine_apply<V><<<(unsigned)nt, RF_T, 0, s>>>(kp[slot], vp[slot], J, A, ix.tile_a.as<uint64_t>(),
                                                    ix.tile_d.as<uint64_t>(), ix.sa.as<V>(), oP, oJ, oG);
    HK_HIP(hipGetLastError());
    uint64_t tot[2];
    HK_HIP(hipMemcpyAsync(&tot[0], ix.tile_a.as<uint64_t>() + nt, 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipMemcpyAsync(&tot[1], ix.tile_d.as<uint64_t>() + nt, 8, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    A = tot[0];
    ix.info.push_back(A);
    if (!A) break;
    if (++rounds > 100000) throw ApiError{-7, "shard refinement did not converge"};
    const uint64_t groups = tot[1];
    int gbits = 0;
    while (gbits < 64 && (1ull << gbits) < groups) ++gbits;
    int qn = (64 - gbits) / kg.b;
    if (qn < 1) throw ApiError{-6, "too many tied groups for one refinement key"};
    cur ^= 1;
    k_refine_keys<V><<<grid_for(A), 256, 0, s>>>(ix.act[cur][0].as<V>(), ix.act[cur][2].as<uint32_t>(), A,
                                                 ix.text.as<uint8_t>(), ix.n, d_lut, kg.b, qn, gbits, h, kp[0],
                                                 vp[0]);
    HK_HIP(hipGetLastError());
    slot = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vp, 0, A, 0, 64, false, s);
    ix.info[0] += ix.sw.passes_run;
    ix.info[1] += ix.sw.passes_skipped;
    J = ix.act[cur][1].as<uint32_t>();
    h += (uint64_t)qn;
  }
  ix.info[2] = (uint64_t)rounds;
}

template <typename V>
void shard_build_t(Index& ix, const uint64_t* ghist, int nranks, int rank) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  KeyGeom kg = geometry(ix);
  // splitters: rank r owns buckets [B[r], B[r+1]) — the first bucket whose prefix count reaches r*n/N
  std::vector<uint64_t> cum(SH_BUCKETS + 1, 0);
  for (int i = 0; i < SH_BUCKETS; ++i) cum[i + 1] = cum[i] + ghist[i];
  if (cum[SH_BUCKETS] != n) throw ApiError{-7, "global shard histogram does not sum to n"};
  auto split = [&](int r) -> uint32_t {
    if (r <= 0) return 0;
    if (r >= nranks) return SH_BUCKETS;
    const uint64_t target = (uint64_t)((__uint128_t)n * (uint64_t)r / (uint64_t)nranks);
    uint32_t lo = 0, hi = SH_BUCKETS;
    while (lo < hi) {  // smallest B with cum[B] >= target
      uint32_t mid = (lo + hi) / 2;
      if (cum[mid] >= target) hi = mid; else lo = mid + 1;
    }
    return lo;
  };
  const uint32_t blo = split(rank), bhi = split(rank + 1);
  ix.shard_lo = cum[blo];
  ix.shard_hi = cum[bhi];
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  ix.info.assign(4, 0);
  ix.info[3] = (uint64_t)kg.q;
  ix.sa.ensure(m * sizeof(V) + 16);
  ix.sharded = true;
  ix.sa_pos64 = sizeof(V) == 8;
  if (!m) {
    ix.have_sa = true;
    return;
  }
  ix.small.ensure(4096);
  uint8_t* d_lut = ix.small.as<uint8_t>() + 2048;
  unsigned long long* d_counter = ix.small.as<unsigned long long>() + 448;
  HK_HIP(hipMemcpyAsync(d_lut, kg.lut, 256, hipMemcpyHostToDevice, s));
  HK_HIP(hipMemsetAsync(d_counter, 0, 8, s));
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(m * 8 + 16);
    ix.vals[i].ensure(m * sizeof(V) + 16);
    ix.act[i][0].ensure(m * sizeof(V) + 16);
    ix.act[i][1].ensure(m * 4 + 16);
    ix.act[i][2].ensure(m * 4 + 16);
  }
  {
    TimedLaunch t(ix.timer, "shard_pack_select", (double)n + (double)m * (8 + sizeof(V)));
    k_pack_select<V><<<grid_for(n, PS_TILE, 8192), 256, 0, s>>>(ix.text.as<uint8_t>(), n, d_lut, kg.b, kg.q,
                                                               kg.bsh, blo, bhi, ix.keys[0].as<uint64_t>(),
                                                               ix.vals[0].as<V>(), d_counter);
    HK_HIP(hipGetLastError());
  }
  uint64_t got = 0;
  HK_HIP(hipMemcpyAsync(&got, d_counter, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (got != m) throw ApiError{-7, "shard selection count mismatch"};
  refine_slice<V>(ix, kg, d_lut, m);
  HK_HIP(hipStreamSynchronize(s));
  ix.have_sa = true;
}

}  // namespace

void shard_histogram(Index& ix, int nranks, int rank, uint64_t* d_hist) {
  KeyGeom kg = geometry(ix);
  hipStream_t s = ix.stream;
  const uint64_t lo = (uint64_t)((__uint128_t)ix.n * (uint64_t)rank / (uint64_t)nranks);
  const uint64_t hi = (uint64_t)((__uint128_t)ix.n * (uint64_t)(rank + 1) / (uint64_t)nranks);
  ix.small.ensure(4096);
  uint8_t* d_lut = ix.small.as<uint8_t>() + 2048;
  HK_HIP(hipMemcpyAsync(d_lut, kg.lut, 256, hipMemcpyHostToDevice, s));
  HK_HIP(hipMemsetAsync(d_hist, 0, SH_BUCKETS * 8, s));
  if (hi > lo) {
    TimedLaunch t(ix.timer, "shard_hist", (double)(hi - lo));
    k_shard_hist<<<grid_for(hi - lo, PS_TILE, 2048), 256, 0, s>>>(ix.text.as<uint8_t>(), ix.n, lo, hi, d_lut,
                                                                 kg.b, kg.q, kg.bsh,
                                                                 reinterpret_cast<unsigned long long*>(d_hist));
    HK_HIP(hipGetLastError());
  }
}

void shard_build(Index& ix, const uint64_t* h_global_hist, int nranks, int rank) {
  if (ix.n > 0xFFFFFFFEull) shard_build_t<uint64_t>(ix, h_global_hist, nranks, rank);
  else shard_build_t<uint32_t>(ix, h_global_hist, nranks, rank);
}

int shard_buckets() { return SH_BUCKETS; }

void shard_get_sa(Index& ix, uint64_t a, uint64_t b, uint64_t* out) {
  const uint64_t m = ix.shard_hi - ix.shard_lo;
  if (!(a <= b && b <= m)) throw ApiError{-4, "shard SA range out of bounds"};
  if (a == b) return;
  hipStream_t s = ix.stream;
  if (ix.sa_pos64) {
    HK_HIP(hipMemcpyAsync(out, ix.sa.as<uint64_t>() + a, (b - a) * 8, hipMemcpyDeviceToHost, s));
  } else {
    std::vector<uint32_t> tmp(b - a);
    HK_HIP(hipMemcpyAsync(tmp.data(), ix.sa.as<uint32_t>() + a, (b - a) * 4, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
    for (uint64_t i = 0; i < b - a; ++i) out[i] = tmp[i];
  }
  HK_HIP(hipStreamSynchronize(s));
}

static ShardComm g_comm;  // one communicator per process (one process per GPU)

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
  DevBuf hist;
  hist.ensure(SH_BUCKETS * 8 + 64);
  shard_histogram(ix, nranks, rank, hist.as<uint64_t>());
  {
    TimedLaunch t(ix.timer, "rccl_allreduce_hist", (double)SH_BUCKETS * 8);
    ncclcheck(ncclAllReduce(hist.p, hist.p, SH_BUCKETS, ncclUint64, ncclSum, g_comm.comm, s), "ncclAllReduce");
  }
  std::vector<uint64_t> h(SH_BUCKETS);
  HK_HIP(hipMemcpyAsync(h.data(), hist.p, SH_BUCKETS * 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  shard_build(ix, h.data(), nranks, rank);
  // merge: all-gather every rank's slice bounds and check that they tile [0, n)
  DevBuf bounds;
  bounds.ensure((size_t)nranks * 16 + 16);
  uint64_t mine[2] = {ix.shard_lo, ix.shard_hi};
  HK_HIP(hipMemcpyAsync(bounds.as<uint64_t>() + 2 * rank, mine, 16, hipMemcpyHostToDevice, s));
  {
    TimedLaunch t(ix.timer, "rccl_allgather_bounds", (double)nranks * 16);
    ncclcheck(ncclAllGather(bounds.as<uint64_t>() + 2 * rank, bounds.p, 2, ncclUint64, g_comm.comm, s),
              "ncclAllGather");
  }
  std::vector<uint64_t> all((size_t)nranks * 2);
  HK_HIP(hipMemcpyAsync(all.data(), bounds.p, nranks * 16, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  uint64_t expect = 0;
  for (int r = 0; r < nranks; ++r) {
    if (all[2 * r] != expect) throw ApiError{-8, "shard slices do not tile the suffix array"};
    expect = all[2 * r + 1];
  }
  if (expect != ix.n) throw ApiError{-8, "shard slices do not cover the suffix array"};
}

void comm_unique_id(uint8_t id[128]) {
  ncclUniqueId uid;
  ncclcheck(ncclGetUniqueId(&uid), "ncclGetUniqueId");
  memcpy(id, uid.internal, 128);
}

}  // namespace hk
