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
#include "hk_keys.hpp"

namespace hk {
namespace {

constexpr int SH_BUCKET_BITS = 14;
constexpr int SH_BUCKETS = 1 << SH_BUCKET_BITS;
constexpr int PS_TILE = 4096;

struct ShardComm {  // one RCCL communicator per process (one process per GPU)
  ncclComm_t comm = nullptr;
  int nranks = 0, rank = -1;
  uint8_t id[128];
};

// bucket of a key: its top SH_BUCKET_BITS bits (key >> bsh)
struct BucketGeom {
  uint64_t R, Rck, Rlast, Rrest;
  int q, pb, ck, bsh;
};

__global__ __launch_bounds__(256) void k_shard_hist(const uint8_t* __restrict__ t, uint64_t n, uint64_t lo,
                                                    uint64_t hi, const uint16_t* __restrict__ lut, BucketGeom g,
                                                    unsigned long long* __restrict__ hist) {
  __shared__ uint32_t H[SH_BUCKETS];
  __shared__ uint16_t c[PS_TILE + 72];
  __shared__ uint16_t L[256];
  L[threadIdx.x] = lut[threadIdx.x];
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256) H[i] = 0;
  __syncthreads();
  // tiles are aligned to PS_TILE in absolute positions so the staged text loads stay aligned
  const uint64_t first = lo / PS_TILE * PS_TILE;
  for (uint64_t base = first + (uint64_t)blockIdx.x * PS_TILE; base < hi; base += (uint64_t)gridDim.x * PS_TILE) {
    stage_text_codes<PS_TILE, 256>(c, L, t, n, base);
    __syncthreads();
    for (int k = 0; k < PS_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      const uint64_t p = base + off;
      if (p >= lo && p < hi)
        atomicAdd(&H[key_chunked(c, off, g.R, g.q, g.pb, g.ck, g.Rck, g.Rlast) >> g.bsh], 1u);
    }
    __syncthreads();
  }
  for (int i = threadIdx.x; i < SH_BUCKETS; i += 256)
    if (H[i]) atomicAdd(&hist[i], (unsigned long long)H[i]);
}

// Every rank scans all of T' and keeps the suffixes whose bucket lies in [blo, bhi).  The first
// 24-bit chunk of the key bounds the bucket to [bucket(lower), bucket(upper)]; when that interval
// misses the rank's range (the common case: (N-1)/N of all positions) the full key is never built.
template <typename V>
__global__ __launch_bounds__(256) void k_pack_select(const uint8_t* __restrict__ t, uint64_t n,
                                                     const uint16_t* __restrict__ lut, BucketGeom g, uint32_t blo,
                                                     uint32_t bhi, uint64_t* __restrict__ keys,
                                                     V* __restrict__ vals, unsigned long long* counter) {
  __shared__ uint16_t c[PS_TILE + 72];
  __shared__ uint16_t L[256];
  __shared__ uint32_t red[4];
  __shared__ unsigned long long gbase;
  L[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const bool pretest = g.q > g.ck;
  const uint64_t pbmask = (1ull << g.pb) - 1;
  for (uint64_t base = (uint64_t)blockIdx.x * PS_TILE; base < n; base += (uint64_t)gridDim.x * PS_TILE) {
    stage_text_codes<PS_TILE, 256>(c, L, t, n, base);
    __syncthreads();
    uint64_t kk[PS_TILE / 256];
    uint32_t sel = 0;
#pragma unroll
    for (int k = 0; k < PS_TILE / 256; ++k) {
      const int off = k * 256 + threadIdx.x;
      kk[k] = 0;
      if (base + off < n) {
        if (pretest) {
          const uint32_t cv0 = chunk_value(c, off + 1, g.ck, (uint32_t)g.R);
          const uint64_t lower = (uint64_t)cv0 * g.Rrest;
          const uint32_t b_lo = (uint32_t)((lower << g.pb) >> g.bsh);
          const uint32_t b_hi = (uint32_t)((((lower + g.Rrest - 1) << g.pb) | pbmask) >> g.bsh);
          if (b_hi >= blo && b_lo < bhi) {
            kk[k] = key_from(c, off, g.R, g.q, g.pb, g.ck, g.Rck, g.Rlast, g.ck + 1, cv0);
            const uint32_t bk = (uint32_t)(kk[k] >> g.bsh);
            if (bk >= blo && bk < bhi) sel |= 1u << k;
          }
        } else {
          kk[k] = key_chunked(c, off, g.R, g.q, g.pb, g.ck, g.Rck, g.Rlast);
          const uint32_t bk = (uint32_t)(kk[k] >> g.bsh);
          if (bk >= blo && bk < bhi) sel |= 1u << k;
        }
      }
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

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

void ncclcheck(ncclResult_t r, const char* what) {
  if (r != ncclSuccess) throw ApiError{-8, std::string(what) + ": " + ncclGetErrorString(r)};
}

int bucket_shift(const KeyGeom& kg) {
  const int sh = kg.key_bits - SH_BUCKET_BITS;
  return sh < 0 ? 0 : sh;
}

BucketGeom bucket_geom(const KeyGeom& kg) {
  const KeyChunks kc = key_chunks(kg.R, kg.q);
  return BucketGeom{kg.R, kc.Rck, kc.Rlast, kc.Rrest, kg.q, kg.pb, kc.ck, bucket_shift(kg)};
}

template <typename V>
void shard_build_t(Index& ix, const uint64_t* ghist, int nranks, int rank) {
  const uint64_t n = ix.n;
  hipStream_t s = ix.stream;
  KeyGeom kg = key_geometry(ix, true);
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
  ix.sharded = true;
  ix.sa_pos64 = sizeof(V) == 8;
  ix.have_sa = ix.have_bwt = ix.have_wt = false;
  ix.sa.ensure(m * sizeof(V) + 16);
  if (!m) {
    ix.have_sa = true;
    return;
  }
  upload_geometry(ix, kg);
  ix.small.ensure(8192);
  unsigned long long* d_counter = ix.small.as<unsigned long long>() + 448;
  HK_HIP(hipMemsetAsync(d_counter, 0, 8, s));
  for (int i = 0; i < 2; ++i) {
    ix.keys[i].ensure(m * 8 + 16);
    ix.vals[i].ensure(m * sizeof(V) + 16);
  }
  {
    TimedLaunch t(ix.timer, "shard_pack_select", (double)n + (double)m * (8 + sizeof(V)));
    k_pack_select<V><<<grid_for(n, PS_TILE, 8192), 256, 0, s>>>(
        ix.text.as<uint8_t>(), n, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048),
        bucket_geom(kg), blo, bhi, ix.keys[0].as<uint64_t>(), ix.vals[0].as<V>(), d_counter);
    HK_HIP(hipGetLastError());
  }
  uint64_t got = 0;
  HK_HIP(hipMemcpyAsync(&got, d_counter, 8, hipMemcpyDeviceToHost, s));
  HK_HIP(hipStreamSynchronize(s));
  if (got != m) throw ApiError{-7, "shard selection count mismatch"};
  uint64_t* kp[2] = {ix.keys[0].as<uint64_t>(), ix.keys[1].as<uint64_t>()};
  V* vp[2] = {ix.vals[0].as<V>(), ix.vals[1].as<V>()};
  const int slot = radix_sort_pairs<V>(ix.sw, ix.timer, kp, vp, 0, m, kg.pb, kg.key_bits, false, s);
  ix.info[0] += ix.sw.passes_run;
  ix.info[1] += ix.sw.passes_skipped;
  std::swap(ix.sa, ix.vals[slot]);
  ix.vals[slot].ensure(m * sizeof(V) + 16);
  refine_after_sort<V>(ix, kg, slot, m, false);
  HK_HIP(hipStreamSynchronize(s));
  ix.have_sa = true;
  ix.have_bwt = true;   // BWT of the slice (bwt[j] for SA[lo + j])
}

}  // namespace

void shard_histogram(Index& ix, int nranks, int rank, uint64_t* d_hist) {
  KeyGeom kg = key_geometry(ix, true);
  hipStream_t s = ix.stream;
  const uint64_t lo = (uint64_t)((__uint128_t)ix.n * (uint64_t)rank / (uint64_t)nranks);
  const uint64_t hi = (uint64_t)((__uint128_t)ix.n * (uint64_t)(rank + 1) / (uint64_t)nranks);
  upload_geometry(ix, kg);
  HK_HIP(hipMemsetAsync(d_hist, 0, SH_BUCKETS * 8, s));
  if (hi > lo) {
    TimedLaunch t(ix.timer, "shard_hist", (double)(hi - lo));
    k_shard_hist<<<grid_for(hi - lo, PS_TILE, 2048), 256, 0, s>>>(
        ix.text.as<uint8_t>(), ix.n, lo, hi, reinterpret_cast<const uint16_t*>(ix.small.as<uint8_t>() + 2048),
        bucket_geom(kg), reinterpret_cast<unsigned long long*>(d_hist));
    HK_HIP(hipGetLastError());
  }
}

void shard_build(Index& ix, const uint64_t* h_global_hist, int nranks, int rank) {
  if (ix.n > 0xFFFFFFFEull || (ix.flags & kFlagPos64)) shard_build_t<uint64_t>(ix, h_global_hist, nranks, rank);
  else shard_build_t<uint32_t>(ix, h_global_hist, nranks, rank);
}

int shard_buckets() { return SH_BUCKETS; }

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
