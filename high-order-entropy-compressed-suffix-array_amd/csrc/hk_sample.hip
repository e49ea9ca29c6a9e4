// hk_sample.hip — SA/ISA sampling, LF-walk locate and extract.
//
// The `epsilon` contract of CompressedSuffixArray(text, epsilon) (tests/benchmark.py:25,32):
// trade the full SA (4n bytes) for samples every s text positions, answering locate/extract by
// LF walks over the wavelet tree.  Results are identical to the full-SA path.
//
//   mark        rank lines over rows: bit i = (SA[i] % s == 0)      n/8 · 8/7 bytes
//   samp_sa     SA[i] of the marked rows, in row order               4 · ceil(n/s) bytes
//   samp_isa    row of text position k·s                             4 · ceil(n/s) bytes
//   fix         the true LF of the rows whose BWT symbol is c* = T'[n-1]   4 · occ(c*) bytes
// (4-byte words while n < 2^32; a replicated index of a text with >= 2^32 suffixes, whose SA is u64,
// keeps 8-byte samples: every kernel below is templated on the word W)
//
// Why `fix`: BWT[row of SA=0] wraps to T'[n-1] (csa/bwt.py:8-11), so the c*-rows of the BWT are
// the suffixes preceded by c* plus the wrapped row.  For every other symbol c, C[c] + occ(c, i)
// is the row of suffix SA[i]-1; for c* it is only when the wrapped row is the first c*-row, which
// fails when c* also occurs inside the text (the reference's '$' quirk).  The walk therefore
// takes the LF of a c*-row from `fix`, making it the exact cyclic predecessor everywhere.
//
//   locate(row):  k = 0; while !mark[row]: row = LF(row), ++k;  SA = samp_sa[rank(row)] + k
//                 (position 0 is always sampled, so the walk never wraps)
//   extract(i,j): one lane per sample interval [k·s, (k+1)·s): start at the row of (k+1)·s (the
//                 row of 0 for the interval ending at n) and emit BWT[row] = T'[p-1] while
//                 stepping row = LF(row).
#include <algorithm>
#include <type_traits>

#include "hk_index.hpp"
#include "hk_wtq.hpp"

namespace hk {
namespace {

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

// one wave per 448-row line: 7 ballots of (SA[j] % s == 0)
template <typename W>
__global__ __launch_bounds__(256) void k_smp_bits(const W* __restrict__ sa, uint64_t n, uint32_t s,
                                                  uint64_t* __restrict__ lines, uint32_t* __restrict__ line_pop,
                                                  uint64_t nlines) {
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t li = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); li < nlines; li += (uint64_t)gridDim.x * 4) {
    const uint64_t base = li * kLineBits;
    uint64_t w[7];
    uint32_t pop = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i) {
      const uint64_t j = base + (uint64_t)i * 64 + lane;
      const bool bit = j < n && sa[j] % s == 0;
      w[i] = ballot64(bit);
      pop += (uint32_t)__popcll(w[i]);
    }
    uint64_t v = 0;
#pragma unroll
    for (int i = 0; i < 7; ++i)
      if (lane == (uint32_t)i + 1) v = w[i];
    if (lane < 8) lines[li * 8 + lane] = v;
    if (lane == 0) line_pop[li] = pop;
  }
}

__global__ __launch_bounds__(256) void k_smp_fill_lines(uint64_t* __restrict__ lines,
                                                        const uint64_t* __restrict__ excl, uint64_t nlines) {
  for (uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x; li < nlines; li += (uint64_t)gridDim.x * 256)
    lines[li * 8] = excl[li];
}

template <typename W>
__global__ __launch_bounds__(256) void k_smp_fill(const W* __restrict__ sa, uint64_t n, uint32_t s,
                                                  const uint64_t* __restrict__ mark, W* __restrict__ ssa,
                                                  W* __restrict__ sisa) {
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < n; j += (uint64_t)gridDim.x * 256) {
    const W p = sa[j];
    if (p % s) continue;
    ssa[rank1(mark, j)] = p;
    sisa[p / s] = (W)j;
  }
}

// c*-rows i: tmp[SA[i]] = occ(c*, i) (their order among the c*-rows)
template <typename W>
__global__ __launch_bounds__(256) void k_fix_a(WtView v, const W* __restrict__ sa,
                                               const uint8_t* __restrict__ bwt, uint8_t cstar_byte, int cstar,
                                               W* __restrict__ tmp) {
  __shared__ QShared q;
  load_qshared(q, v);
  const uint64_t n = v.n;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    if (bwt[i] != cstar_byte) continue;
    uint64_t x = i, y = i;
    lf_pair(q, cstar, x, y);
    tmp[sa[i]] = (W)(x - v.Ccode[cstar]);
  }
}

// rows j of the c* bucket: the c*-row whose suffix is SA[j]+1 (cyclically) has true LF j
template <typename W>
__global__ __launch_bounds__(256) void k_fix_b(const W* __restrict__ sa, uint64_t n, uint64_t b0, uint64_t cnt,
                                               const W* __restrict__ tmp, W* __restrict__ fix) {
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < cnt; k += (uint64_t)gridDim.x * 256) {
    const uint64_t j = b0 + k;
    uint64_t p = (uint64_t)sa[j] + 1;
    if (p == n) p = 0;
    fix[tmp[p]] = (W)j;
  }
}

// The same with few c*-rows (the usual case: c* = the '$' that ends T' occurs once), without the
// n-entry scratch: pos[k] = SA of the c*-row of rank k, then one workgroup matches each pos[k] - 1
// against the c* bucket's SA entries held in LDS (fix[k] = the bucket row j with SA[j] = pos[k] - 1).
constexpr uint64_t kFixSmall = 4096;

template <typename W>
__global__ __launch_bounds__(256) void k_fix_a_rank(WtView v, const W* __restrict__ sa,
                                                    const uint8_t* __restrict__ bwt, uint8_t cstar_byte, int cstar,
                                                    W* __restrict__ pos) {
  __shared__ QShared q;
  load_qshared(q, v);
  const uint64_t n = v.n;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    if (bwt[i] != cstar_byte) continue;
    uint64_t x = i, y = i;
    lf_pair(q, cstar, x, y);
    pos[x - v.Ccode[cstar]] = sa[i];
  }
}

template <typename W>
__global__ __launch_bounds__(1024) void k_fix_b_small(const W* __restrict__ sa, uint64_t n, uint64_t b0, uint32_t cnt,
                                                      const W* __restrict__ pos, W* __restrict__ fix) {
  __shared__ W B[kFixSmall];
  for (uint32_t j = threadIdx.x; j < cnt; j += 1024) B[j] = sa[b0 + j];
  __syncthreads();
  for (uint32_t k = threadIdx.x; k < cnt; k += 1024) {
    const uint64_t p = pos[k];
    const W want = (W)(p == 0 ? n - 1 : p - 1);
    for (uint32_t j = 0; j < cnt; ++j)
      if (B[j] == want) {
        fix[k] = (W)(b0 + j);
        break;
      }
  }
}

template <typename W>
struct SmpView {
  const uint64_t* mark;
  const W* ssa;
  const W* sisa;
  const W* fix;
  uint64_t cbase;   // C[c*] (first row of the c* bucket)
  int cstar;
  uint32_t s;
};

// exact cyclic LF (row of suffix SA[x]-1) and the BWT code of row x
template <typename W>
__device__ __forceinline__ uint64_t lf_exact(const QShared& q, const WtView& v, const SmpView<W>& m, uint64_t x,
                                             int& code) {
  uint64_t y = lf_access(q, v.sigma, x, code);
  if (code == m.cstar) y = m.fix[y - m.cbase];
  return y;
}

template <typename W>
__device__ __forceinline__ uint64_t sa_of_row(const QShared& q, const WtView& v, const SmpView<W>& m, uint64_t x) {
  uint64_t k = 0;
  for (;;) {
    uint32_t b;
    const uint64_t r = rank1_bit(m.mark, x, b);
    if (b) return (uint64_t)m.ssa[r] + k;
    int c;
    x = lf_exact(q, v, m, x, c);
    ++k;
  }
}

constexpr uint64_t kSmallOcc = 32;
constexpr uint64_t kHugeOcc = 1ull << 16;   // one pattern spread over every workgroup

template <typename W>
__global__ __launch_bounds__(256) void k_locate_smp_small(WtView v, SmpView<W> m, const int64_t* __restrict__ lr,
                                                          const uint64_t* __restrict__ oo, uint64_t P,
                                                          uint64_t* __restrict__ pos, uint64_t* big,
                                                          unsigned long long* nbig) {
  __shared__ QShared q;
  load_qshared(q, v);
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (uint64_t)gridDim.x * 256) {
    const int64_t l = lr[2 * p];
    if (l < 0) continue;
    const uint64_t c = (uint64_t)(lr[2 * p + 1] - l + 1);
    if (c > kSmallOcc) {   // big: one workgroup each; huge: every workgroup (listed from the end of big)
      if (c > kHugeOcc) big[P - 1 - atomicAdd(nbig + 1, 1ull)] = p;
      else big[atomicAdd(nbig, 1ull)] = p;
      continue;
    }
    const uint64_t o = oo[p];
    for (uint64_t i = 0; i < c; ++i) pos[o + i] = sa_of_row(q, v, m, (uint64_t)l + i);
  }
}

template <typename W>
__global__ __launch_bounds__(256) void k_locate_smp_big(WtView v, SmpView<W> m, const int64_t* __restrict__ lr,
                                                        const uint64_t* __restrict__ oo,
                                                        const uint64_t* __restrict__ big,
                                                        const unsigned long long* __restrict__ nbig, uint64_t P,
                                                        uint64_t* __restrict__ pos) {
  __shared__ QShared q;
  load_qshared(q, v);
  const uint64_t nb = nbig[0], nh = nbig[1];
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t p = big[b];
    const uint64_t l = (uint64_t)lr[2 * p];
    const uint64_t c = (uint64_t)(lr[2 * p + 1] + 1) - l;
    const uint64_t o = oo[p];
    for (uint64_t i = threadIdx.x; i < c; i += 256) pos[o + i] = sa_of_row(q, v, m, l + i);
  }
  for (uint64_t h = 0; h < nh; ++h) {   // a pattern with more than kHugeOcc rows (e.g. the empty one)
    const uint64_t p = big[P - 1 - h];
    const uint64_t l = (uint64_t)lr[2 * p];
    const uint64_t c = (uint64_t)(lr[2 * p + 1] + 1) - l;
    const uint64_t o = oo[p];
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < c; i += (uint64_t)gridDim.x * 256)
      pos[o + i] = sa_of_row(q, v, m, l + i);
  }
}

// SA[lo + t] for t < count (full-array export in compressed mode)
template <typename W>
__global__ __launch_bounds__(256) void k_sa_range_smp(WtView v, SmpView<W> m, uint64_t lo, uint64_t count,
                                                      uint64_t* __restrict__ out) {
  __shared__ QShared q;
  load_qshared(q, v);
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < count; t += (uint64_t)gridDim.x * 256)
    out[t] = sa_of_row(q, v, m, lo + t);
}

// BWT[lo + t] by WT access
__global__ __launch_bounds__(256) void k_bwt_range(WtView v, uint64_t lo, uint64_t count,
                                                   const uint8_t* __restrict__ inv, uint8_t* __restrict__ out) {
  __shared__ QShared q;
  load_qshared(q, v);
  for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < count; t += (uint64_t)gridDim.x * 256) {
    int c;
    (void)lf_access(q, v.sigma, lo + t, c);
    out[t] = inv[c];
  }
}

// T'[i:j): one lane per sample interval
template <typename W>
__global__ __launch_bounds__(256) void k_extract_smp(WtView v, SmpView<W> m, uint64_t i, uint64_t j,
                                                     const uint8_t* __restrict__ inv, uint8_t* __restrict__ out) {
  __shared__ QShared q;
  load_qshared(q, v);
  const uint64_t n = v.n, s = m.s;
  const uint64_t k0 = i / s, k1 = (j - 1) / s;
  for (uint64_t k = k0 + (uint64_t)blockIdx.x * 256 + threadIdx.x; k <= k1; k += (uint64_t)gridDim.x * 256) {
    uint64_t e = (k + 1) * s;
    if (e > n) e = n;
    uint64_t row = e == n ? m.sisa[0] : m.sisa[e / s];
    const uint64_t stop = k * s > i ? k * s : i;
    for (uint64_t p = e; p > stop;) {   // emits T'[p-1]
      --p;
      int c;
      row = lf_exact(q, v, m, row, c);
      if (p < j) out[p - i] = inv[c];
    }
  }
}

template <typename W>
SmpView<W> smp_view(const Index& ix) {
  return SmpView<W>{ix.smp_mark.as<uint64_t>(), ix.smp_sa.as<W>(), ix.smp_isa.as<W>(), ix.smp_fix.as<W>(),
                    ix.Ccode[ix.smp_cstar], ix.smp_cstar, ix.smp_rate};
}

template <typename W>
void build_samples_t(Index& ix, uint32_t rate) {
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  const uint64_t nlines = n / kLineBits + 1;
  const W* sa = ix.sa.as<W>();
  ix.smp_mark.ensure(nlines * 64);
  ix.tile_b.ensure(nlines * 4 + 16);
  ix.tile_a.ensure(nlines * 8 + 16);
  {
    TimedLaunch t(ix.timer, "smp_mark", (double)n * sizeof(W) + (double)nlines * 64);
    k_smp_bits<W><<<grid_for(nlines, 4, 8192), 256, 0, s>>>(sa, n, rate, ix.smp_mark.as<uint64_t>(),
                                                            ix.tile_b.as<uint32_t>(), nlines);
    HK_HIP(hipGetLastError());
  }
  scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nlines, false, s);
  k_smp_fill_lines<<<grid_for(nlines), 256, 0, s>>>(ix.smp_mark.as<uint64_t>(), ix.tile_a.as<uint64_t>(), nlines);
  HK_HIP(hipGetLastError());
  const uint64_t ns = ceil_div(n, rate);   // positions 0, s, 2s, ... < n
  ix.smp_sa.ensure(ns * sizeof(W) + 16);
  ix.smp_isa.ensure(ns * sizeof(W) + 16);
  {
    TimedLaunch t(ix.timer, "smp_fill", (double)n * sizeof(W) + (double)ns * 2 * sizeof(W));
    k_smp_fill<W><<<grid_for(n), 256, 0, s>>>(sa, n, rate, ix.smp_mark.as<uint64_t>(), ix.smp_sa.as<W>(),
                                              ix.smp_isa.as<W>());
    HK_HIP(hipGetLastError());
  }
  // exact LF of the c*-rows
  uint8_t last = 0;
  if (ix.tail_valid) {   // read with the byte histogram
    last = ix.tail[std::min<uint64_t>(n, 70) - 1];
  } else {
    HK_HIP(hipMemcpyAsync(&last, ix.text.as<uint8_t>() + n - 1, 1, hipMemcpyDeviceToHost, s));
    HK_HIP(hipStreamSynchronize(s));
  }
  const int cstar = ix.code_of[last];
  const uint64_t cnt = ix.Ccode[cstar + 1] - ix.Ccode[cstar];
  ix.smp_fix.ensure(cnt * sizeof(W) + 16);
  if (cnt <= kFixSmall) {   // few c*-rows: a cnt-entry scratch
    ix.tile_d.ensure(cnt * sizeof(W) + 16);
    TimedLaunch t(ix.timer, "smp_fix", (double)n * 1 + (double)cnt * 4 * sizeof(W));
    k_fix_a_rank<W><<<grid_for(n, 256, 8192), 256, 0, s>>>(ix.view(), sa, ix.bwt.as<uint8_t>(), last, cstar,
                                                           ix.tile_d.as<W>());
    HK_HIP(hipGetLastError());
    k_fix_b_small<W><<<1, 1024, 0, s>>>(sa, n, ix.Ccode[cstar], (uint32_t)cnt, ix.tile_d.as<W>(), ix.smp_fix.as<W>());
    HK_HIP(hipGetLastError());
  } else {
    // scratch tmp[SA[i]] for the c*-rows: an n-entry buffer of the construction workspace when one is
    // resident (no allocation), else the ISA buffer
    W* tmp = nullptr;
    for (DevBuf* b : {&ix.keys[0], &ix.keys[1], &ix.vals[0], &ix.vals[1], &ix.isa})
      if (!tmp && b->p && b->bytes >= n * sizeof(W)) tmp = b->as<W>();
    if (!tmp) {
      ix.isa.ensure(n * sizeof(W) + 16);
      tmp = ix.isa.as<W>();
    }
    TimedLaunch t(ix.timer, "smp_fix", (double)n * (1 + sizeof(W)) + (double)cnt * 4 * sizeof(W));
    k_fix_a<W><<<grid_for(n, 256, 8192), 256, 0, s>>>(ix.view(), sa, ix.bwt.as<uint8_t>(), last, cstar, tmp);
    HK_HIP(hipGetLastError());
    k_fix_b<W><<<grid_for(cnt), 256, 0, s>>>(sa, n, ix.Ccode[cstar], cnt, tmp, ix.smp_fix.as<W>());
    HK_HIP(hipGetLastError());
  }
  ix.smp_inv.ensure(256);
  HK_HIP(hipMemcpyAsync(ix.smp_inv.p, ix.syms, 256, hipMemcpyHostToDevice, s));
  HK_HIP(hipStreamSynchronize(s));
  ix.smp_rate = rate;
  ix.smp_count = ns;
  ix.smp_fixn = cnt;
  ix.smp_cstar = cstar;
  ix.smp_w64 = sizeof(W) == 8;
  ix.have_samples = true;
}

}  // namespace

// A replicated sharded index (shard_replicate: the whole u64 SA on every rank) samples like a single-GPU
// one; a slice-only sharded index has no whole SA to sample.
void build_samples(Index& ix, uint32_t rate) {
  if (rate == 0) throw ApiError{-2, "sample rate must be positive"};
  if (!ix.have_sa || ix.sharded) throw ApiError{-3, "samples: whole suffix array not built (a slice-only sharded index)"};
  if (!ix.have_bwt || !ix.have_text) throw ApiError{-3, "samples: BWT not built"};
  if (!ix.have_wt) build_wt(ix);
  if (ix.sa_pos64) build_samples_t<uint64_t>(ix, rate);
  else build_samples_t<uint32_t>(ix, rate);
}

void compact(Index& ix) {
  if (!ix.have_samples) throw ApiError{-3, "compact: build the SA samples first"};
  HK_HIP(hipStreamSynchronize(ix.stream));
  ix.sa.release();
  ix.bwt.release();
  ix.text.release();
  ix.have_sa = false;
  ix.have_text = false;
  ix.bwt_in_wt = true;
  release_workspace(ix);
}

void sampled_locate_gather(Index& ix, const int64_t* d_lr, const uint64_t* d_occ_offs, uint64_t P, uint64_t* d_pos) {
  if (!ix.have_samples) throw ApiError{-3, "locate: no suffix array and no samples"};
  if (!P) return;
  hipStream_t s = ix.stream;
  ix.tile_c.ensure((P + 2) * 8);
  ix.small.ensure(8192);
  unsigned long long* nbig = ix.small.as<unsigned long long>() + 520;
  HK_HIP(hipMemsetAsync(nbig, 0, 16, s));   // big and huge pattern counts
  TimedLaunch t(ix.timer, "fm_locate_sampled", 0.0);
  auto run = [&](auto m) {
    using W = std::remove_const_t<std::remove_pointer_t<decltype(m.ssa)>>;
    k_locate_smp_small<W><<<grid_for(P, 256, 65535), 256, 0, s>>>(ix.view(), m, d_lr, d_occ_offs, P, d_pos,
                                                                  ix.tile_c.as<uint64_t>(), nbig);
    HK_HIP(hipGetLastError());
    k_locate_smp_big<W><<<1024, 256, 0, s>>>(ix.view(), m, d_lr, d_occ_offs, ix.tile_c.as<uint64_t>(), nbig, P, d_pos);
    HK_HIP(hipGetLastError());
  };
  if (ix.smp_w64) run(smp_view<uint64_t>(ix));
  else run(smp_view<uint32_t>(ix));
}

void sampled_sa_range(Index& ix, uint64_t lo, uint64_t count, uint64_t* d_out) {
  if (!ix.have_samples) throw ApiError{-3, "no suffix array and no samples"};
  if (!count) return;
  if (ix.smp_w64)
    k_sa_range_smp<uint64_t><<<grid_for(count, 256, 65535), 256, 0, ix.stream>>>(ix.view(), smp_view<uint64_t>(ix), lo,
                                                                                 count, d_out);
  else
    k_sa_range_smp<uint32_t><<<grid_for(count, 256, 65535), 256, 0, ix.stream>>>(ix.view(), smp_view<uint32_t>(ix), lo,
                                                                                 count, d_out);
  HK_HIP(hipGetLastError());
}

void wt_bwt_range(Index& ix, uint64_t lo, uint64_t count, uint8_t* d_out) {
  if (!ix.have_wt) throw ApiError{-3, "BWT: wavelet tree not built"};
  if (!count) return;
  ix.smp_inv.ensure(256);
  HK_HIP(hipMemcpyAsync(ix.smp_inv.p, ix.syms, 256, hipMemcpyHostToDevice, ix.stream));
  k_bwt_range<<<grid_for(count, 256, 65535), 256, 0, ix.stream>>>(ix.view(), lo, count, ix.smp_inv.as<uint8_t>(),
                                                                  d_out);
  HK_HIP(hipGetLastError());
}

void sampled_extract(Index& ix, uint64_t i, uint64_t j, uint8_t* d_out) {
  if (!ix.have_samples) throw ApiError{-3, "extract: no text and no samples"};
  if (j <= i) return;
  const uint64_t lanes = (j - 1) / ix.smp_rate - i / ix.smp_rate + 1;
  TimedLaunch t(ix.timer, "extract_sampled", 0.0);
  if (ix.smp_w64)
    k_extract_smp<uint64_t><<<grid_for(lanes, 256, 65535), 256, 0, ix.stream>>>(ix.view(), smp_view<uint64_t>(ix), i,
                                                                                j, ix.smp_inv.as<uint8_t>(), d_out);
  else
    k_extract_smp<uint32_t><<<grid_for(lanes, 256, 65535), 256, 0, ix.stream>>>(ix.view(), smp_view<uint32_t>(ix), i,
                                                                                j, ix.smp_inv.as<uint8_t>(), d_out);
  HK_HIP(hipGetLastError());
}

}  // namespace hk
