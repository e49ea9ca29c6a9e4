// hk_wt.hip — levelwise wavelet tree over the BWT and the batched FM-index queries.
//
// Wavelet tree (reference: csa/wavelet_tree.py:65-100, split rule :78-80).
//   Dense codes 0..sigma-1 = rank of each byte among those present.  A node covering codes
//   [lo,hi) splits at mid = lo + (hi-lo)/2 (the reference's len(alphabet)//2); bit = code >= mid.
//   Levels are stored levelwise: level d is the BWT stably partitioned by depth-d node, nodes
//   left to right, so node [lo,hi) occupies [C[lo], C[hi]) and the reference's left-spine level
//   d is the prefix of our level d of length C[sigma_d].  Codes whose leaf is shallower than the
//   tree keep bit 0 and never move.
//
// Rank lines: every 64-B line holds u64 "ones before this line" + 7 data words (448 bits), so
//   rank1(x) touches exactly one line (one 64-B block per rank per level).
//
// Queries (csa/enhanced_fm_index.py:21-32 backward search):
//   one lane per pattern walks the levels for each symbol.  Because node starts are C-array
//   offsets, the absolute position reached at the leaf IS the LF value C[c] + occ(c, x):
//     bit 0: x <- x - rank1(x) + obn      bit 1: x <- rbase + rank1(x)
//   with obn = ones before the node, rbase = node start + zeros in node - obn (per level/code
//   tables in LDS).

#include "hk_index.hpp"
#include "hk_wtq.hpp"

namespace hk {

WtView Index::view() const {
  WtView v{};
  for (int d = 0; d < kMaxLevels; ++d) v.lines[d] = d < wt_levels ? wt_lines[d].as<uint64_t>() : nullptr;
  v.obn = wt_obn.as<uint64_t>();
  v.rbase = wt_rbase.as<uint64_t>();
  v.bit = wt_bit.as<uint8_t>();
  v.depth = wt_depth.as<uint8_t>();
  v.code = wt_code.as<int16_t>();
  v.Ccode = wt_C.as<uint64_t>();
  v.levels = wt_levels;
  v.sigma = sigma;
  v.n = n;
  return v;
}

namespace {

// Level kernels process WT_G lines (448 symbols each) per wave iteration with all their symbol loads
// issued up front (one byte per lane per 64 symbols): the single-line form kept only 7 x 64 B in
// flight per wave and ran latency-bound at 10-20 % of HBM bandwidth (profiles/r2_kernel_stats.csv).
// Level 0 reads the BWT bytes themselves through a byte -> code table (no separate code-mapping pass).
constexpr int WT_G = 4;

// one wave per WT_G lines: 7 ballots per line -> 7 words; word 0 later receives the ones-before count
__global__ __launch_bounds__(256) void k_wt_bits(const uint8_t* __restrict__ S, uint64_t n,
                                                 const uint8_t* __restrict__ bitlut,
                                                 uint64_t* __restrict__ lines,
                                                 uint32_t* __restrict__ line_pop, uint64_t nlines) {
  __shared__ uint8_t B[256];
  B[threadIdx.x] = bitlut[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g * WT_G < nlines; g += (uint64_t)gridDim.x * 4) {
    const uint64_t base = g * WT_G * kLineBits;
    uint8_t sym[WT_G * 7];
#pragma unroll
    for (int i = 0; i < WT_G * 7; ++i) {
      const uint64_t j = base + (uint64_t)i * 64 + lane;
      sym[i] = j < n ? S[j] : 0;
    }
#pragma unroll
    for (int q = 0; q < WT_G; ++q) {
      const uint64_t li = g * WT_G + q;
      if (li >= nlines) break;
      uint64_t w[7];
      uint32_t pop = 0;
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint64_t j = base + (uint64_t)(q * 7 + i) * 64 + lane;
        w[i] = ballot64(j < n && B[sym[q * 7 + i]]);
        pop += (uint32_t)__popcll(w[i]);
      }
      uint64_t v = 0;
#pragma unroll
      for (int i = 0; i < 7; ++i)
        if (lane == (uint32_t)i + 1) v = w[i];
      if (lane >= 1 && lane < 8) lines[li * 8 + lane] = v;
      if (lane == 0) line_pop[li] = pop;
    }
  }
}

__global__ __launch_bounds__(256) void k_wt_fill(uint64_t* __restrict__ lines,
                                                 const uint64_t* __restrict__ excl, uint64_t nlines) {
  for (uint64_t li = (uint64_t)blockIdx.x * 256 + threadIdx.x; li < nlines; li += (uint64_t)gridDim.x * 256)
    lines[li * 8] = excl[li];
}

__global__ void k_wt_tables(const uint64_t* __restrict__ lines, int sigma,
                            const uint64_t* __restrict__ start, const uint64_t* __restrict__ zeros,
                            uint64_t* __restrict__ obn, uint64_t* __restrict__ rbase) {
  const int c = threadIdx.x;
  if (c < sigma) {
    const uint64_t o = rank1(lines, start[c]);
    obn[c] = o;
    rbase[c] = start[c] + zeros[c] - o;
  }
}

// stable partition of level d's sequence into level d+1 (one wave per WT_G lines); `code` maps the
// input symbols to dense codes (level 0 reads BWT bytes) or is the identity
__global__ __launch_bounds__(256) void k_wt_partition(const uint8_t* __restrict__ S, uint8_t* __restrict__ out,
                                                      uint64_t n, const uint64_t* __restrict__ lines,
                                                      uint64_t nlines, const uint64_t* __restrict__ obn,
                                                      const uint64_t* __restrict__ rbase,
                                                      const uint8_t* __restrict__ code) {
  __shared__ uint64_t OB[256], RB[256];
  __shared__ uint8_t CODE[256];
  OB[threadIdx.x] = obn[threadIdx.x];
  RB[threadIdx.x] = rbase[threadIdx.x];
  CODE[threadIdx.x] = code[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63;
  for (uint64_t g0 = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); g0 * WT_G < nlines;
       g0 += (uint64_t)gridDim.x * 4) {
    const uint64_t g = __builtin_amdgcn_readfirstlane((uint32_t)g0);
    const uint64_t base = g * WT_G * kLineBits;
    uint8_t sym[WT_G * 7];
#pragma unroll
    for (int i = 0; i < WT_G * 7; ++i) {
      const uint64_t j = base + (uint64_t)i * 64 + lane;
      sym[i] = j < n ? S[j] : 0;
    }
#pragma unroll
    for (int q = 0; q < WT_G; ++q) {
      const uint64_t li = g * WT_G + q;
      if (li >= nlines) break;
      const uint64_t* L = lines + li * 8;
      uint64_t pre = L[0];
#pragma unroll
      for (int i = 0; i < 7; ++i) {
        const uint64_t w = L[1 + i];
        const uint64_t j = base + (uint64_t)(q * 7 + i) * 64 + lane;
        if (j < n) {
          const uint8_t c = CODE[sym[q * 7 + i]];
          const uint64_t ob = pre + mbcnt(w);
          const uint64_t dst = ((w >> lane) & 1ull) ? RB[c] + ob : j - ob + OB[c];
          out[dst] = c;
        }
        pre += (uint64_t)__popcll(w);
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_wt_extract(const uint64_t* __restrict__ lines, uint64_t nwords,
                                                    uint64_t* __restrict__ words) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nwords; w += (uint64_t)gridDim.x * 256)
    words[w] = lines[(w / 7) * 8 + 1 + (w % 7)];
}

// ------------------------------------------------------------ queries
__global__ __launch_bounds__(256) void k_count(WtView v, const uint8_t* __restrict__ pats,
                                               const uint64_t* __restrict__ offs, uint64_t P,
                                               int64_t* __restrict__ lr, uint64_t* __restrict__ cnt) {
  __shared__ QShared q;
  load_qshared(q, v);
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (uint64_t)gridDim.x * 256) {
    const uint64_t s = offs[p];
    uint64_t k = offs[p + 1];
    uint64_t xl = 0, xr = v.n;
    bool ok = true;
    while (k > s) {
      --k;
      const int c = q.code[pats[k]];
      if (c < 0) { ok = false; break; }
      lf_pair(q, c, xl, xr);
      if (xl >= xr) { ok = false; break; }
    }
    lr[2 * p] = ok ? (int64_t)xl : -1;
    lr[2 * p + 1] = ok ? (int64_t)xr - 1 : -1;
    if (cnt) cnt[p] = ok ? xr - xl : 0;
  }
}

__global__ __launch_bounds__(256) void k_rank(WtView v, const uint8_t* __restrict__ cs,
                                              const uint64_t* __restrict__ is, uint64_t K,
                                              uint64_t* __restrict__ out) {
  __shared__ QShared q;
  load_qshared(q, v);
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < K; k += (uint64_t)gridDim.x * 256) {
    const int c = q.code[cs[k]];
    if (c < 0) { out[k] = 0; continue; }
    uint64_t x = is[k] < v.n ? is[k] : v.n;
    uint64_t y = x;
    lf_pair(q, c, x, y);
    out[k] = x - v.Ccode[c];
  }
}

constexpr uint64_t kSmallOcc = 32;

template <typename S>
__global__ __launch_bounds__(256) void k_locate_small(const S* __restrict__ sa,
                                                      const int64_t* __restrict__ lr,
                                                      const uint64_t* __restrict__ oo, uint64_t P,
                                                      uint64_t* __restrict__ pos, uint64_t* big,
                                                      unsigned long long* nbig) {
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (uint64_t)gridDim.x * 256) {
    const int64_t l = lr[2 * p];
    if (l < 0) continue;
    const uint64_t c = (uint64_t)(lr[2 * p + 1] - l + 1);
    if (c > kSmallOcc) {
      big[atomicAdd(nbig, 1ull)] = p;
      continue;
    }
    const uint64_t o = oo[p];
    for (uint64_t i = 0; i < c; ++i) pos[o + i] = sa[l + i];
  }
}

template <typename S>
__global__ __launch_bounds__(256) void k_locate_big(const S* __restrict__ sa,
                                                    const int64_t* __restrict__ lr,
                                                    const uint64_t* __restrict__ oo,
                                                    const uint64_t* __restrict__ big,
                                                    const unsigned long long* __restrict__ nbig,
                                                    uint64_t* __restrict__ pos) {
  const uint64_t nb = *nbig;
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t p = big[b];
    const uint64_t l = (uint64_t)lr[2 * p];
    const uint64_t c = (uint64_t)(lr[2 * p + 1] + 1) - l;
    const uint64_t o = oo[p];
    for (uint64_t i = threadIdx.x; i < c; i += 256) pos[o + i] = sa[l + i];
  }
}

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace

void build_wt(Index& ix) {
  if (!ix.have_bwt) throw ApiError{-3, "build_wt: BWT not built"};
  if (ix.sharded) throw ApiError{-3, "build_wt: a sharded index holds only a slice of the BWT"};
  compute_alphabet(ix);
  hipStream_t s = ix.stream;
  const uint64_t n = ix.n;
  const int sigma = ix.sigma;
  int L = 0;
  while ((1 << L) < sigma) ++L;
  if (L > kMaxLevels) throw ApiError{-6, "alphabet too large"};
  ix.wt_levels = L;

  // host tables: node of every code at every depth
  WtTables& T = ix.tabs;
  memset(&T, 0, sizeof(T));
  for (int c = 0; c < sigma; ++c) {
    int lo = 0, hi = sigma, dep = 0;
    for (int d = 0; d < L; ++d) {
      T.start[d][c] = ix.Ccode[lo];
      if (hi - lo <= 1) {  // leaf reached: bit 0, stays in place
        T.bit[d][c] = 0;
        T.zeros[d][c] = ix.Ccode[hi] - ix.Ccode[lo];
        continue;
      }
      const int mid = lo + (hi - lo) / 2;
      T.zeros[d][c] = ix.Ccode[mid] - ix.Ccode[lo];
      dep = d + 1;
      if (c >= mid) { T.bit[d][c] = 1; lo = mid; }
      else { T.bit[d][c] = 0; hi = mid; }
    }
    T.depth[c] = (uint8_t)dep;
  }

  ix.wt_obn.ensure(kMaxLevels * 256 * 8);
  ix.wt_rbase.ensure(kMaxLevels * 256 * 8);
  ix.wt_bit.ensure(kMaxLevels * 256);
  ix.wt_depth.ensure(256);
  ix.wt_code.ensure(256 * 2);
  ix.wt_C.ensure(257 * 8);
  HK_HIP(hipMemsetAsync(ix.wt_obn.p, 0, kMaxLevels * 256 * 8, s));
  HK_HIP(hipMemsetAsync(ix.wt_rbase.p, 0, kMaxLevels * 256 * 8, s));
  HK_HIP(hipMemcpyAsync(ix.wt_bit.p, T.bit, sizeof(T.bit), hipMemcpyHostToDevice, s));
  HK_HIP(hipMemcpyAsync(ix.wt_depth.p, T.depth, 256, hipMemcpyHostToDevice, s));
  HK_HIP(hipMemcpyAsync(ix.wt_code.p, ix.code_of, 512, hipMemcpyHostToDevice, s));
  HK_HIP(hipMemcpyAsync(ix.wt_C.p, ix.Ccode, 257 * 8, hipMemcpyHostToDevice, s));
  DevBuf tab_in;
  tab_in.ensure(2 * kMaxLevels * 256 * 8);
  HK_HIP(hipMemcpyAsync(tab_in.p, T.start, sizeof(T.start), hipMemcpyHostToDevice, s));
  HK_HIP(hipMemcpyAsync(tab_in.as<uint8_t>() + sizeof(T.start), T.zeros, sizeof(T.zeros),
                        hipMemcpyHostToDevice, s));

  const uint64_t nlines = n / kLineBits + 1;
  ix.wt_nlines = nlines;
  if (L > 0) {
    ix.seq[0].ensure(n + 64);
    ix.seq[1].ensure(n + 64);
    // level 0 reads the BWT bytes: byte -> level-0 bit and byte -> dense code tables; deeper levels
    // read dense codes (identity code table)
    uint8_t lut0[2][256];
    for (int b = 0; b < 256; ++b) {
      const int c = ix.code_of[b];
      lut0[0][b] = c < 0 ? 0 : T.bit[0][c];
      lut0[1][b] = (uint8_t)(c < 0 ? 0 : c);
    }
    uint8_t ident[256];
    for (int b = 0; b < 256; ++b) ident[b] = (uint8_t)b;
    ix.wt_lut.ensure(3 * 256);
    HK_HIP(hipMemcpyAsync(ix.wt_lut.p, lut0, sizeof(lut0), hipMemcpyHostToDevice, s));
    HK_HIP(hipMemcpyAsync(ix.wt_lut.as<uint8_t>() + 512, ident, 256, hipMemcpyHostToDevice, s));
    ix.tile_b.ensure(nlines * 4 + 16);
    ix.tile_a.ensure(nlines * 8 + 16);
    int cur = 0;
    const unsigned gl = grid_for(ceil_div(nlines, WT_G), 4, 8192);
    for (int d = 0; d < L; ++d) {
      ix.wt_lines[d].ensure(nlines * 64);
      uint64_t* lines = ix.wt_lines[d].as<uint64_t>();
      const uint8_t* in = d == 0 ? ix.bwt.as<uint8_t>() : ix.seq[cur].as<uint8_t>();
      {
        TimedLaunch t(ix.timer, "wt_bits", (double)n * (1 + 1.0 / 8));
        k_wt_bits<<<gl, 256, 0, s>>>(in, n, d == 0 ? ix.wt_lut.as<uint8_t>() : ix.wt_bit.as<uint8_t>() + d * 256,
                                     lines, ix.tile_b.as<uint32_t>(), nlines);
        HK_HIP(hipGetLastError());
      }
      scan_exclusive_u32_to_u64(ix.sw, ix.tile_b.as<uint32_t>(), ix.tile_a.as<uint64_t>(), nlines, false, s);
      k_wt_fill<<<grid_for(nlines), 256, 0, s>>>(lines, ix.tile_a.as<uint64_t>(), nlines);
      HK_HIP(hipGetLastError());
      k_wt_tables<<<1, 256, 0, s>>>(lines, sigma, tab_in.as<uint64_t>() + d * 256,
                                    tab_in.as<uint64_t>() + kMaxLevels * 256 + d * 256,
                                    ix.wt_obn.as<uint64_t>() + d * 256, ix.wt_rbase.as<uint64_t>() + d * 256);
      HK_HIP(hipGetLastError());
      if (d + 1 < L) {
        TimedLaunch t(ix.timer, "wt_partition", (double)n * (1 + 1 + 1.0 / 8));
        uint8_t* outp = d == 0 ? ix.seq[0].as<uint8_t>() : ix.seq[cur ^ 1].as<uint8_t>();
        k_wt_partition<<<gl, 256, 0, s>>>(in, outp, n, lines, nlines, ix.wt_obn.as<uint64_t>() + d * 256,
                                          ix.wt_rbase.as<uint64_t>() + d * 256,
                                          ix.wt_lut.as<uint8_t>() + (d == 0 ? 256 : 512));
        HK_HIP(hipGetLastError());
        if (d > 0) cur ^= 1;
      }
    }
  }
  HK_HIP(hipStreamSynchronize(s));
  ix.have_wt = true;
}

void query_count(Index& ix, const uint8_t* d_pats, const uint64_t* d_offs, uint64_t P, int64_t* d_lr,
                 uint64_t* d_cnt) {
  if (!ix.have_wt || ix.sharded) throw ApiError{-3, "count: wavelet tree not built"};
  if (!P) return;
  TimedLaunch t(ix.timer, "fm_count", 0.0);
  k_count<<<grid_for(P, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_pats, d_offs, P, d_lr, d_cnt);
  HK_HIP(hipGetLastError());
}

void query_locate_gather(Index& ix, const int64_t* d_lr, const uint64_t* d_occ_offs, uint64_t P,
                         uint64_t* d_pos) {
  if (!ix.have_sa && ix.have_samples) return sampled_locate_gather(ix, d_lr, d_occ_offs, P, d_pos);
  if (!ix.have_sa) throw ApiError{-3, "locate: suffix array not built"};
  if (!P) return;
  hipStream_t s = ix.stream;
  ix.tile_c.ensure((P + 2) * 8);
  ix.small.ensure(8192);
  unsigned long long* nbig = ix.small.as<unsigned long long>() + 512;   // byte 4096: clear of the build LUTs
  HK_HIP(hipMemsetAsync(nbig, 0, 8, s));
  TimedLaunch t(ix.timer, "fm_locate", 0.0);
  if (ix.sa_pos64) {   // replicated sharded SA of a text with n >= 2^32
    k_locate_small<uint64_t><<<grid_for(P, 256, 65535), 256, 0, s>>>(ix.sa.as<uint64_t>(), d_lr, d_occ_offs, P,
                                                                     d_pos, ix.tile_c.as<uint64_t>(), nbig);
    HK_HIP(hipGetLastError());
    k_locate_big<uint64_t><<<1024, 256, 0, s>>>(ix.sa.as<uint64_t>(), d_lr, d_occ_offs, ix.tile_c.as<uint64_t>(),
                                                nbig, d_pos);
  } else {
    k_locate_small<uint32_t><<<grid_for(P, 256, 65535), 256, 0, s>>>(ix.sa.as<uint32_t>(), d_lr, d_occ_offs, P,
                                                                     d_pos, ix.tile_c.as<uint64_t>(), nbig);
    HK_HIP(hipGetLastError());
    k_locate_big<uint32_t><<<1024, 256, 0, s>>>(ix.sa.as<uint32_t>(), d_lr, d_occ_offs, ix.tile_c.as<uint64_t>(),
                                                nbig, d_pos);
  }
  HK_HIP(hipGetLastError());
}

void query_rank(Index& ix, const uint8_t* d_c, const uint64_t* d_i, uint64_t k, uint64_t* d_out) {
  if (!ix.have_wt) throw ApiError{-3, "rank: wavelet tree not built"};
  if (!k) return;
  k_rank<<<grid_for(k, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_c, d_i, k, d_out);
  HK_HIP(hipGetLastError());
}

void wt_level_words(Index& ix, int depth, uint64_t* d_words) {
  const uint64_t nw = ceil_div(ix.n, 64);
  k_wt_extract<<<grid_for(nw), 256, 0, ix.stream>>>(ix.wt_lines[depth].as<uint64_t>(), nw, d_words);
  HK_HIP(hipGetLastError());
}

}  // namespace hk
