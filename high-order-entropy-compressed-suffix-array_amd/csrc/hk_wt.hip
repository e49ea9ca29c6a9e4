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

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <type_traits>
#include <vector>

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

// Level kernels: every lane reads 16 consecutive symbols with one 16-B load, so a wave reads 1 KiB
// per instruction (the byte-per-lane forms moved 64 B per instruction and ran at 18-26 % of HBM,
// profiles/r2b_sq_counters.json).  16 rank lines hold 16 x 448 = 7 x 1024 symbols, so 7 loads per
// lane cover 16 whole lines, and every 64-bit data word is the 16-bit slices of 4 adjacent lanes.
// Per level one u16 table maps the input symbol (BWT byte at level 0, dense code below) to
// bit << 15 | node << 8 | code (a depth-d node index is < 2^d <= 128).
constexpr int WT_V = 16;   // lines per wave group

__device__ __forceinline__ uint32_t byte_of(const uint4& v, int i) {
  const uint32_t w = i < 4 ? v.x : i < 8 ? v.y : i < 12 ? v.z : v.w;
  return (w >> (8 * (i & 3))) & 255u;
}

// Small alphabets (sigma <= 8, every byte < 128): four symbols per VALU step.  Level 0 maps BWT
// bytes to dense codes by per-byte threshold compares on whole words (code = number of code-start
// bytes <= the byte; bit 7 of (byte | 0x80) - t is byte >= t, no borrow between bytes); the level's
// bit of each code comes from an 8-entry byte table by v_perm_b32, and one multiply gathers the
// four 0/1 bytes into 4 bits (b0 | b1 << 1 | b2 << 2 | b3 << 3 at bits 24..27).
struct WtSmall {
  uint32_t lut_lo, lut_hi;   // bit of codes 0..3 / 4..7, one byte each
  uint32_t thr[7];           // code-start byte of codes 1..7, replicated to the 4 bytes
  int nthr;                  // sigma - 1 at level 0, 0 below (the input is already codes)
  int p2sh;                  // sigma = 256 (dense code = byte, a perfect tree): the level's bit is
                             // (byte >> p2sh) & 1, four symbols per VALU step; -1 otherwise
};

// bits of four bytes at one bit position, gathered as in small_bits4
__device__ __forceinline__ uint32_t p2_bits4(uint32_t w, int sh) {
  return ((((w >> sh) & 0x01010101u) * 0x01020408u) >> 24) & 15u;
}

__device__ __forceinline__ uint32_t small_codes(uint32_t x, const WtSmall& a) {
  if (!a.nthr) return x;
  const uint32_t xo = x | 0x80808080u;
  uint32_t c = 0;
#pragma unroll
  for (int k = 0; k < 7; ++k)
    if (k < a.nthr) c += ((xo - a.thr[k]) & 0x80808080u) >> 7;
  return c;
}

// (bytes past n are arbitrary: a selector of 8..15 yields 0x00 / 0xFF / sign bytes, so every byte is
// cut to its bit 0 before the multiply, or its carries would reach the neighbours' bits)
__device__ __forceinline__ uint32_t small_bits4(uint32_t codes, const WtSmall& a) {
  const uint32_t b = __builtin_amdgcn_perm(a.lut_hi, a.lut_lo, codes) & 0x01010101u;
  return ((b * 0x01020408u) >> 24) & 15u;
}

// one wave per WT_V lines: data words from lane slices, line popcounts (word 0 later receives the
// ones-before count)
template <bool SMALL>
__global__ __launch_bounds__(256) void k_wt_bits(const uint8_t* __restrict__ S, uint64_t n,
                                                 const uint16_t* __restrict__ lut, uint64_t* __restrict__ lines,
                                                 uint32_t* __restrict__ line_pop, uint64_t nlines, WtSmall sa) {
  __shared__ uint16_t LU[256];
  __shared__ uint8_t Q[4][7 * WT_V];   // popcount of every data word of the group
  LU[threadIdx.x] = lut[threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t ngroups = (nlines + WT_V - 1) / WT_V;
  for (uint64_t g = (uint64_t)blockIdx.x * 4 + wv; g < ngroups; g += (uint64_t)gridDim.x * 4) {
    const uint64_t base = g * WT_V * kLineBits;
    uint4 v[7];
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const uint64_t j = base + (uint64_t)it * 1024 + lane * 16u;
      v[it] = j < n ? *reinterpret_cast<const uint4*>(S + j) : make_uint4(0, 0, 0, 0);   // 64 pad bytes past n
    }
#pragma unroll
    for (int it = 0; it < 7; ++it) {
      const uint64_t j = base + (uint64_t)it * 1024 + lane * 16u;
      uint32_t bits = 0;
      if (SMALL) {
        const uint32_t w4[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) bits |= small_bits4(small_codes(w4[k], sa), sa) << (4 * k);
        if (j + 16 > n) bits &= j >= n ? 0u : (1u << (uint32_t)(n - j)) - 1;
      } else if (sa.p2sh >= 0) {
        const uint32_t w4[4] = {v[it].x, v[it].y, v[it].z, v[it].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) bits |= p2_bits4(w4[k], sa.p2sh) << (4 * k);
        if (j + 16 > n) bits &= j >= n ? 0u : (1u << (uint32_t)(n - j)) - 1;
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) bits |= (((uint32_t)LU[byte_of(v[it], i)] >> 15) & 1u) << i;
        if (j + 16 > n) bits &= j >= n ? 0u : (1u << (uint32_t)(n - j)) - 1;   // the text's last chunk
      }
      const uint64_t w = (uint64_t)bits | ((uint64_t)__shfl_down(bits, 1, 64) << 16) |
                         ((uint64_t)__shfl_down(bits, 2, 64) << 32) | ((uint64_t)__shfl_down(bits, 3, 64) << 48);
      if ((lane & 3u) == 0) {
        const uint32_t q = it * 16 + (lane >> 2);   // data word of the group, line q / 7
        const uint64_t li = g * WT_V + q / 7;
        if (li < nlines) lines[li * 8 + 1 + q % 7] = w;
        Q[wv][q] = (uint8_t)__popcll(w);
      }
    }
    __builtin_amdgcn_wave_barrier();
    if (lane < WT_V) {
      const uint64_t li = g * WT_V + lane;
      uint32_t pop = 0;
#pragma unroll
      for (int k = 0; k < 7; ++k) pop += Q[wv][lane * 7 + k];
      if (li < nlines) line_pop[li] = pop;
    }
    __builtin_amdgcn_wave_barrier();
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

// stable partition of level d's sequence into level d+1.  Each wave takes a contiguous run of
// 1024-symbol spans; a span's ones-before come from its line (count word + the data words before
// it) and a wave scan.  Spans inside one node (all but the <= 2^d listed in `bspan`) extend two
// contiguous output runs (zeros, ones): their bytes are staged in LDS at the destination's offset
// mod 16, whole aligned 16-B chunks are written as they fill and the partial last chunk is carried
// to the next span, so bytes are stored one at a time only where a run starts or ends.  A span
// across a node boundary ends both runs and scatters its bytes.  VALU per span was the limit of the
// byte-edge form (722 wave-instructions per span, tools/gpu_pmc_kernel.sh).
struct WtRun {
  uint64_t rd;     // destination of staging byte 0 (16-aligned)
  uint32_t fill;   // staged bytes [own0, fill) not yet written
  uint32_t own0;   // first owned staging byte of the run's first chunk
  bool live;
};

__device__ __forceinline__ void wt_run_flush(WtRun& r, const uint8_t* st, uint8_t* __restrict__ out, uint32_t lane) {
  if (r.live && lane < 16 && lane >= r.own0 && lane < r.fill) out[r.rd + lane] = st[lane];
  r.live = false;
}

template <bool SMALL>
__global__ __launch_bounds__(256) void k_wt_partition(const uint8_t* __restrict__ S, uint8_t* __restrict__ out,
                                                      uint64_t n, const uint64_t* __restrict__ lines,
                                                      const uint64_t* __restrict__ obn,
                                                      const uint64_t* __restrict__ rbase,
                                                      const uint16_t* __restrict__ lut,
                                                      const uint64_t* __restrict__ bspan, uint32_t nbspan,
                                                      int translate, WtSmall sa) {
  __shared__ uint64_t OB[256], RB[256];
  __shared__ uint16_t LU[256];
  __shared__ uint64_t BS[256];
  __shared__ __attribute__((aligned(16))) uint8_t ST[4][2][1024 + 48];
  OB[threadIdx.x] = obn[threadIdx.x];
  RB[threadIdx.x] = rbase[threadIdx.x];
  LU[threadIdx.x] = lut[threadIdx.x];
  BS[threadIdx.x] = threadIdx.x < nbspan ? bspan[threadIdx.x] : ~0ull;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t nspans = (n + 1023) / 1024, nw = (uint64_t)gridDim.x * 4;
  const uint64_t per = (nspans + nw - 1) / nw, gw = (uint64_t)blockIdx.x * 4 + wv;
  const uint64_t t0 = gw * per, t1 = t0 + per < nspans ? t0 + per : nspans;
  WtRun run[2] = {{0, 0, 0, false}, {0, 0, 0, false}};
  uint32_t bi = 0;   // boundary spans below t
  while (bi < nbspan && BS[bi] < t0) ++bi;
  // ones before the wave's first span from its rank line; after that the wave carries the count
  // (its spans are contiguous), so no span waits on a line read, and the next span's symbols are
  // loaded while this one is partitioned (0.76 -> 0.68 ms per 1 GiB level against a line read per span)
  uint64_t onesbase = 0;
  if (t0 < t1) {
    const uint64_t base = t0 * 1024, li0 = base / kLineBits;
    const uint32_t wi0 = (uint32_t)(base - li0 * kLineBits) / 64;
    uint64_t part = 0;
    if (lane < wi0) part = (uint64_t)__popcll(lines[li0 * 8 + 1 + lane]);
    else if (lane == 7) part = lines[li0 * 8];
    onesbase = wave_sum<uint64_t>(part);
  }
  // unconditional loads (a load under a runtime condition makes hipcc wait for every load in flight
  // before it): past the text the address is clamped to readable bytes, which the valid mask drops
  const uint64_t jmax = n & ~15ull;
  auto load_span = [&](uint64_t t) {
    const uint64_t j = t * 1024 + lane * 16u;
    return *reinterpret_cast<const uint4*>(S + (j < n ? j : jmax));
  };
  uint4 vnext = t0 < t1 ? load_span(t0) : make_uint4(0, 0, 0, 0);
  for (uint64_t t = t0; t < t1; ++t) {
    const uint64_t base = t * 1024, j0 = base + lane * 16u;
    const uint4 vv = vnext;
    vnext = load_span(t + 1 < t1 ? t + 1 : t);
    const uint32_t nv = j0 >= n ? 0u : (n - j0 >= 16 ? 16u : (uint32_t)(n - j0));
    const uint32_t valid = nv == 16 ? 0xFFFFu : (1u << nv) - 1;
    uint32_t bits = 0;
    uint32_t cw[4] = {vv.x, vv.y, vv.z, vv.w};
    if (SMALL) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        cw[k] = small_codes(cw[k], sa);
        bits |= small_bits4(cw[k], sa) << (4 * k);
      }
    } else if (sa.p2sh >= 0) {   // sigma = 256: codes are the bytes, bits by shifts
#pragma unroll
      for (int k = 0; k < 4; ++k) bits |= p2_bits4(cw[k], sa.p2sh) << (4 * k);
    } else if (translate) {   // level 0: BWT bytes -> dense codes
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        uint32_t o = 0;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const uint32_t e = LU[(cw[k] >> (8 * i)) & 255u];
          bits |= (e >> 15) << (4 * k + i);
          o |= (e & 255u) << (8 * i);
        }
        cw[k] = o;
      }
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) bits |= ((uint32_t)LU[(cw[i >> 2] >> (8 * (i & 3))) & 255u] >> 15) << i;
    }
    bits &= valid;
    const uint32_t ones = __popc(bits), nz = nv - ones;
    const uint32_t oinc = wave_incl_sum<uint32_t>(ones), zinc = wave_incl_sum<uint32_t>(nz);
    const uint32_t opre = oinc - ones, zpre = zinc - nz;
    const uint64_t onesnext = onesbase + (uint32_t)__shfl(oinc, 63, 64);   // the next span's ones before
    const uint32_t c0 = (uint32_t)__shfl(cw[0] & 255u, 0, 64);   // code of the span's first symbol
    const bool boundary = bi < nbspan && BS[bi] == t;
    if (boundary) ++bi;
    if (!boundary) {
      const uint32_t tot[2] = {(uint32_t)__shfl(zinc, 63, 64), (uint32_t)__shfl(oinc, 63, 64)};
      const uint64_t dst[2] = {base - onesbase + OB[c0], RB[c0] + onesbase};
      uint32_t at[2];
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        WtRun& R = run[r];
        if (!R.live || R.rd + R.fill != dst[r]) {   // a new run (first span, or after a boundary)
          wt_run_flush(R, ST[wv][r], out, lane);
          R.rd = dst[r] & ~15ull;
          R.fill = R.own0 = (uint32_t)(dst[r] & 15u);
          R.live = true;
        }
        at[r] = R.fill;
      }
      // one byte store per symbol: the two staging runs are adjacent, so the destination is
      // zeros' slot zk or (1024 + 48) + ones' slot ok
      uint32_t zk = at[0] + zpre, ok = at[1] + opre;
      uint8_t* const st0 = ST[wv][0];
      constexpr uint32_t kRun1 = (uint32_t)(sizeof(ST[0][0]));
      if (base + 1024 <= n) {   // a full span: every lane's 16 symbols are valid, no store guard
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t b = (bits >> i) & 1u;
          st0[b ? kRun1 + ok : zk] = (uint8_t)(cw[i >> 2] >> (8 * (i & 3)));
          ok += b;
          zk += 1u - b;
        }
      } else {
#pragma unroll
        for (int i = 0; i < 16; ++i) {
          const uint32_t b = (bits >> i) & 1u;
          if ((valid >> i) & 1u) st0[b ? kRun1 + ok : zk] = (uint8_t)(cw[i >> 2] >> (8 * (i & 3)));
          ok += b;
          zk += ((valid >> i) & 1u) - b;
        }
      }
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        WtRun& R = run[r];
        const uint32_t end = R.fill + tot[r], full = end / 16;
        uint8_t* st = ST[wv][r];
        for (uint32_t ch = lane; ch < full; ch += 64) {
          const uint4 q = *reinterpret_cast<const uint4*>(st + ch * 16);
          if (ch == 0 && R.own0) {
#pragma unroll
            for (int b = 0; b < 16; ++b)
              if ((uint32_t)b >= R.own0) out[R.rd + b] = (uint8_t)byte_of(q, b);
          } else {
            *reinterpret_cast<uint4*>(out + R.rd + ch * 16) = q;
          }
        }
        if (full) {
          R.own0 = 0;
          R.rd += (uint64_t)full * 16;
          __builtin_amdgcn_wave_barrier();
          if (lane == 0) *reinterpret_cast<uint4*>(st) = *reinterpret_cast<const uint4*>(st + full * 16);
        }
        R.fill = end - full * 16;
      }
      __builtin_amdgcn_wave_barrier();
    } else {
      wt_run_flush(run[0], ST[wv][0], out, lane);
      wt_run_flush(run[1], ST[wv][1], out, lane);
      uint64_t ob = onesbase + opre;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if ((valid >> i) & 1u) {
          const uint8_t c = (uint8_t)(cw[i >> 2] >> (8 * (i & 3)));
          const uint64_t j = j0 + i;
          if ((bits >> i) & 1u) out[RB[c] + ob++] = c;
          else out[j - ob + OB[c]] = c;
        }
      }
    }
    onesbase = onesnext;
  }
  __builtin_amdgcn_wave_barrier();
  wt_run_flush(run[0], ST[wv][0], out, lane);
  wt_run_flush(run[1], ST[wv][1], out, lane);
}

__global__ __launch_bounds__(256) void k_wt_extract(const uint64_t* __restrict__ lines, uint64_t nwords,
                                                    uint64_t* __restrict__ words) {
  for (uint64_t w = (uint64_t)blockIdx.x * 256 + threadIdx.x; w < nwords; w += (uint64_t)gridDim.x * 256)
    words[w] = lines[(w / 7) * 8 + 1 + (w % 7)];
}

// ------------------------------------------------------------ queries
// ------------------------------------------------------------ flat occ directory (sigma <= 8)
// The reference's find_range takes occ(c, i) from its dense occ table (utils/utils.py:26-32,
// csa/enhanced_fm_index.py:34-40).  For small alphabets the batched count reads the same values from
// a directory of the BWT instead of walking the wavelet tree: 64-B lines of OC_S = 128 symbols, each
// 8 u16 counts (occurrences of every code before the line, relative to its superblock of 256 lines)
// and the codes as 3 bit-planes of 128 bits; per superblock 8 u64 counts.  occ(c, x) = superblock
// count + line count + popcount of the codes equal to c below x in the line: one 64-B line per rank
// (the WT needs one per level), 0.5 B per symbol.
constexpr int OC_S = 128, OC_LPS = 256;

// one workgroup per superblock, 32 lines per round: 8 threads per line, 16 symbols each (one 16-byte
// load: the wave's loads are contiguous), whose plane bits are assembled in LDS with the line's
// counts; exclusive counts inside the superblock, superblock totals per code (scanned afterwards)
__global__ __launch_bounds__(256) void k_occ_lines(const uint8_t* __restrict__ bwt, uint64_t n,
                                                   const int16_t* __restrict__ code, uint64_t nlines,
                                                   uint4* __restrict__ lines, uint64_t* __restrict__ sbt) {
  __shared__ int16_t CD[256];
  __shared__ uint4 img[32 * 4];
  __shared__ uint32_t lc[32][8];
  __shared__ uint32_t carry[8], tot[8];
  const uint32_t tid = threadIdx.x, ln = tid >> 3, j = tid & 7;
  CD[tid] = code[tid];
  if (tid < 8) carry[tid] = 0;
  __syncthreads();
  uint16_t* const img16 = reinterpret_cast<uint16_t*>(img);
  for (int it = 0; it < OC_LPS / 32; ++it) {
    const uint64_t l0 = (uint64_t)blockIdx.x * OC_LPS + (uint64_t)it * 32;
    if (l0 >= nlines) break;   // uniform
    const uint64_t li = l0 + ln, p = li * OC_S + 16 * j;
    // bytes past n: code 0 (after every queried position; the BWT holds n + 64 bytes)
    const uint4 v = li < nlines && p < n ? *reinterpret_cast<const uint4*>(bwt + p) : make_uint4(0, 0, 0, 0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t pq[3] = {0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int c = p + i < n ? CD[(w[i >> 2] >> (8 * (i & 3))) & 255u] : 0;
#pragma unroll
      for (int q = 0; q < 3; ++q) pq[q] |= (uint32_t)((c >> q) & 1) << i;
    }
    // counts of the 8 codes in these 16 symbols (pairwise plane products), one byte each, summed over
    // the line's 8 threads (<= 128 per byte, no carry)
    const uint32_t n0 = ~pq[0] & 0xFFFFu, n1 = ~pq[1] & 0xFFFFu, n2 = ~pq[2] & 0xFFFFu;
    const uint32_t a[4] = {n0 & n1, pq[0] & n1, n0 & pq[1], pq[0] & pq[1]};
    uint64_t cb = 0;
#pragma unroll
    for (int c = 0; c < 8; ++c) cb |= (uint64_t)__popc(a[c & 3] & ((c & 4) ? pq[2] : n2)) << (8 * c);
    cb += __shfl_xor(cb, 1, 64);
    cb += __shfl_xor(cb, 2, 64);
    cb += __shfl_xor(cb, 4, 64);
    lc[ln][j] = (uint32_t)(cb >> (8 * j)) & 255u;   // this line's count of code j
#pragma unroll
    for (int q = 0; q < 3; ++q) img16[ln * 32 + 8 * (1 + q) + j] = (uint16_t)pq[q];
    __syncthreads();
    {   // thread (code tid >> 5, line tid & 31): the code's occurrences before the line (32-lane scan)
      const uint32_t c8 = tid >> 5, l32 = tid & 31u, v0 = lc[l32][c8];
      uint32_t inc = v0;
#pragma unroll
      for (int d = 1; d < 32; d <<= 1) {
        const uint32_t t = __shfl_up(inc, d, 32);
        inc += l32 >= (uint32_t)d ? t : 0u;
      }
      img16[l32 * 32 + c8] = (uint16_t)(carry[c8] + inc - v0);
      if (l32 == 31) tot[c8] = inc;
    }
    __syncthreads();
    if (tid < 8) carry[tid] += tot[tid];
    if (tid < 128 && l0 + (tid >> 2) < nlines) lines[l0 * 4 + tid] = img[tid];
    __syncthreads();
  }
  if (tid < 8) sbt[(uint64_t)tid * gridDim.x + blockIdx.x] = carry[tid];   // [code][superblock]
}

__device__ __forceinline__ uint64_t occ_rank(const uint4* __restrict__ lines, const uint64_t* __restrict__ sb,
                                             uint64_t nsb, int c, uint64_t x) {
  const uint64_t li = x >> 7;
  const uint32_t off = (uint32_t)x & 127u;
  const uint4* L = lines + li * 4;
  const uint4 h = L[0], a = L[1], b = L[2], d = L[3];
  const uint32_t hw = c < 4 ? (c < 2 ? h.x : h.y) : (c < 6 ? h.z : h.w);
  const uint32_t cnt = (hw >> (16 * (c & 1))) & 0xFFFFu;
  const uint64_t p00 = ((uint64_t)a.y << 32) | a.x, p01 = ((uint64_t)a.w << 32) | a.z;
  const uint64_t p10 = ((uint64_t)b.y << 32) | b.x, p11 = ((uint64_t)b.w << 32) | b.z;
  const uint64_t p20 = ((uint64_t)d.y << 32) | d.x, p21 = ((uint64_t)d.w << 32) | d.z;
  uint64_t m0 = ((c & 1) ? p00 : ~p00) & ((c & 2) ? p10 : ~p10) & ((c & 4) ? p20 : ~p20);
  uint64_t m1 = ((c & 1) ? p01 : ~p01) & ((c & 2) ? p11 : ~p11) & ((c & 4) ? p21 : ~p21);
  m0 &= off >= 64 ? ~0ull : ((1ull << off) - 1ull);
  m1 &= off > 64 ? ((1ull << (off - 64)) - 1ull) : 0ull;
  return sb[(uint64_t)c * nsb + (li >> 8)] + cnt + (uint64_t)(__popcll(m0) + __popcll(m1));
}

// Two-level 16-ary occ directory (8 < sigma <= 256).  With g = max(0, levels - 4), level 0 is the
// BWT mapped to the WT node of each code at depth g (<= 16 nodes, each of <= 16 codes) and level 1 is
// the WT's depth-g sequence (the BWT stably partitioned by those nodes) mapped to code - node start
// (g = 0: the BWT's codes).  With h, v the node and value of code c, B[h] the node's start (= C of its
// first code) and A[c] = C[c] - (values v in the nodes before h):
//   LF(c, x) = C[c] + occ(c, x) = A[c] + rank1_v(B[h] + rank0_h(x))
// so an LF step reads two 64-B lines (one for g = 0) where the WT reads one per level.
// Line: 64 symbols in 64 B: the 16 values' u16 counts before the line (relative to its superblock of
// NB_LPS lines) + 4 bit-planes of 64 bits; per superblock 16 u64 counts, [value][superblock].
constexpr int NB_S = 64, NB_LPS = 1024;

// one workgroup per superblock, 64 lines a round: 4 threads per line, 16 symbols each (one 16-B load)
__global__ __launch_bounds__(256) void k_nib_lines(const uint8_t* __restrict__ seq, uint64_t n,
                                                   const uint8_t* __restrict__ map, uint64_t nlines,
                                                   uint4* __restrict__ lines, uint64_t* __restrict__ sbt) {
  __shared__ uint8_t MP[256];
  __shared__ uint4 img[64 * 4];
  __shared__ uint32_t lc[64][17];
  const uint32_t tid = threadIdx.x, ln = tid >> 2, j = tid & 3, lane = tid & 63, wv = tid >> 6;
  MP[tid] = map[tid];
  uint32_t carry[4] = {0, 0, 0, 0};   // this wave's values 4 wv .. 4 wv + 3 (wave-uniform)
  __syncthreads();
  uint16_t* const img16 = reinterpret_cast<uint16_t*>(img);
  for (int it = 0; it < NB_LPS / 64; ++it) {
    const uint64_t l0 = (uint64_t)blockIdx.x * NB_LPS + (uint64_t)it * 64;
    if (l0 >= nlines) break;   // uniform
    const uint64_t li = l0 + ln, p = li * NB_S + 16 * j;
    // symbols past n: value 0 (after every queried position; the input holds n + 64 bytes)
    const uint4 v = li < nlines && p < n ? *reinterpret_cast<const uint4*>(seq + p) : make_uint4(0, 0, 0, 0);
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    uint32_t pq[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const uint32_t x = p + i < n ? MP[(w[i >> 2] >> (8 * (i & 3))) & 255u] : 0u;
#pragma unroll
      for (int q = 0; q < 4; ++q) pq[q] |= ((x >> q) & 1u) << i;
    }
    // the 16 values' counts in these 16 symbols, a byte each (<= 64 over the line's 4 threads)
    const uint32_t nq[4] = {~pq[0] & 0xFFFFu, ~pq[1] & 0xFFFFu, ~pq[2] & 0xFFFFu, ~pq[3] & 0xFFFFu};
    const uint32_t a01[4] = {nq[0] & nq[1], pq[0] & nq[1], nq[0] & pq[1], pq[0] & pq[1]};
    const uint32_t a23[4] = {nq[2] & nq[3], pq[2] & nq[3], nq[2] & pq[3], pq[2] & pq[3]};
    uint32_t cb[4] = {0, 0, 0, 0};
#pragma unroll
    for (int x = 0; x < 16; ++x) cb[x >> 2] |= (uint32_t)__popc(a01[x & 3] & a23[x >> 2]) << (8 * (x & 3));
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      cb[k] += __shfl_xor(cb[k], 1, 64);
      cb[k] += __shfl_xor(cb[k], 2, 64);
    }
    // thread j records values 4j .. 4j + 3 of its line
#pragma unroll
    for (int k = 0; k < 4; ++k) lc[ln][4 * j + k] = (cb[j] >> (8 * k)) & 255u;
#pragma unroll
    for (int q = 0; q < 4; ++q) img16[ln * 32 + 16 + 4 * q + j] = (uint16_t)pq[q];
    __syncthreads();
    // wave wv, lane = line: the counts of values 4 wv + k before each line of the superblock
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t val = 4 * wv + k, x = lc[lane][val];
      const uint32_t inc = wave_incl_sum<uint32_t>(x);
      img16[lane * 32 + val] = (uint16_t)(carry[k] + inc - x);
      carry[k] += __shfl(inc, 63, 64);
    }
    __syncthreads();
    if (l0 + (tid >> 2) < nlines) lines[l0 * 4 + tid] = img[tid];
    __syncthreads();
  }
  if (lane < 4) sbt[(uint64_t)(4 * wv + lane) * gridDim.x + blockIdx.x] = lane == 0 ? carry[0] : lane == 1 ? carry[1]
                                                                          : lane == 2 ? carry[2] : carry[3];
}

// per value, the exclusive prefix of its superblock totals (in place; one workgroup per value)
__global__ __launch_bounds__(1024) void k_nib_sbscan(uint64_t* __restrict__ sbt, uint64_t nsb) {
  __shared__ uint64_t ws[16];
  uint64_t* const row = sbt + (uint64_t)blockIdx.x * nsb;
  const uint32_t tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  uint64_t carry = 0;
  for (uint64_t b = 0; b < nsb; b += 1024) {
    const uint64_t i = b + tid;
    const uint64_t x = i < nsb ? row[i] : 0;
    const uint64_t inc = wave_incl_sum<uint64_t>(x);
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      pre += k < (int)wv ? ws[k] : 0;
      tot += ws[k];
    }
    if (i < nsb) row[i] = carry + pre + inc - x;
    carry += tot;
    __syncthreads();
  }
}

__device__ __forceinline__ uint64_t nib_rank(const uint4* __restrict__ lines, const uint64_t* __restrict__ sb,
                                             uint64_t nsb, uint32_t v, uint64_t x) {
  const uint64_t li = x >> 6;
  const uint32_t off = (uint32_t)x & 63u;
  const uint4* L = lines + li * 4;
  const uint4 h = L[v >> 3], a = L[2], b = L[3];
  const uint32_t hw = (v & 4) ? ((v & 2) ? h.w : h.z) : ((v & 2) ? h.y : h.x);
  const uint32_t cnt = (hw >> (16 * (v & 1))) & 0xFFFFu;
  const uint64_t p0 = ((uint64_t)a.y << 32) | a.x, p1 = ((uint64_t)a.w << 32) | a.z;
  const uint64_t p2 = ((uint64_t)b.y << 32) | b.x, p3 = ((uint64_t)b.w << 32) | b.z;
  uint64_t m = ((v & 1) ? p0 : ~p0) & ((v & 2) ? p1 : ~p1) & ((v & 4) ? p2 : ~p2) & ((v & 8) ? p3 : ~p3);
  m &= (1ull << off) - 1ull;
  return sb[(uint64_t)v * nsb + (li >> 10)] + cnt + (uint64_t)__popcll(m);
}

// ranks of one value at two positions: a second line (and superblock count) only for lanes whose
// positions fall in different lines (a narrow range, as most backward-search steps past the first
// few symbols, reads one line)
__device__ __forceinline__ void nib_rank2(const uint4* __restrict__ lines, const uint64_t* __restrict__ sb,
                                          uint64_t nsb, uint32_t v, uint64_t xl, uint64_t xr, uint64_t& rl,
                                          uint64_t& rr) {
  const uint64_t ll = xl >> 6, lr = xr >> 6;
  const uint4* L = lines + ll * 4;
  uint4 h = L[v >> 3], a = L[2], b = L[3];
  uint64_t s0 = sb[(uint64_t)v * nsb + (ll >> 10)], s1 = s0;
  auto one = [&](const uint4& hh, const uint4& aa, const uint4& bb, uint64_t sbv, uint32_t off) -> uint64_t {
    const uint32_t hw = (v & 4) ? ((v & 2) ? hh.w : hh.z) : ((v & 2) ? hh.y : hh.x);
    const uint32_t cnt = (hw >> (16 * (v & 1))) & 0xFFFFu;
    const uint64_t p0 = ((uint64_t)aa.y << 32) | aa.x, p1 = ((uint64_t)aa.w << 32) | aa.z;
    const uint64_t p2 = ((uint64_t)bb.y << 32) | bb.x, p3 = ((uint64_t)bb.w << 32) | bb.z;
    uint64_t m = ((v & 1) ? p0 : ~p0) & ((v & 2) ? p1 : ~p1) & ((v & 4) ? p2 : ~p2) & ((v & 8) ? p3 : ~p3);
    m &= (1ull << off) - 1ull;
    return sbv + cnt + (uint64_t)__popcll(m);
  };
  rl = one(h, a, b, s0, (uint32_t)xl & 63u);
  if (lr != ll) {
    const uint4* R = lines + lr * 4;
    h = R[v >> 3];
    a = R[2];
    b = R[3];
    s1 = sb[(uint64_t)v * nsb + (lr >> 10)];
  }
  rr = one(h, a, b, s1, (uint32_t)xr & 63u);
}

struct NibView {
  const uint4* l0 = nullptr;
  const uint64_t* sb0 = nullptr;
  const uint4* l1 = nullptr;
  const uint64_t* sb1 = nullptr;
  uint64_t nsb = 0;
  const uint8_t* tab = nullptr;   // grp[256] | val[256] | map0[256] | map1[256] | A u64[256] | B u64[16]
  int g = 0;
};

struct NibShared {
  uint64_t A[256];
  uint64_t B[16];
  uint8_t grp[256], val[256];
};

__device__ __forceinline__ void load_nib(NibShared& s, const NibView& v) {
  const uint32_t t = threadIdx.x;   // blockDim == 256
  s.grp[t] = v.tab[t];
  s.val[t] = v.tab[256 + t];
  s.A[t] = reinterpret_cast<const uint64_t*>(v.tab + 1024)[t];
  if (t < 16) s.B[t] = reinterpret_cast<const uint64_t*>(v.tab + 3072)[t];
}

// LF of the pair (xl, xr) for code c
__device__ __forceinline__ void nib_lf_pair(const NibView& v, const NibShared& s, int c, uint64_t& xl, uint64_t& xr) {
  uint64_t yl = xl, yr = xr;
  if (v.g) {
    const uint32_t h = s.grp[c];
    nib_rank2(v.l0, v.sb0, v.nsb, h, xl, xr, yl, yr);
    yl += s.B[h];
    yr += s.B[h];
  }
  uint64_t rl, rr;
  nib_rank2(v.l1, v.sb1, v.nsb, s.val[c], yl, yr, rl, rr);
  xl = s.A[c] + rl;
  xr = s.A[c] + rr;
}

__device__ __forceinline__ uint64_t nib_lf(const NibView& v, const NibShared& s, int c, uint64_t x) {
  uint64_t y = x;
  if (v.g) {
    const uint32_t h = s.grp[c];
    y = s.B[h] + nib_rank(v.l0, v.sb0, v.nsb, h, x);
  }
  return s.A[c] + nib_rank(v.l1, v.sb1, v.nsb, s.val[c], y);
}

// Batched backward search, one lane per pattern (csa/enhanced_fm_index.py:21-32): the state (xl, xr)
// is the half-open row range, a symbol outside the alphabet or an empty range ends the search.  With
// a k-mer table (K > 0) the last K symbols of a pattern take one lookup of the state they lead to
// from the full range (k_kmer_table: the same LF steps, so identical results) instead of K steps.
// MODE 1 (FLAT, sigma <= 8): the LF steps read the flat occ directory (one line per rank) instead of
// the WT; MODE 2 (NIB, 8 < sigma): the two-level 16-ary directory (two lines per rank).
template <int NC, int MODE = 0>
__global__ __launch_bounds__(256) void k_count(WtView v, const uint8_t* __restrict__ pats,
                                               const uint64_t* __restrict__ offs, uint64_t P,
                                               int64_t* __restrict__ lr, uint64_t* __restrict__ cnt,
                                               const ulonglong2* __restrict__ kmer, int K, uint64_t lim,
                                               uint32_t* __restrict__ bad, const uint4* __restrict__ ol = nullptr,
                                               const uint64_t* __restrict__ osb = nullptr, uint64_t onsb = 0,
                                               NibView nv = NibView{}) {
  constexpr bool FLAT = MODE == 1, NIB = MODE == 2;
  __shared__ QSharedT<NIB ? 1 : NC> q;
  __shared__ typename std::conditional<NIB, NibShared, uint8_t>::type nsx;
  NibShared* const ns = reinterpret_cast<NibShared*>(&nsx);
  __shared__ uint64_t CC[8];
  if (FLAT && threadIdx.x < 8) CC[threadIdx.x] = threadIdx.x < (unsigned)v.sigma ? v.Ccode[threadIdx.x] : 0;
  if constexpr (NIB) {
    q.code[threadIdx.x] = v.code[threadIdx.x];
    load_nib(ns[0], nv);
    __syncthreads();
  } else {
    load_qshared(q, v);
  }
  for (uint64_t p = (uint64_t)blockIdx.x * 256 + threadIdx.x; p < P; p += (uint64_t)gridDim.x * 256) {
    const uint64_t s = offs[p];
    uint64_t k = offs[p + 1];
    uint64_t xl = 0, xr = v.n;
    bool ok = true;
    if (k < s || k > lim) {   // offsets out of order or past the pattern bytes: no read, the call fails
      *bad = 1u;
      ok = false;
      k = s;
    }
    if (K > 0 && k - s >= (uint64_t)K) {
      uint32_t idx = 0;
      for (int j = 0; j < K; ++j) {
        const int c = q.code[pats[k - K + j]];
        ok &= c >= 0;
        idx = idx * (uint32_t)v.sigma + (uint32_t)(c < 0 ? 0 : c);
      }
      k -= K;
      if (ok) {
        const ulonglong2 e = kmer[idx];
        xl = e.x;
        xr = e.y;
        ok = xl < xr;
      }
    }
    while (ok && k > s) {
      --k;
      const int c = q.code[pats[k]];
      if (c < 0) { ok = false; break; }
      if constexpr (FLAT) {
        xl = CC[c] + occ_rank(ol, osb, onsb, c, xl);
        xr = CC[c] + occ_rank(ol, osb, onsb, c, xr);
      } else if constexpr (NIB) {
        nib_lf_pair(nv, ns[0], c, xl, xr);
      } else {
        lf_pair(q, c, xl, xr);
      }
      if (xl >= xr) { ok = false; break; }
    }
    lr[2 * p] = ok ? (int64_t)xl : -1;
    lr[2 * p + 1] = ok ? (int64_t)xr - 1 : -1;
    if (cnt) cnt[p] = ok ? xr - xl : 0;
  }
}

// k-mer table: entry idx (the codes c_0 .. c_{K-1} of a K-symbol string, c_0 most significant in
// radix sigma) = the state after the backward search of that string from the full range; an empty
// state is stored as (1, 0)
template <int NC, int MODE = 0>
__global__ __launch_bounds__(256) void k_kmer_table(WtView v, int K, uint64_t total, ulonglong2* __restrict__ tab,
                                                    const uint4* __restrict__ ol = nullptr,
                                                    const uint64_t* __restrict__ osb = nullptr, uint64_t onsb = 0,
                                                    NibView nv = NibView{}) {
  constexpr bool FLAT = MODE == 1, NIB = MODE == 2;
  __shared__ QSharedT<NIB ? 1 : NC> q;
  __shared__ typename std::conditional<NIB, NibShared, uint8_t>::type nsx;
  NibShared* const ns = reinterpret_cast<NibShared*>(&nsx);
  __shared__ uint64_t CC[8];
  if (FLAT && threadIdx.x < 8) CC[threadIdx.x] = threadIdx.x < (unsigned)v.sigma ? v.Ccode[threadIdx.x] : 0;
  if constexpr (NIB) {
    load_nib(ns[0], nv);
    __syncthreads();
  } else {
    load_qshared(q, v);
  }
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (uint64_t)gridDim.x * 256) {
    uint64_t xl = 0, xr = v.n, x = i;
    bool ok = true;
    for (int j = 0; j < K; ++j) {   // the last symbol (least significant digit) first
      const int c = (int)(x % (uint64_t)v.sigma);
      x /= (uint64_t)v.sigma;
      if constexpr (FLAT) {
        xl = CC[c] + occ_rank(ol, osb, onsb, c, xl);
        xr = CC[c] + occ_rank(ol, osb, onsb, c, xr);
      } else if constexpr (NIB) {
        nib_lf_pair(nv, ns[0], c, xl, xr);
      } else {
        lf_pair(q, c, xl, xr);
      }
      if (xl >= xr) { ok = false; break; }
    }
    tab[i] = ok ? make_ulonglong2(xl, xr) : make_ulonglong2(1, 0);
  }
}

// occ(c, i) = LF(c, i) - C[c]: the WT walk, or NIB the two-level directory (two lines)
template <bool NIB = false>
__global__ __launch_bounds__(256) void k_rank(WtView v, const uint8_t* __restrict__ cs,
                                              const uint64_t* __restrict__ is, uint64_t K,
                                              uint64_t* __restrict__ out, NibView nv = NibView{}) {
  __shared__ QSharedT<NIB ? 1 : 256> q;
  __shared__ typename std::conditional<NIB, NibShared, uint8_t>::type nsx;
  NibShared* const ns = reinterpret_cast<NibShared*>(&nsx);
  if constexpr (NIB) {
    q.code[threadIdx.x] = v.code[threadIdx.x];
    load_nib(ns[0], nv);
    __syncthreads();
  } else {
    load_qshared(q, v);
  }
  for (uint64_t k = (uint64_t)blockIdx.x * 256 + threadIdx.x; k < K; k += (uint64_t)gridDim.x * 256) {
    const int c = q.code[cs[k]];
    if (c < 0) { out[k] = 0; continue; }
    uint64_t x = is[k] < v.n ? is[k] : v.n;
    if constexpr (NIB) {
      x = nib_lf(nv, ns[0], c, x);
    } else {
      uint64_t y = x;
      lf_pair(q, c, x, y);
    }
    out[k] = x - v.Ccode[c];
  }
}

constexpr uint64_t kSmallOcc = 32;
constexpr uint64_t kHugeOcc = 1ull << 16;   // one pattern spread over every workgroup

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
    if (c > kSmallOcc) {   // big: one workgroup each; huge: every workgroup (listed from the end of big)
      if (c > kHugeOcc) big[P - 1 - atomicAdd(nbig + 1, 1ull)] = p;
      else big[atomicAdd(nbig, 1ull)] = p;
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
                                                    const unsigned long long* __restrict__ nbig, uint64_t P,
                                                    uint64_t* __restrict__ pos) {
  const uint64_t nb = nbig[0], nh = nbig[1];
  for (uint64_t b = blockIdx.x; b < nb; b += gridDim.x) {
    const uint64_t p = big[b];
    const uint64_t l = (uint64_t)lr[2 * p];
    const uint64_t c = (uint64_t)(lr[2 * p + 1] + 1) - l;
    const uint64_t o = oo[p];
    for (uint64_t i = threadIdx.x; i < c; i += 256) pos[o + i] = sa[l + i];
  }
  for (uint64_t h = 0; h < nh; ++h) {   // (e.g. the empty pattern: all n rows)
    const uint64_t p = big[P - 1 - h];
    const uint64_t l = (uint64_t)lr[2 * p];
    const uint64_t c = (uint64_t)(lr[2 * p + 1] + 1) - l;
    const uint64_t o = oo[p];
    for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < c; i += (uint64_t)gridDim.x * 256)
      pos[o + i] = sa[l + i];
  }
}

inline unsigned grid_for(uint64_t n, unsigned per = 256, unsigned cap = 16384) {
  uint64_t g = ceil_div(n ? n : 1, per);
  return (unsigned)(g < cap ? g : cap);
}

}  // namespace

namespace {
NibView nib_view(const Index& ix) {
  NibView nv;
  nv.l0 = ix.nib_lines[0].as<uint4>();
  nv.sb0 = ix.nib_sb[0].as<uint64_t>();
  nv.l1 = ix.nib_lines[1].as<uint4>();
  nv.sb1 = ix.nib_sb[1].as<uint64_t>();
  nv.nsb = ix.nib_nsb;
  nv.tab = ix.nib_tab.as<uint8_t>();
  nv.g = ix.nib_g;
  return nv;
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
  // two-level 16-ary occ directory for the batched count (8 < sigma):
  // node groups at depth g, their tables, and level 0 from the BWT (level 1 follows the WT partition
  // that writes the depth-g sequence, or the BWT itself for g = 0)
  const bool nib = sigma > 8;
  const int ng = nib ? std::max(0, L - 4) : 0;
  std::vector<uint8_t> nibh(3072 + 128, 0);   // host source of the table upload (alive to the sync)
  const uint64_t nbl = n / NB_S + 1, nbsb = ceil_div(nbl, (uint64_t)NB_LPS);
  ix.nib_ok = false;
  auto nib_level = [&](int lv, const uint8_t* in, const uint8_t* d_map) {
    ix.nib_lines[lv].ensure(nbl * 64 + 64);
    ix.nib_sb[lv].ensure(nbsb * 16 * 8 + 64);
    TimedLaunch t(ix.timer, "fm_nib_lines", (double)n * 2);
    k_nib_lines<<<(unsigned)nbsb, 256, 0, s>>>(in, n, d_map, nbl, ix.nib_lines[lv].as<uint4>(),
                                               ix.nib_sb[lv].as<uint64_t>());
    HK_HIP(hipGetLastError());
    k_nib_sbscan<<<16, 1024, 0, s>>>(ix.nib_sb[lv].as<uint64_t>(), nbsb);
    HK_HIP(hipGetLastError());
  };
  if (nib) {
    uint8_t* grp = nibh.data();
    uint8_t* val = grp + 256;
    uint8_t* map0 = grp + 512;
    uint8_t* map1 = grp + 768;
    uint64_t* A = reinterpret_cast<uint64_t*>(grp + 1024);
    uint64_t* B = reinterpret_cast<uint64_t*>(grp + 3072);
    int lo[17] = {0}, nh = 0;
    for (int c = 0; c < sigma; ++c) {
      if (c == 0 || (ng > 0 && T.start[ng][c] != T.start[ng][c - 1])) lo[nh++] = c;
      grp[c] = (uint8_t)(nh - 1);
      val[c] = (uint8_t)(c - lo[nh - 1]);
    }
    lo[nh] = sigma;
    if (nh > 16) throw ApiError{-6, "build_wt: more than 16 nodes at the directory depth"};
    for (int h = 0; h < nh; ++h) {
      if (lo[h + 1] - lo[h] > 16) throw ApiError{-6, "build_wt: a directory node of more than 16 codes"};
      B[h] = ix.Ccode[lo[h]];
    }
    for (int c = 0; c < sigma; ++c) {
      uint64_t below = 0;   // value val[c] in the nodes before c's
      for (int h = 0; h < grp[c]; ++h)
        if (lo[h] + val[c] < lo[h + 1]) below += ix.Ccode[lo[h] + val[c] + 1] - ix.Ccode[lo[h] + val[c]];
      A[c] = ix.Ccode[c] - below;
    }
    for (int x = 0; x < 256; ++x) {
      const int c = ix.code_of[x];
      map0[x] = c >= 0 ? grp[c] : 0;
      map1[x] = ng == 0 ? (c >= 0 ? (uint8_t)c : 0) : (x < sigma ? val[x] : 0);
    }
    ix.nib_tab.ensure(nibh.size());
    HK_HIP(hipMemcpyAsync(ix.nib_tab.p, nibh.data(), nibh.size(), hipMemcpyHostToDevice, s));
    ix.nib_g = ng;
    ix.nib_nsb = nbsb;
    if (ng > 0) nib_level(0, ix.bwt.as<uint8_t>(), ix.nib_tab.as<uint8_t>() + 512);
    else nib_level(1, ix.bwt.as<uint8_t>(), ix.nib_tab.as<uint8_t>() + 768);
  }
  // host sources of asynchronous copies: alive until the synchronize at the end of the build
  std::vector<uint16_t> lutv((size_t)kMaxLevels * 256, 0);
  uint16_t (*lut)[256] = reinterpret_cast<uint16_t (*)[256]>(lutv.data());
  std::vector<uint64_t> bsp((size_t)kMaxLevels * 256, 0);
  ix.wt_nlines = nlines;
  if (L > 0) {
    ix.seq[0].ensure(n + 64);
    ix.seq[1].ensure(n + 64);
    // per level: input symbol (BWT byte at level 0, dense code below) -> bit << 15 | node << 8 | code
    for (int d = 0; d < L; ++d) {
      uint16_t node_of[256] = {0};
      int nd = -1;
      for (int c = 0; c < sigma; ++c) {
        if (c == 0 || T.start[d][c] != T.start[d][c - 1]) ++nd;
        node_of[c] = (uint16_t)nd;
      }
      if (nd >= 128) throw ApiError{-6, "build_wt: more than 128 nodes on a level"};
      for (int x = 0; x < 256; ++x) {
        const int c = d == 0 ? ix.code_of[x] : (x < sigma ? x : -1);
        lut[d][x] = c < 0 ? 0 : (uint16_t)((T.bit[d][c] << 15) | (node_of[c] << 8) | c);
      }
    }
    ix.wt_lut.ensure(lutv.size() * 2);
    HK_HIP(hipMemcpyAsync(ix.wt_lut.p, lutv.data(), (size_t)L * 512, hipMemcpyHostToDevice, s));
    // small alphabets: the SWAR level kernels
    bool small = sigma <= 8;
    int byte_of_code[8] = {0};
    for (int b = 0; b < 256; ++b)
      if (ix.code_of[b] >= 0) {
        if (b >= 128) small = false;
        else if (ix.code_of[b] < 8) byte_of_code[ix.code_of[b]] = b;
      }
    WtSmall sml[kMaxLevels];
    memset(sml, 0, sizeof(sml));
    // sigma = 256: every byte present, dense code = byte, the tree perfect: level bits by shifts
    for (int d = 0; d < L; ++d) sml[d].p2sh = sigma == 256 && L == 8 ? 7 - d : -1;
    for (int d = 0; d < L && small; ++d) {
      for (int c = 0; c < sigma; ++c) {
        const uint32_t bit = T.bit[d][c];
        if (c < 4) sml[d].lut_lo |= bit << (8 * c); else sml[d].lut_hi |= bit << (8 * (c - 4));
      }
      if (d == 0) {
        sml[d].nthr = sigma - 1;
        for (int k = 1; k < sigma; ++k) sml[d].thr[k - 1] = 0x01010101u * (uint32_t)byte_of_code[k];
      }
    }
    ix.tile_b.ensure(nlines * 4 + 16);
    ix.tile_a.ensure(nlines * 8 + 16);
    // per level, the 1024-symbol spans holding a node start (k_wt_partition scatters those bytewise);
    // copied once, read after the synchronize at the end of the build
    uint32_t nbsp[kMaxLevels] = {0};
    for (int d = 0; d < L; ++d) {
      std::vector<uint64_t> v;
      for (int c = 1; c < sigma; ++c)
        if (T.start[d][c] != T.start[d][c - 1] && T.start[d][c] % 1024 && T.start[d][c] < n)
          v.push_back(T.start[d][c] / 1024);
      std::sort(v.begin(), v.end());
      v.erase(std::unique(v.begin(), v.end()), v.end());
      if (v.size() > 256) throw ApiError{-6, "build_wt: more than 256 node boundaries on a level"};
      std::copy(v.begin(), v.end(), bsp.begin() + (size_t)d * 256);
      nbsp[d] = (uint32_t)v.size();
    }
    ix.tile_d.ensure(bsp.size() * 8);
    HK_HIP(hipMemcpyAsync(ix.tile_d.p, bsp.data(), bsp.size() * 8, hipMemcpyHostToDevice, s));
    int cur = 0;
    const unsigned gb = grid_for(ceil_div(nlines, WT_V), 4, 8192), gp = grid_for(ceil_div(n, 1024), 4, 8192);
    for (int d = 0; d < L; ++d) {
      ix.wt_lines[d].ensure(nlines * 64);
      uint64_t* lines = ix.wt_lines[d].as<uint64_t>();
      const uint8_t* in = d == 0 ? ix.bwt.as<uint8_t>() : ix.seq[cur].as<uint8_t>();
      {
        TimedLaunch t(ix.timer, "wt_bits", (double)n * (1 + 1.0 / 8));
        if (small)
          k_wt_bits<true><<<gb, 256, 0, s>>>(in, n, ix.wt_lut.as<uint16_t>() + d * 256, lines,
                                             ix.tile_b.as<uint32_t>(), nlines, sml[d]);
        else
          k_wt_bits<false><<<gb, 256, 0, s>>>(in, n, ix.wt_lut.as<uint16_t>() + d * 256, lines,
                                              ix.tile_b.as<uint32_t>(), nlines, sml[d]);
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
        if (small)
          k_wt_partition<true><<<gp, 256, 0, s>>>(in, outp, n, lines, ix.wt_obn.as<uint64_t>() + d * 256,
                                                  ix.wt_rbase.as<uint64_t>() + d * 256,
                                                  ix.wt_lut.as<uint16_t>() + d * 256, ix.tile_d.as<uint64_t>() + d * 256,
                                                  nbsp[d], d == 0 ? 1 : 0, sml[d]);
        else
          k_wt_partition<false><<<gp, 256, 0, s>>>(in, outp, n, lines, ix.wt_obn.as<uint64_t>() + d * 256,
                                                   ix.wt_rbase.as<uint64_t>() + d * 256,
                                                   ix.wt_lut.as<uint16_t>() + d * 256,
                                                   ix.tile_d.as<uint64_t>() + d * 256, nbsp[d], d == 0 ? 1 : 0, sml[d]);
        HK_HIP(hipGetLastError());
        if (nib && ng > 0 && d + 1 == ng) nib_level(1, outp, ix.nib_tab.as<uint8_t>() + 768);
        if (d > 0) cur ^= 1;
      }
    }
  }
  // flat occ directory for the batched count (sigma <= 8)
  ix.occ_ok = false;
  if (sigma >= 2 && sigma <= 8) {
    const uint64_t nl = n / OC_S + 1, nsb = ceil_div(nl, (uint64_t)OC_LPS);
    ix.occ_lines.ensure(nl * 64 + 64);
    ix.occ_sb.ensure(nsb * 64 + 64);   // [8 codes][nsb]
    TimedLaunch t(ix.timer, "fm_occ_lines", (double)n * (1 + 0.5));
    k_occ_lines<<<(unsigned)nsb, 256, 0, s>>>(ix.bwt.as<uint8_t>(), n, ix.wt_code.as<int16_t>(), nl,
                                             ix.occ_lines.as<uint4>(), ix.occ_sb.as<uint64_t>());
    HK_HIP(hipGetLastError());
    for (int c = 0; c < 8; ++c)   // per code, the superblocks' exclusive prefix (in place)
      scan_exclusive_u64(ix.sw, ix.occ_sb.as<uint64_t>() + (uint64_t)c * nsb, ix.occ_sb.as<uint64_t>() + (uint64_t)c * nsb,
                         nsb, false, s);
    ix.occ_nsb = nsb;
    ix.occ_ok = true;
  }
  ix.nib_ok = nib;
  // k-mer table for the batched count: K = the most symbols with sigma^K <= 2^20 entries (<= 16 MiB
  // of (l, r) pairs, MALL-resident; DNA + '$': K = 8, printable: 3, bytes: 2), at most 12
  ix.kmer_k = 0;
  if (L > 0 && sigma >= 2) {
    int K = 0;
    uint64_t tot = 1;
    const uint64_t cap = ix.occ_ok || ix.nib_ok ? (1ull << 21) : (1ull << 20);   // a directory builds it cheaply
    while (K < 12 && tot * (uint64_t)sigma <= cap) {
      tot *= (uint64_t)sigma;
      ++K;
    }
    if (K >= 2) {
      ix.kmer.ensure(tot * 16 + 16);
      TimedLaunch t(ix.timer, "fm_kmer_table", (double)tot * 16);
      if (ix.occ_ok)
        k_kmer_table<16, 1><<<grid_for(tot, 256, 8192), 256, 0, s>>>(ix.view(), K, tot, ix.kmer.as<ulonglong2>(),
                                                                    ix.occ_lines.as<uint4>(),
                                                                    ix.occ_sb.as<uint64_t>(), ix.occ_nsb);
      else if (ix.nib_ok)
        k_kmer_table<16, 2><<<grid_for(tot, 256, 8192), 256, 0, s>>>(ix.view(), K, tot, ix.kmer.as<ulonglong2>(),
                                                                    nullptr, nullptr, 0, nib_view(ix));
      else if (sigma <= 16)
        k_kmer_table<16><<<grid_for(tot, 256, 8192), 256, 0, s>>>(ix.view(), K, tot, ix.kmer.as<ulonglong2>());
      else
        k_kmer_table<256><<<grid_for(tot, 256, 8192), 256, 0, s>>>(ix.view(), K, tot, ix.kmer.as<ulonglong2>());
      HK_HIP(hipGetLastError());
      ix.kmer_k = K;
    }
  }
  HK_HIP(hipStreamSynchronize(s));
  ix.have_wt = true;
}

void query_count(Index& ix, const uint8_t* d_pats, const uint64_t* d_offs, uint64_t P, int64_t* d_lr,
                 uint64_t* d_cnt, uint64_t lim, uint32_t* d_bad) {
  if (!ix.have_wt || ix.sharded) throw ApiError{-3, "count: wavelet tree not built"};
  if (!P) return;
  TimedLaunch t(ix.timer, "fm_count", 0.0);
  const ulonglong2* km = ix.kmer_k ? ix.kmer.as<ulonglong2>() : nullptr;
  if (!d_bad) throw ApiError{-1, "count: no offsets flag"};
  if (ix.occ_ok)
    k_count<16, 1><<<grid_for(P, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_pats, d_offs, P, d_lr, d_cnt, km,
                                                                    ix.kmer_k, lim, d_bad, ix.occ_lines.as<uint4>(),
                                                                    ix.occ_sb.as<uint64_t>(), ix.occ_nsb);
  else if (ix.nib_ok)
    k_count<16, 2><<<grid_for(P, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_pats, d_offs, P, d_lr, d_cnt, km,
                                                                    ix.kmer_k, lim, d_bad, nullptr, nullptr, 0, nib_view(ix));
  else if (ix.sigma <= 16)
    k_count<16><<<grid_for(P, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_pats, d_offs, P, d_lr, d_cnt, km,
                                                                 ix.kmer_k, lim, d_bad);
  else
    k_count<256><<<grid_for(P, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_pats, d_offs, P, d_lr, d_cnt, km,
                                                                  ix.kmer_k, lim, d_bad);
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
  HK_HIP(hipMemsetAsync(nbig, 0, 16, s));   // big and huge pattern counts
  TimedLaunch t(ix.timer, "fm_locate", 0.0);
  if (ix.sa_pos64) {   // replicated sharded SA of a text with n >= 2^32
    k_locate_small<uint64_t><<<grid_for(P, 256, 65535), 256, 0, s>>>(ix.sa.as<uint64_t>(), d_lr, d_occ_offs, P,
                                                                     d_pos, ix.tile_c.as<uint64_t>(), nbig);
    HK_HIP(hipGetLastError());
    k_locate_big<uint64_t><<<1024, 256, 0, s>>>(ix.sa.as<uint64_t>(), d_lr, d_occ_offs, ix.tile_c.as<uint64_t>(),
                                                nbig, P, d_pos);
  } else {
    k_locate_small<uint32_t><<<grid_for(P, 256, 65535), 256, 0, s>>>(ix.sa.as<uint32_t>(), d_lr, d_occ_offs, P,
                                                                     d_pos, ix.tile_c.as<uint64_t>(), nbig);
    HK_HIP(hipGetLastError());
    k_locate_big<uint32_t><<<1024, 256, 0, s>>>(ix.sa.as<uint32_t>(), d_lr, d_occ_offs, ix.tile_c.as<uint64_t>(),
                                                nbig, P, d_pos);
  }
  HK_HIP(hipGetLastError());
}

void query_rank(Index& ix, const uint8_t* d_c, const uint64_t* d_i, uint64_t k, uint64_t* d_out) {
  if (!ix.have_wt) throw ApiError{-3, "rank: wavelet tree not built"};
  if (!k) return;
  if (ix.nib_ok)
    k_rank<true><<<grid_for(k, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_c, d_i, k, d_out, nib_view(ix));
  else
    k_rank<><<<grid_for(k, 256, 65535), 256, 0, ix.stream>>>(ix.view(), d_c, d_i, k, d_out);
  HK_HIP(hipGetLastError());
}

void wt_level_words(Index& ix, int depth, uint64_t* d_words) {
  const uint64_t nw = ceil_div(ix.n, 64);
  k_wt_extract<<<grid_for(nw), 256, 0, ix.stream>>>(ix.wt_lines[depth].as<uint64_t>(), nw, d_words);
  HK_HIP(hipGetLastError());
}

}  // namespace hk
