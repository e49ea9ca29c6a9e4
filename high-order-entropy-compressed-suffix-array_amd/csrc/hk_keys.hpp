// hk_keys.hpp — suffix keys from LDS-staged dense codes, shared by the single-GPU pack
// (hk_sa.hip) and the sharded histogram / pack+select kernels (hk_shard.hip).
//
// key(p) = (code(T[p]) .. code(T[p+q-1]) as a radix-R number) << pb | code(T[p-1]).
// Codes are dense ranks + 1 (0 = past the end of T'), so radix order = Python str order.
#pragma once

#include "hk_common.hpp"

namespace hk {

// radix-R Horner in 24-bit chunks: R^ck < 2^24, so each symbol costs one v_mul_u32_u24 + add;
// chunks are combined in 64-bit.  Rlast = R^(length of the final chunk).
struct KeyChunks {
  int ck = 1;
  uint64_t Rck = 2, Rlast = 2;
  uint64_t Rrest = 1;   // R^(q - ck): weight of the first chunk (q > ck), for bucket pre-tests
};

inline KeyChunks key_chunks(uint64_t R, int q) {
  KeyChunks k;
  k.ck = 1;
  k.Rck = R;
  while (k.Rck * R < (1ull << 24)) {
    k.Rck *= R;
    ++k.ck;
  }
  k.Rlast = 1;
  for (int i = 0; i < (q % k.ck ? q % k.ck : k.ck); ++i) k.Rlast *= R;
  k.Rrest = 1;
  for (int i = k.ck; i < q; ++i) k.Rrest *= R;
  return k;
}

// c[i] = code of position base + i - 1 for i in [0, tile + 64]; aligned 32-bit text loads where
// the text allows it (base is a multiple of the tile, a multiple of 4).
template <int TILE, int NT>
__device__ __forceinline__ void stage_text_codes(uint16_t* c, const uint16_t* L, const uint8_t* __restrict__ t,
                                                 uint64_t n, uint64_t base) {
  if (threadIdx.x == 0) c[0] = L[t[base == 0 ? n - 1 : base - 1]];
  for (int wI = threadIdx.x; wI < (TILE + 64) / 4; wI += NT) {
    const uint64_t p = base + 4 * (uint64_t)wI;
    if (p + 4 <= n) {
      const uint32_t w4 = *reinterpret_cast<const uint32_t*>(t + p);
      c[4 * wI + 1] = L[w4 & 255];
      c[4 * wI + 2] = L[(w4 >> 8) & 255];
      c[4 * wI + 3] = L[(w4 >> 16) & 255];
      c[4 * wI + 4] = L[w4 >> 24];
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) c[4 * wI + 1 + u] = p + u < n ? L[t[p + u]] : 0;
    }
  }
}

// The same staging split in two so a tile's text loads can be issued a tile ahead (software
// pipelining: the loads of tile i+1 are in flight while tile i is processed).  The text buffer
// holds n + 64 bytes, so an aligned word starting below n is always readable.
template <int TILE, int NT>
struct TextWords {
  static constexpr int NWORDS = (TILE + 64) / 4;
  static constexpr int PER = (NWORDS + NT - 1) / NT;
  uint32_t w[PER];
  uint32_t prev;
};

template <int TILE, int NT>
__device__ __forceinline__ void load_text_words(TextWords<TILE, NT>& tw, const uint8_t* __restrict__ t, uint64_t n,
                                                uint64_t base) {
#pragma unroll
  for (int i = 0; i < TextWords<TILE, NT>::PER; ++i) {
    const int wI = threadIdx.x + i * NT;
    const uint64_t p = base + 4 * (uint64_t)wI;
    tw.w[i] = (wI < TextWords<TILE, NT>::NWORDS && p < n) ? *reinterpret_cast<const uint32_t*>(t + p) : 0u;
  }
  tw.prev = threadIdx.x == 0 ? t[base == 0 ? n - 1 : base - 1] : 0u;
}

template <int TILE, int NT>
__device__ __forceinline__ void store_text_codes(uint16_t* c, const uint16_t* L, const TextWords<TILE, NT>& tw,
                                                 uint64_t n, uint64_t base) {
  if (threadIdx.x == 0) c[0] = L[tw.prev];
#pragma unroll
  for (int i = 0; i < TextWords<TILE, NT>::PER; ++i) {
    const int wI = threadIdx.x + i * NT;
    if (wI < TextWords<TILE, NT>::NWORDS) {
      const uint64_t p = base + 4 * (uint64_t)wI;
      const uint32_t w4 = tw.w[i];
      if (p + 4 <= n) {
        c[4 * wI + 1] = L[w4 & 255];
        c[4 * wI + 2] = L[(w4 >> 8) & 255];
        c[4 * wI + 3] = L[(w4 >> 16) & 255];
        c[4 * wI + 4] = L[w4 >> 24];
      } else {
#pragma unroll
        for (int u = 0; u < 4; ++u) c[4 * wI + 1 + u] = p + u < n ? L[(w4 >> (8 * u)) & 255] : 0;
      }
    }
  }
}

// Staged code arrays hold tile + 64 look-ahead codes; kCodePad leaves a little slack past that.
constexpr int kCodePad = 72 + 16;

// value of `len` codes starting at c[j] (len <= ck)
__device__ __forceinline__ uint32_t chunk_value(const uint16_t* c, int j, int len, uint32_t R) {
  uint32_t cv = 0;
  for (int u = 0; u < len; ++u) cv = __umul24(cv, R) + c[j + u];
  return cv;
}

// full mixed-radix key of the suffix whose codes start at c[off + 1] (c[off] = preceding symbol),
// optionally continuing from an already computed first chunk (first = chunk_value(c, off+1, ck))
__device__ __forceinline__ uint64_t key_from(const uint16_t* c, int off, uint64_t R, int q, int pb, int ck,
                                             uint64_t Rck, uint64_t Rlast, int j, uint64_t key) {
  while (j <= q) {
    const int len = q - j + 1 < ck ? q - j + 1 : ck;
    const uint32_t cv = chunk_value(c, off + j, len, (uint32_t)R);
    key = key * (len == ck ? Rck : Rlast) + cv;
    j += len;
  }
  return (key << pb) | (pb ? c[off] : 0u);
}

__device__ __forceinline__ uint64_t key_chunked(const uint16_t* c, int off, uint64_t R, int q, int pb, int ck,
                                                uint64_t Rck, uint64_t Rlast) {
  return key_from(c, off, R, q, pb, ck, Rck, Rlast, 1, 0);
}


// ---------------------------------------------------------------- keyed layout (see KeyGeom)
struct KeyedArgs {
  uint64_t Rk, Rck, Rlast;
  uint64_t s_start;
  int q, ck, pb, hq;   // hq > 0: the bucket is the first hq symbols (radix 2^k, exact split)
};

// sym field of suffix p: its first q keyed codes as a radix-Rk number, or the boundary key of a
// short suffix.  c[off] holds T'[p-1], c[off+1..] T'[p..]; each code is keyed code | byte << 8.
__device__ __forceinline__ uint64_t keyed_sym(const uint16_t* c, int off, uint64_t p, const KeyedArgs& g,
                                              const uint64_t* SK) {
  if (p >= g.s_start) return SK[p - g.s_start];
  uint64_t key = 0;
  int j = 1;
  while (j <= g.q) {
    const int len = g.q - j + 1 < g.ck ? g.q - j + 1 : g.ck;
    uint32_t cv = 0;
    for (int u = 0; u < len; ++u) cv = __umul24(cv, (uint32_t)g.Rk) + (c[off + j + u] & 255u);
    key = key * (len == g.ck ? g.Rck : g.Rlast) + cv;
    j += len;
  }
  return key;
}


// Text-side key source of a radix pass that builds its keys itself (the first pass of the
// single-GPU bucket build): key(p) = keyed_sym(p) << pb | dense code of T'[p-1].
struct TextKeySrc {
  const uint8_t* text;
  uint64_t n;
  const uint16_t* lutk;   // keyed code | byte << 8
  const uint16_t* lutp;   // byte -> dense code
  const uint64_t* skey;   // boundary keys of the short suffixes
  KeyedArgs g;
};

}  // namespace hk
