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
  int lb = 0;          // radix 2^lb with sym = q*lb bits exactly: keys are bit windows of a packed stream
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


// keyed sym of up to 28 symbols held in 8 little-endian words starting at byte `sh` of w[0]:
// realigned with alignbyte, then a fully unrolled chunked Horner (uniform branches on q / ck)
__device__ __forceinline__ uint64_t keyed_horner28(const uint32_t (&w)[8], uint32_t sh, const KeyedArgs& g,
                                                   const uint16_t* LK) {
  uint32_t r[7];
#pragma unroll
  for (int i = 0; i < 7; ++i) r[i] = __builtin_amdgcn_alignbyte(w[i + 1], w[i], sh);
  uint64_t key = 0;
  uint32_t cv = 0;
  int in = 0;
#pragma unroll
  for (int j = 0; j < 28; ++j) {
    if (j < g.q) {
      cv = __umul24(cv, (uint32_t)g.Rk) + (LK[(r[j >> 2] >> (8 * (j & 3))) & 255u] & 255u);
      if (++in == g.ck || j == g.q - 1) {
        key = key * (in == g.ck ? g.Rck : g.Rlast) + cv;
        cv = 0;
        in = 0;
      }
    }
  }
  return key;
}

// keyed_sym of the suffix whose first byte is byte b of the LDS word array W (the text staged as
// raw words); short suffixes are the caller's
__device__ __forceinline__ uint64_t keyed_sym_words(const uint32_t* W, uint32_t b, const KeyedArgs& g,
                                                    const uint16_t* LK) {
  if (g.q <= 28) {
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = W[(b >> 2) + i];
    return keyed_horner28(w, b & 3u, g, LK);
  }
  const uint8_t* B = reinterpret_cast<const uint8_t*>(W) + b;
  uint64_t key = 0;
  int j = 0;
  while (j < g.q) {
    const int len = g.q - j < g.ck ? g.q - j : g.ck;
    uint32_t cv = 0;
    for (int u = 0; u < len; ++u) cv = __umul24(cv, (uint32_t)g.Rk) + (LK[B[j + u]] & 255u);
    key = key * (len == g.ck ? g.Rck : g.Rlast) + cv;
    j += len;
  }
  return key;
}

// keyed_sym of suffix p read straight from the text (aligned word loads, bytes through the keyed
// code table LK), for passes that build keys of scattered positions without staging their tile.
__device__ __forceinline__ uint64_t keyed_sym_text(const uint8_t* __restrict__ t, uint64_t p, const KeyedArgs& g,
                                                   const uint16_t* LK, const uint64_t* SK) {
  if (p >= g.s_start) return SK[p - g.s_start];
  if (g.q <= 28) {
    // up to 28 symbols: eight independent word loads (T' has 64 readable pad bytes)
    const uint32_t* wp = reinterpret_cast<const uint32_t*>(t + (p & ~3ull));
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = wp[i];
    return keyed_horner28(w, (uint32_t)(p & 3u), g, LK);
  }
  const uint32_t* w = reinterpret_cast<const uint32_t*>(t + (p & ~3ull));
  uint32_t cur = w[0] >> (8u * (uint32_t)(p & 3u));
  int avail = 4 - (int)(p & 3u);
  uint64_t key = 0;
  int j = 0;
  while (j < g.q) {
    const int len = g.q - j < g.ck ? g.q - j : g.ck;
    uint32_t cv = 0;
    for (int u = 0; u < len; ++u) {
      if (avail == 0) {
        cur = *++w;
        avail = 4;
      }
      cv = __umul24(cv, (uint32_t)g.Rk) + (LK[cur & 255u] & 255u);
      cur >>= 8;
      --avail;
    }
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

// The keys of one radix tile straight from the text (item k of lane `lane` of a wave is suffix
// wbase + 64k + lane).  Radix 2^lb (src.g.lb): each staging thread maps 32 text bytes to codes and
// packs them MSB-first into lb words; a key is the q*lb-bit window at bit off*lb of that stream
// (3 LDS words).  Otherwise the tile's codes are staged and each key is a chunked Horner sum.
// LDS: codes[T*I + kCodePad] (generic) or pk[(T*I + 64)/4 + 4] + raw[T*I + 64] (packed), which
// may alias each other; contains barriers (call from every thread of the block).
// LB > 0: the packed path with lb = LB known at compile time (fully unrolled packing, static
// register indices); LB = 0: lb from src.g.lb at run time (0 = the Horner path).
template <int T, int I, int LB = 0>
__device__ __forceinline__ void text_keys(uint64_t (&key)[I], const TextKeySrc& src, uint64_t n, uint64_t tbase,
                                          uint64_t wbase, uint32_t lane, uint16_t* codes, uint32_t* pk,
                                          uint8_t* raw, uint32_t* prev0, const uint16_t* L, const uint16_t* LP,
                                          const uint64_t* SK) {
  constexpr int TILE = T * I;
  const uint32_t tid = threadIdx.x;
  if (LB || src.g.lb) {
    // radix 2^lb: each staging thread maps 32 text bytes to codes and packs them MSB-first into
    // lb words; a key is then the q*lb-bit window at bit off*lb of the stream (3 LDS words)
    const int lb = LB ? LB : src.g.lb;
    if (tid == 0) *prev0 = src.text[tbase == 0 ? n - 1 : tbase - 1];
    for (uint32_t c = tid; c < (uint32_t)(TILE + 64) / 32; c += T) {
      const uint64_t p0 = tbase + 32ull * c;
      uint4 a = make_uint4(0, 0, 0, 0), b = a;
      if (p0 < n) {   // T' has 64 readable pad bytes; positions past n only feed short suffixes
        const uint4* q4 = reinterpret_cast<const uint4*>(src.text + p0);
        a = q4[0];
        b = q4[1];
      }
      const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
      *reinterpret_cast<uint4*>(&raw[32 * c]) = a;
      *reinterpret_cast<uint4*>(&raw[32 * c + 16]) = b;
      if (LB) {
        constexpr int PER = LB ? 32 / LB : 1;
#pragma unroll
        for (int o = 0; o < LB; ++o) {
          uint32_t word = 0;
#pragma unroll
          for (int u = 0; u < PER; ++u) {
            const int i = o * PER + u;
            word = (word << LB) | (L[(w[i >> 2] >> (8 * (i & 3))) & 255u] & 255u);
          }
          pk[c * LB + o] = word;
        }
      } else {
        const int per = 32 / lb;   // codes per word
        for (int o = 0; o < lb; ++o) {
          uint32_t word = 0;
          for (int u = 0; u < per; ++u) {
            const int i = o * per + u;
            word = (word << lb) | (L[(w[i >> 2] >> (8 * (i & 3))) & 255u] & 255u);
          }
          pk[c * lb + o] = word;
        }
      }
    }
    __syncthreads();
    const int kbits = src.g.q * lb;
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const uint64_t j = wbase + (uint64_t)k * 64 + lane;
      const uint32_t off = (uint32_t)(j - tbase);
      uint64_t sym;
      if (j >= src.g.s_start) {
        sym = j < n ? SK[j - src.g.s_start] : 0;
      } else {
        const uint32_t bit = off * (uint32_t)lb, w0 = bit >> 5, o = bit & 31u;
        const uint64_t hi = ((uint64_t)pk[w0] << 32) | pk[w0 + 1];
        const uint64_t win = o ? (hi << o) | (pk[w0 + 2] >> (32 - o)) : hi;
        sym = kbits >= 64 ? win : win >> (64 - kbits);
      }
      const uint32_t pbyte = off ? raw[off - 1] : *prev0;
      key[k] = j < n ? (sym << src.g.pb) | LP[pbyte] : ~0ull;
    }
  } else {
    stage_text_codes<TILE, T>(codes, L, src.text, n, tbase);
    __syncthreads();
#pragma unroll
    for (int k = 0; k < I; ++k) {
      const uint64_t j = wbase + (uint64_t)k * 64 + lane;
      const int off = (int)(j - tbase);
      key[k] = j < n ? (keyed_sym(codes, off, j, src.g, SK) << src.g.pb) | LP[codes[off] >> 8]
                     : ~0ull;
    }
  }
}

// Pass A of the packed-record build (radix 2^2 codes, 16 items per thread): item k of thread tid is
// position tbase + 16 tid + k, so the thread's 16 windows and prev codes all come from the three packed
// words at its own 16 symbols (plus the word before) with compile-time shifts: 4 LDS reads per thread
// instead of 5 per key (text_keys' lane-strided items need a fresh 3-word window, a raw byte and a
// table lookup each).  The prev field is the keyed code straight from the stream (the packed records'
// prev code: the unique terminal, code 0 in both, precedes only position 0), LP only for the byte
// before the tile.
// The staging half: the tile's packed codes into pk (one 32-byte chunk per thread), then this thread's
// three words and the word before; consec2_key turns them into item k's key.
struct Consec2Words {
  uint32_t a, b, c, pw;
};

template <int T>
__device__ __forceinline__ Consec2Words consec2_words(const TextKeySrc& src, uint64_t n, uint64_t tbase, uint32_t* pk,
                                                      uint32_t* prev0, const uint16_t* L) {
  constexpr int TILE = T * 16;
  const uint32_t tid = threadIdx.x;
  if (tid == 0) *prev0 = src.text[tbase == 0 ? n - 1 : tbase - 1];
  for (uint32_t c = tid; c < (uint32_t)(TILE + 64) / 32; c += T) {
    const uint64_t p0 = tbase + 32ull * c;
    uint4 a = make_uint4(0, 0, 0, 0), b = a;
    if (p0 < n) {   // T' has 64 readable pad bytes; positions past n only feed short suffixes
      const uint4* q4 = reinterpret_cast<const uint4*>(src.text + p0);
      a = q4[0];
      b = q4[1];
    }
    const uint32_t w[8] = {a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w};
#pragma unroll
    for (int o = 0; o < 2; ++o) {
      uint32_t word = 0;
#pragma unroll
      for (int u = 0; u < 16; ++u) {
        const int i = o * 16 + u;
        word = (word << 2) | (L[(w[i >> 2] >> (8 * (i & 3))) & 255u] & 255u);
      }
      pk[c * 2 + o] = word;
    }
  }
  __syncthreads();
  return Consec2Words{pk[tid], pk[tid + 1], pk[tid + 2], tid ? pk[tid - 1] : 0u};
}

// key of item k (position tbase + 16 tid + k) from the thread's words (k compile-time after unrolling)
__device__ __forceinline__ uint64_t consec2_key(const Consec2Words& w, int k, const TextKeySrc& src, uint64_t n,
                                                uint64_t tbase, const uint32_t* prev0, const uint16_t* LP,
                                                const uint64_t* SK) {
  const uint32_t tid = threadIdx.x;
  const uint64_t hi = ((uint64_t)w.a << 32) | w.b;
  const int kbits = src.g.q * 2;
  const uint64_t j = tbase + 16ull * tid + (uint64_t)k;
  const uint64_t win = k ? (hi << (2 * k)) | (w.c >> (32 - 2 * k)) : hi;
  uint64_t sym = kbits >= 64 ? win : win >> (64 - kbits);
  if (j >= src.g.s_start) sym = j < n ? SK[j - src.g.s_start] : 0;
  const uint32_t pc = k ? (w.a >> (32 - 2 * k)) & 3u : (tid ? w.pw & 3u : LP[*prev0]);
  return j < n ? (sym << src.g.pb) | pc : ~0ull;
}

// Pass A of the packed-record build (radix 2^2 codes, 16 items per thread): item k of thread tid is
// position tbase + 16 tid + k, so the thread's 16 windows and prev codes all come from the three packed
// words at its own 16 symbols (plus the word before) with compile-time shifts: 4 LDS reads per thread
// instead of 5 per key (text_keys' lane-strided items need a fresh 3-word window, a raw byte and a
// table lookup each).  The prev field is the keyed code straight from the stream (the packed records'
// prev code: the unique terminal, code 0 in both, precedes only position 0), LP only for the byte
// before the tile.
template <int T>
__device__ __forceinline__ void text_keys_consec2(uint64_t (&key)[16], const TextKeySrc& src, uint64_t n,
                                                  uint64_t tbase, uint32_t* pk, uint32_t* prev0,
                                                  const uint16_t* L, const uint16_t* LP, const uint64_t* SK) {
  const Consec2Words w = consec2_words<T>(src, n, tbase, pk, prev0, L);
#pragma unroll
  for (int k = 0; k < 16; ++k) key[k] = consec2_key(w, k, src, n, tbase, prev0, LP, SK);
}

}  // namespace hk
