/*
 * hkcsa_oracle.c — CPU restatement of the reference's hot path. TEST INFRASTRUCTURE ONLY:
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg as the checker;
 * never linked into or called by the product (libhkcsa.so / the csa package).
 *
 * Pinned against the reference's own outputs: the fixtures in tests/golden/ were produced by
 * importing the reference (tests/golden/make_golden.py) and tests/test_oracle.py checks this
 * file against every vector there.
 *
 * Each function cites the reference code it restates (paths relative to the reference root).
 */
#include <stdint.h>
#include <stdlib.h>
#ifdef _OPENMP
#include <omp.h>
#endif
#include <string.h>
#include <math.h>

/* ---------------------------------------------------------------- suffix order
 * csa/suffix_array.py:131-134 sorts (text[i:], i) tuples: Python str order, i.e. code point
 * order with a proper prefix first.  Suffixes are distinct, so the index never breaks a tie. */
static const uint8_t* g_t;
static uint64_t g_n;

static int suffix_cmp(const void* pa, const void* pb) {
  const uint64_t a = *(const uint64_t*)pa, b = *(const uint64_t*)pb;
  const uint64_t la = g_n - a, lb = g_n - b;
  const uint64_t m = la < lb ? la : lb;
  int c = memcmp(g_t + a, g_t + b, m);
  if (c) return c;
  return la < lb ? -1 : (la > lb ? 1 : 0);
}

int oracle_suffix_array(const uint8_t* t, uint64_t n, uint64_t* sa) {
  for (uint64_t i = 0; i < n; ++i) sa[i] = i;
  g_t = t;
  g_n = n;
  qsort(sa, n, sizeof(uint64_t), suffix_cmp);
  return 0;
}

/* csa/bwt.py:3-13: bwt[i] = text[sa[i]-1], wrapping to text[n-1] */
void oracle_bwt(const uint8_t* t, uint64_t n, const uint64_t* sa, uint8_t* bwt) {
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) bwt[i] = t[sa[i] == 0 ? n - 1 : sa[i] - 1];
}

/* utils/utils.py:16-24: C[c] = number of symbols < c (C[256] = n) */
void oracle_count(const uint8_t* t, uint64_t n, uint64_t C[257]) {
  uint64_t h[256] = {0};
  for (uint64_t i = 0; i < n; ++i) h[t[i]]++;
  uint64_t acc = 0;
  for (int c = 0; c < 256; ++c) {
    C[c] = acc;
    acc += h[c];
  }
  C[256] = acc;
}

/* ------------------------------------------------------------------- occ
 * utils/utils.py:26-32 stores occ[c][i] = #c in bwt[0:i) for every i; here a sampled table answers the
 * same query: for the symbols present (dense columns), u64 counts every 65536 positions and u16 counts
 * relative to them every 64 positions, then a scan of < 64 bytes.  u64 superblocks: texts past 2^32
 * symbols (a symbol may occur more than 2^32 times) are answered exactly. */
typedef struct {
  const uint8_t* bwt;
  uint64_t n;
  int sig;                 /* present symbols (columns) */
  int16_t col[256];        /* symbol -> column, -1 if absent */
  uint64_t* sup;           /* (n >> 16) + 1 rows x sig */
  uint16_t* sub;           /* (n >> 6) + 1 rows x sig, relative to the row's superblock */
} occ_t;

void* oracle_occ_new(const uint8_t* bwt, uint64_t n) {
  occ_t* o = (occ_t*)malloc(sizeof(occ_t));
  o->bwt = bwt;
  o->n = n;
  int T = 1;
#ifdef _OPENMP
  T = omp_get_max_threads();
#endif
  const uint64_t nsup = (n >> 16) + 1, nsub = (n >> 6) + 1;
  /* chunks of whole superblocks: per-chunk symbol totals, their exclusive prefix, then each chunk fills
   * its rows from its prefix */
  const uint64_t per = (nsup + T - 1) / T;
  uint64_t* tot = (uint64_t*)calloc((size_t)(T + 1) * 256, sizeof(uint64_t));
#pragma omp parallel for schedule(static, 1)
  for (int c = 0; c < T; ++c) {
    const uint64_t i0 = (per * c) << 16, i1 = (per * (c + 1)) << 16;
    for (uint64_t i = i0; i < i1 && i < n; ++i) tot[(size_t)(c + 1) * 256 + bwt[i]]++;
  }
  for (int c = 1; c <= T; ++c)
    for (int s2 = 0; s2 < 256; ++s2) tot[(size_t)c * 256 + s2] += tot[(size_t)(c - 1) * 256 + s2];
  o->sig = 0;
  for (int s2 = 0; s2 < 256; ++s2) o->col[s2] = tot[(size_t)T * 256 + s2] ? (int16_t)o->sig++ : (int16_t)-1;
  const int sig = o->sig ? o->sig : 1;
  o->sup = (uint64_t*)calloc(nsup * sig, sizeof(uint64_t));
  o->sub = (uint16_t*)calloc(nsub * sig, sizeof(uint16_t));
#pragma omp parallel for schedule(static, 1)
  for (int c = 0; c < T; ++c) {
    const uint64_t i0 = (per * c) << 16, i1 = (per * (c + 1)) << 16;
    uint64_t cur[256], base[256];
    for (int s2 = 0; s2 < 256; ++s2) cur[s2] = tot[(size_t)c * 256 + s2];
    for (uint64_t i = i0; i < i1 && i <= n; ++i) {
      if ((i & 0xFFFF) == 0) {
        for (int s2 = 0; s2 < 256; ++s2) {
          base[s2] = cur[s2];
          if (o->col[s2] >= 0) o->sup[(i >> 16) * sig + o->col[s2]] = cur[s2];
        }
      }
      if ((i & 63) == 0)
        for (int s2 = 0; s2 < 256; ++s2)
          if (o->col[s2] >= 0) o->sub[(i >> 6) * sig + o->col[s2]] = (uint16_t)(cur[s2] - base[s2]);
      if (i < n) cur[bwt[i]]++;
    }
  }
  free(tot);
  return o;
}

void oracle_occ_free(void* p) {
  occ_t* o = (occ_t*)p;
  if (!o) return;
  free(o->sup);
  free(o->sub);
  free(o);
}

/* csa/enhanced_fm_index.py:34-40: rank(c, i) = occ[c][min(i, n)] (absent c -> 0; the caller
 * handles absent symbols) */
uint64_t oracle_occ(const void* p, uint8_t c, uint64_t i) {
  const occ_t* o = (const occ_t*)p;
  if (i > o->n) i = o->n;
  const int k = o->col[c];
  if (k < 0) return 0;
  uint64_t r = o->sup[(i >> 16) * o->sig + k] + o->sub[(i >> 6) * o->sig + k];
  for (uint64_t q = i & ~(uint64_t)63; q < i; ++q) r += o->bwt[q] == c;
  return r;
}

/* csa/enhanced_fm_index.py:21-32 backward search over P patterns (concatenated, offsets) */
void oracle_find_range(const void* p, const uint64_t C[257], const uint8_t* present, const uint8_t* pats,
                       const uint64_t* offs, uint64_t P, int64_t* lr) {
  const occ_t* o = (const occ_t*)p;
  for (uint64_t q = 0; q < P; ++q) {
    int64_t l = 0, r = (int64_t)o->n - 1;
    int ok = 1;
    for (uint64_t k = offs[q + 1]; k > offs[q];) {
      --k;
      const uint8_t c = pats[k];
      int64_t nl, nr;
      if (!present[c]) {
        nl = 0;
        nr = -1;
      } else {
        nl = (int64_t)(oracle_occ(o, c, (uint64_t)l) + C[c]);
        nr = (int64_t)(oracle_occ(o, c, (uint64_t)(r + 1)) + C[c]) - 1;
      }
      if (nl > nr) {
        ok = 0;
        break;
      }
      l = nl;
      r = nr;
    }
    lr[2 * q] = ok ? l : -1;
    lr[2 * q + 1] = ok ? r : -1;
  }
}

/* ------------------------------------------------------------- SA checker
 * O(n) proof that sa is THE suffix array of t (so it equals build_suffix_array's output):
 * sa is a permutation and every adjacent pair is ordered — first symbols, then (when they are
 * equal) the ranks of the suffixes one further, with end-of-text ranking lowest.
 * Returns 0 when valid, 1 + offending index otherwise. */
uint64_t oracle_check_sa(const uint8_t* t, uint64_t n, const uint64_t* sa) {
  if (n == 0) return 0;
  uint64_t* isa = (uint64_t*)malloc(n * sizeof(uint64_t));
  uint64_t bad = UINT64_MAX;   /* smallest offending index (threads: OpenMP, one per core) */
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) isa[i] = UINT64_MAX;
#pragma omp parallel for schedule(static) reduction(min : bad)
  for (uint64_t j = 0; j < n; ++j) {
    if (sa[j] >= n) bad = j < bad ? j : bad;
    else isa[sa[j]] = j;
  }
  /* a permutation iff every entry reads back its own slot (a duplicate loses one of its writes) */
#pragma omp parallel for schedule(static) reduction(min : bad)
  for (uint64_t j = 0; j < n; ++j)
    if (sa[j] < n && isa[sa[j]] != j) bad = j < bad ? j : bad;
#pragma omp parallel for schedule(static) reduction(min : bad)
  for (uint64_t j = 1; j < n; ++j) {
    const uint64_t a = sa[j - 1], b = sa[j];
    if (a >= n || b >= n) continue;
    int ok;
    if (t[a] != t[b]) ok = t[a] < t[b];
    else if (a + 1 == n) ok = 1;          /* suffix a is a proper prefix of suffix b */
    else if (b + 1 == n) ok = 0;
    else ok = isa[a + 1] < isa[b + 1];
    if (!ok) bad = j < bad ? j : bad;
  }
  free(isa);
  return bad == UINT64_MAX ? 0 : 1 + bad;
}

/* ------------------------------------------------------------- synthetic text
 * Same counter-based generator as the device (hk_sa.hip k_synth). */
static uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

void oracle_synth_text(uint64_t n, const uint8_t* alpha, int sigma, uint64_t seed, uint8_t term, uint8_t* out) {
  const uint64_t key = seed * 0xD1B54A32D192ED03ull;
#pragma omp parallel for schedule(static)
  for (uint64_t i = 0; i < n; ++i) {
    if (i + 1 == n) out[i] = term;
    else out[i] = alpha[(uint32_t)(splitmix64(key ^ i) >> 32) % (uint32_t)sigma];
  }
}

/* ------------------------------------------------------------- wavelet tree
 * csa/wavelet_tree.py:72-100 splits a node's sorted alphabet at len//2 (bit 1 = right half) and
 * stably filters the sequence into the children; the reference keeps only the leftmost child.
 * This builds every node, level by level (nodes left to right), returning L levels of n bits
 * (one byte per bit).  Symbols whose leaf is shallower keep bit 0 and their position. */
int oracle_wt_levels(const uint8_t* seq, uint64_t n, uint8_t* bits /* 8*n */) {
  int present[256] = {0}, code[256], sigma = 0;
  for (uint64_t i = 0; i < n; ++i) present[seq[i]] = 1;
  for (int c = 0; c < 256; ++c) code[c] = present[c] ? sigma++ : -1;
  int L = 0;
  while ((1 << L) < sigma) ++L;
  uint64_t cnt[257] = {0};
  for (uint64_t i = 0; i < n; ++i) cnt[code[seq[i]] + 1]++;
  for (int c = 0; c < sigma; ++c) cnt[c + 1] += cnt[c]; /* cnt[c] = #codes < c */
  int* cur = (int*)malloc((n + 1) * sizeof(int));
  int* nxt = (int*)malloc((n + 1) * sizeof(int));
  for (uint64_t i = 0; i < n; ++i) cur[i] = code[seq[i]];
  for (int d = 0; d < L; ++d) {
    uint64_t fill_left[256], fill_right[256];
    int lo_of[256], hi_of[256], mid_of[256];
    for (int c = 0; c < sigma; ++c) {
      int lo = 0, hi = sigma;
      for (int dd = 0; dd < d && hi - lo > 1; ++dd) {
        int mid = lo + (hi - lo) / 2;
        if (c >= mid) lo = mid; else hi = mid;
      }
      lo_of[c] = lo;
      hi_of[c] = hi;
      mid_of[c] = hi - lo > 1 ? lo + (hi - lo) / 2 : hi;
    }
    for (int c = 0; c < sigma; ++c) {
      fill_left[c] = cnt[lo_of[c]];
      fill_right[c] = cnt[mid_of[c]];
    }
    /* per node fill pointers, keyed by the node's lo */
    uint64_t fl[256], fr[256];
    for (int c = 0; c < sigma; ++c) {
      fl[lo_of[c]] = fill_left[c];
      fr[lo_of[c]] = fill_right[c];
    }
    for (uint64_t i = 0; i < n; ++i) {
      const int c = cur[i];
      const int b = (hi_of[c] - lo_of[c] > 1) && c >= mid_of[c];
      bits[(uint64_t)d * n + i] = (uint8_t)b;
      if (b) nxt[fr[lo_of[c]]++] = c;
      else nxt[fl[lo_of[c]]++] = c;
    }
    int* tmp = cur;
    cur = nxt;
    nxt = tmp;
  }
  free(cur);
  free(nxt);
  return L;
}

/* ------------------------------------------------------------- shard partition
 * Host restatement of the sharded build's partition (hk_sa.hip key_geometry, hk_shard.hip):
 * the key of suffix p is its first q dense codes (code 0 past the end) as one radix-R number,
 * R = sigma + 1, shifted above the pb-bit code of T[p-1] (T[n-1] for p = 0).  q minimises
 * passes * n + 30 * min(n, n^2 * sum(p_c^2)^q).  The bucket is the top 14 bits of the key. */
static int mixed_radix_bits(uint64_t R, int q) {
  unsigned __int128 p = 1;
  for (int i = 0; i < q; ++i) {
    p *= R;
    if (p > ((unsigned __int128)1 << 64)) return 65;
  }
  p -= 1;
  int b = 0;
  while (p) {
    ++b;
    p >>= 1;
  }
  return b;
}

int oracle_key_geometry(const uint8_t* t, uint64_t n, int* q_out, int* pb_out, uint64_t* R_out, int* kb_out,
                        uint16_t code[256]) {
  uint64_t h[256] = {0};
  for (uint64_t i = 0; i < n; ++i) h[t[i]]++;
  int sigma = 0;
  for (int c = 0; c < 256; ++c) code[c] = h[c] ? (uint16_t)(++sigma) : 0;
  const uint64_t R = (uint64_t)sigma + 1;
  int pb = 1;
  while ((1 << pb) < sigma + 1) ++pb;
  double p2 = 0, nn = (double)(n ? n : 1);
  for (int c = 0; c < 256; ++c) p2 += ((double)h[c] / nn) * ((double)h[c] / nn);
  double best = 1e300;
  int bq = 1, bsb = 0;
  for (int q = 1; q <= 64; ++q) {
    const int sb = mixed_radix_bits(R, q);
    if (pb + sb > 64) break;
    double ties = nn * nn * pow(p2, (double)q);
    if (ties > nn) ties = nn;
    const double cost = (double)((sb + 7) / 8) * nn + 30.0 * ties;
    if (cost <= best) {
      best = cost;
      bq = q;
      bsb = sb;
    }
  }
  *q_out = bq;
  *pb_out = pb;
  *R_out = R;
  *kb_out = pb + bsb;
  return sigma;
}

/* Partition geometry of the sharded build (hk_shard.hip partition_geometry): codes and R as
 * above, no prev field (pb = 0: a bucket must be a range of the suffix order, which the prev
 * field would split), and as many symbols as fit in 64 bits, so the top 14 bits are as fine a
 * prefix split as possible. */
static int partition_geometry(const uint8_t* t, uint64_t n, int* q_out, int* pb_out, uint64_t* R_out, int* kb_out,
                              uint16_t code[256]) {
  int q, pb, kb;
  const int sigma = oracle_key_geometry(t, n, &q, &pb, R_out, &kb, code);
  q = 1;
  while (q < 64 && mixed_radix_bits(*R_out, q + 1) <= 64) ++q;
  *q_out = q;
  *pb_out = 0;
  *kb_out = mixed_radix_bits(*R_out, q);
  return sigma;
}

/* bucket (top 14 key bits) of suffix p under the partition geometry */
static uint64_t shard_bucket(const uint8_t* t, uint64_t n, uint64_t p, const uint16_t* code, int q, int pb,
                             uint64_t R, int bsh) {
  uint64_t key = 0;
  for (int j = 0; j < q; ++j) key = key * R + (p + j < n ? code[t[p + j]] : 0);
  key = (key << pb) | code[t[p == 0 ? n - 1 : p - 1]];
  return key >> bsh;
}

/* Keyed coarse scheme of the sharded build (hk_bucket.hip key_geometry_keyed, shard_coarse_hist):
 * the keyed alphabet is every byte present except a terminal T[n-1] that occurs exactly once (when
 * at least two bytes are present); a keyed byte's digit is the number of keyed bytes below it.  The
 * scheme applies when the keyed radix Rk = max(#keyed, 2) is 2^lb with lb in {1, 2, 4, 8}.  The coarse
 * bucket of suffix p is the first H = 16 / lb digits of its digit string as one radix-Rk number: the
 * digits of T[p..] up to the unkeyed terminal or the end of the text, then one digit (the number of
 * keyed bytes below the terminal, or 0 when the text just ends), then zeros.  Returns lb (0: the
 * sampled partition key below applies instead). */
int oracle_shard_scheme(const uint8_t* t, uint64_t n, uint16_t dig[256], int* unkeyed_term, int* mterm) {
  uint64_t h[256] = {0};
  for (uint64_t i = 0; i < n; ++i) h[t[i]]++;
  int sigma = 0;
  for (int c = 0; c < 256; ++c) sigma += h[c] != 0;
  const int term = n ? t[n - 1] : -1;
  const int unk = n && h[term] == 1 && sigma >= 2;
  int rk = 0, below = 0;
  for (int c = 0; c < 256; ++c) {
    const int keyed = h[c] && !(unk && c == term);
    dig[c] = (uint16_t)rk;
    if (unk && c < term && keyed) ++below;
    rk += keyed;
  }
  if (rk < 2) rk = 2;
  *unkeyed_term = unk ? term : -1;
  *mterm = unk ? below : 0;
  switch (rk) {
    case 2: return 1;
    case 4: return 2;
    case 16: return 4;
    case 256: return 8;
    default: return 0;
  }
}

static uint32_t coarse_bucket(const uint8_t* t, uint64_t n, uint64_t p, const uint16_t* dig, int lb, int uterm,
                              int mterm) {
  const int H = 16 / lb;
  uint32_t v = 0;
  int i = 0, done = 0;
  for (; i < H && !done; ++i) {
    const uint64_t j = p + (uint64_t)i;
    uint32_t d;
    if (j >= n) {
      d = 0;
      done = 1;
    } else if ((int)t[j] == uterm && j == n - 1) {
      d = (uint32_t)mterm;
      done = 1;
    } else {
      d = dig[t[j]];
    }
    v = (v << lb) | d;
  }
  for (; i < H; ++i) v <<= lb;
  return v;
}

/* Sharded partition histogram of the positions [lo, hi): keyed scheme: the exact coarse histogram
 * (65536 bins); else the sampled key-prefix histogram of the positions p % 64 == 0 (hk_shard.hip,
 * SH_SAMPLE) in the first 16384 bins: the splitters only need balance; exact slice sizes come from
 * oracle_shard_below. */
void oracle_shard_hist(const uint8_t* t, uint64_t n, uint64_t lo, uint64_t hi, uint64_t* hist /* 65536 */) {
  memset(hist, 0, 65536 * sizeof(uint64_t));
  uint16_t dig[256];
  int uterm, mterm;
  const int lb = oracle_shard_scheme(t, n, dig, &uterm, &mterm);
  if (lb) {
    for (uint64_t p = lo; p < hi; ++p) hist[coarse_bucket(t, n, p, dig, lb, uterm, mterm)]++;
    return;
  }
  uint16_t code[256];
  int q, pb, kb;
  uint64_t R;
  partition_geometry(t, n, &q, &pb, &R, &kb, code);
  int bsh = kb - 14;
  if (bsh < 0) bsh = 0;
  for (uint64_t p = (lo + 63) / 64 * 64; p < hi; p += 64) hist[shard_bucket(t, n, p, code, q, pb, R, bsh)]++;
}

/* below[j] = #{p in [lo, hi) : bucket(p) < B[j]} for j < nb (the scheme's bucket) */
void oracle_shard_below(const uint8_t* t, uint64_t n, uint64_t lo, uint64_t hi, const uint32_t* B, int nb,
                        uint64_t* below) {
  for (int j = 0; j < nb; ++j) below[j] = 0;
  uint16_t dig[256];
  int uterm, mterm;
  const int lb = oracle_shard_scheme(t, n, dig, &uterm, &mterm);
  if (lb) {
    for (uint64_t p = lo; p < hi; ++p) {
      const uint32_t b = coarse_bucket(t, n, p, dig, lb, uterm, mterm);
      for (int j = 0; j < nb; ++j) below[j] += b < B[j];
    }
    return;
  }
  uint16_t code[256];
  int q, pb, kb;
  uint64_t R;
  partition_geometry(t, n, &q, &pb, &R, &kb, code);
  int bsh = kb - 14;
  if (bsh < 0) bsh = 0;
  for (uint64_t p = lo; p < hi; ++p) {
    const uint64_t b = shard_bucket(t, n, p, code, q, pb, R, bsh);
    for (int j = 0; j < nb; ++j) below[j] += b < B[j];
  }
}

/* Golomb-Rice code of the runs of ones of bits[0:n) with parameter m
 * (csa/wavelet_tree.py:40-63): per maximal run of L ones, L/m zeros, a one, then L%m in m
 * binary digits MSB first.  Writes the code as 0/1 bytes into out (NULL: size only) and
 * returns its length. */
uint64_t oracle_golomb(const uint8_t* bits, uint64_t n, uint32_t m, uint8_t* out) {
  uint64_t o = 0, run = 0;
  for (uint64_t i = 0; i <= n; ++i) {
    if (i < n && bits[i]) {
      ++run;
      continue;
    }
    if (run) {
      const uint64_t q = run / m, r = run % m;
      if (out) {
        for (uint64_t k = 0; k < q; ++k) out[o + k] = 0;
        out[o + q] = 1;
        for (uint32_t k = 0; k < m; ++k) out[o + q + 1 + k] = (uint8_t)((r >> (m - 1 - k)) & 1);
      }
      o += q + 1 + m;
      run = 0;
    }
  }
  return o;
}
