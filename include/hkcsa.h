/*
 * hkcsa.h — C-ABI of libhkcsa.so, the MI355X-native H_k-CSA build + query path.
 *
 * The reference (ajaynair710/High-Order-Entropy-Compressed-Suffix-Array) has no
 * FFI: its "boundary" is the Python class EnhancedFMIndex and the module
 * functions it calls.  Each entry point below states which reference interface
 * it replaces (file:line under the reference tree).  The Python package
 * `csa` (high-order-entropy-compressed-suffix-array_amd/csa) binds these with
 * ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions
 *  - Every function returns 0 on success or a negative HKCSA_E* code; the
 *    message is available from hkcsa_last_error() (thread-local).
 *  - Host buffers are caller-owned; device buffers live inside the opaque
 *    handle.  A handle is not thread-safe (one HIP stream per handle).
 *  - Texts are byte strings.  The caller appends the reference's '$'
 *    sentinel itself (csa/enhanced_fm_index.py:9); the library treats '$' as
 *    an ordinary byte and end-of-text as smaller than every byte, i.e. Python
 *    str order (csa/suffix_array.py:131-134).
 *  - Suffix-array entries are 64-bit at the ABI.
 */
#ifndef HKCSA_H
#define HKCSA_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HKCSA_ABI_VERSION 1

#define HKCSA_OK 0
#define HKCSA_E_INVALID (-1)   /* bad argument                        */
#define HKCSA_E_HIP (-2)       /* HIP runtime error                   */
#define HKCSA_E_STATE (-3)     /* stage not built yet / wrong order   */
#define HKCSA_E_RANGE (-4)     /* index out of range                  */
#define HKCSA_E_NOMEM (-5)     /* device allocation failed            */
#define HKCSA_E_TOOBIG (-6)    /* size beyond what this build handles */
#define HKCSA_E_DEVICE (-7)    /* kernel reported an internal failure */
#define HKCSA_E_COMM (-8)      /* RCCL failure                        */

typedef struct hkcsa_index hkcsa_index;
typedef struct hkcsa_queries hkcsa_queries;

#define HKCSA_FLAG_POS64 1u    /* sharded builds keep 64-bit positions at any n             */
#define HKCSA_FLAG_NO_SPLIT 2u /* sharded: sort 64-bit positions whole on the global path    */
                               /* (default: u32 low halves, the high bits below the key)    */
#define HKCSA_FLAG_GLOBAL_SORT 4u /* full-width LSD radix sort of every suffix key (default:   */
                                  /* top-bit passes + LDS bucket sorts); single GPU and slices */
#define HKCSA_FLAG_MUL_BINS 8u /* sharded slices: multiplicative bucket bins even where the  */
                               /* shift bins would do (diagnostic; chosen automatically)    */
#define HKCSA_FLAG_MAX_BUCKETS 16u /* single GPU: 2^16 buckets (2^17 with half items) at any n, */
                                   /* so small texts take the 1 GiB pipeline (diagnostic)       */
#define HKCSA_FLAG_SLICES 32u  /* single GPU: the multi-slice build (taken by itself when    */
                               /* n >= 2^32 - 1) at any n, in 4 slices (parity tests)        */
#define HKCSA_FLAG_LINKS 64u   /* single GPU: link shifted-copy groups in the first doubling  */
                               /* round at any tie count (default: when a third or more of   */
                               /* the suffixes reach doubling; parity tests)                 */
#define HKCSA_FLAG_NO_LINKS 128u /* single GPU: never link (diagnostic)                       */

typedef struct hkcsa_opts {
  int32_t device;   /* HIP device ordinal (-1 = current)                 */
  uint32_t flags;   /* HKCSA_FLAG_* bits, 0 by default                   */
  uint64_t reserved[2];
} hkcsa_opts;

/* ---- library ---------------------------------------------------------- */
int hkcsa_abi_version(void);
int hkcsa_device_count(int* n);
const char* hkcsa_last_error(void);

/* ---- construction ----------------------------------------------------- */
/* Upload text T' (n bytes, sentinel already appended) to the device.
 * Replaces the text handling of EnhancedFMIndex.__init__
 * (csa/enhanced_fm_index.py:8-9). */
int hkcsa_create(const uint8_t* text, uint64_t n, const hkcsa_opts* o, hkcsa_index** out);
/* The same from `nparts` host pieces uploaded back to back (T' = parts[0] + parts[1] + ...):
 * EnhancedFMIndex's `text + "$"` (csa/enhanced_fm_index.py:9) without building the
 * concatenation on the host — the caller passes its text buffer and the sentinel. */
int hkcsa_create_parts(const uint8_t* const* parts, const uint64_t* lens, int nparts, const hkcsa_opts* o,
                       hkcsa_index** out);
/* Generate a synthetic text on the device: n-1 iid bytes drawn from the
 * `sigma` symbols `alphabet[0..sigma)` by a counter-based hash of (seed, i),
 * followed by the byte `terminator`.  Reproducible on the host with
 * oracle/hkcsa_oracle.c:oracle_synth_text. (bench input, no reference twin) */
int hkcsa_create_synthetic(uint64_t n, const uint8_t* alphabet, int sigma, uint64_t seed,
                           uint8_t terminator, const hkcsa_opts* o, hkcsa_index** out);
/* Suffix array of T'.  Replaces build_suffix_array (csa/suffix_array.py:131-134).
 * Default: keyed bucket build (q-symbol suffix keys grouped by bucket with two
 * lookback-free scatter passes whose destinations come from per-span cursors — or
 * two stable LSD passes when the alphabet has no whole-symbol buckets — LDS bucket
 * sorts that write SA and BWT together, chunk refinement of tied suffixes, GPU
 * prefix doubling over an ISA for texts whose ties persist);
 * HKCSA_FLAG_GLOBAL_SORT: full-width LSD sort of the keys instead of bucket sorts.
 * Texts of n >= 2^32 - 1 symbols (64-bit positions; the reference's SA has no size
 * limit) are built on the one device as slices of ~2^30 suffixes of the final SA, one
 * after another, straight into one full SA / BWT: slice bounds from one partition
 * histogram of the whole text, ties that outlast a slice's chunk refinement finished by
 * prefix doubling over one ISA of the full SA (HKCSA_FLAG_SLICES takes this path at
 * any n).  Recomputes the byte histogram / C array every call. */
int hkcsa_build_sa(hkcsa_index* ix);
/* BWT of T' (bwt_transform, csa/bwt.py:3-13).  The SA build already writes the
 * BWT in sorted order, so this is a no-op after hkcsa_build_sa; it gathers
 * T'[SA[i]-1] only when the SA came without its BWT. */
int hkcsa_build_bwt(hkcsa_index* ix);
/* C array + levelwise wavelet tree over the BWT with interleaved rank lines.
 * Replaces build_count (utils/utils.py:16-24), build_occ (utils/utils.py:26-32)
 * as the rank structure, and WaveletTree.build_tree (csa/wavelet_tree.py:72-100).
 * Also builds the batched count's accelerators: the backward-search state of every
 * K-symbol string (sigma^K <= 2^20, 2^21 for sigma <= 8) and, for sigma <= 8, a flat occ directory of the
 * BWT (one 64-B line per 128 symbols); both give results identical to the WT walk. */
int hkcsa_build_wt(hkcsa_index* ix);
/* SA + BWT + WT in one call (EnhancedFMIndex.__init__, csa/enhanced_fm_index.py:8-13). */
int hkcsa_build_all(hkcsa_index* ix);
/* Drop the construction workspace (keys, ISA, ...) kept for repeated builds, and the device
 * workspace of hkcsa_count_batch / hkcsa_locate_batch (those calls keep buffers of <= 64 MiB
 * between calls and free larger ones when the call ends). */
int hkcsa_release_workspace(hkcsa_index* ix);
/* SA sampling for the epsilon space/time contract of CompressedSuffixArray(text, epsilon)
 * (tests/benchmark.py:25,32; the class itself is absent from the reference, csa/csa.py:3):
 * keeps SA[i] for the rows with SA[i] % rate == 0, the row of every position k*rate, and the
 * exact LF of the rows whose BWT symbol is T'[n-1] (the wrapped row, csa/bwt.py:8-11).
 * Needs the single-GPU SA; builds the BWT/WT if missing. */
int hkcsa_build_samples(hkcsa_index* ix, uint32_t rate);
/* Compressed mode: release SA, BWT array, T' and workspace.  Afterwards SA entries, locate,
 * BWT bytes and text/extract are answered by LF walks over the WT to the samples — results
 * identical to the full arrays; construction calls fail with HKCSA_E_STATE. */
int hkcsa_compact(hkcsa_index* ix);
/* Empirical k-th order entropy of the whole buffer T (csa/high_order_entropy.py:4-32,
 * calculate_high_order_entropy): H_0 for k = 0; for k > 0 the sum over length-k contexts w of
 * (n_w / n) * H_0(symbols following w) over positions i < n - k; 0 when n <= k or k < 0.
 * Builds the SA if missing (contexts are SA runs).  Double precision; the reference's
 * summation order differs, so agreement is to rounding (relative 1e-9 in the tests). */
int hkcsa_entropy(hkcsa_index* ix, int k, double* out);
/* Resident bytes: out[0] text, [1] SA, [2] BWT array, [3] WT rank lines, [4] sample marks,
 * [5] SA/ISA samples + LF fixes, [6] sample rate, [7] 1 if samples are built. */
int hkcsa_space(hkcsa_index* ix, uint64_t out[8]);
int hkcsa_synchronize(hkcsa_index* ix);
void hkcsa_free(hkcsa_index* ix);

/* Module-level helpers (no index semantics of their own):
 * BWT gather over a caller-supplied SA (bwt_transform, csa/bwt.py:3-13): out[i] =
 * text[sa[i]-1], text[n-1] when sa[i]==0; every sa[i] must be < n. */
int hkcsa_bwt_gather(const uint8_t* text, uint64_t n, const uint64_t* sa, uint8_t* out);
/* Treat the handle's text itself as the sequence to index with the wavelet tree
 * (WaveletTree(seq), csa/wavelet_tree.py:66-70; build_occ(bwt), utils/utils.py:26-32). */
int hkcsa_use_text_as_bwt(hkcsa_index* ix);

/* ---- inspection / parity exports ------------------------------------- */
int hkcsa_get_n(const hkcsa_index* ix, uint64_t* n);
/* SA[lo:hi) into out (hi-lo entries). EnhancedFMIndex.suffix_array. */
int hkcsa_get_sa(hkcsa_index* ix, uint64_t lo, uint64_t hi, uint64_t* out);
/* BWT[lo:hi). EnhancedFMIndex.bwt. */
int hkcsa_get_bwt(hkcsa_index* ix, uint64_t lo, uint64_t hi, uint8_t* out);
/* T'[lo:hi). */
int hkcsa_get_text(hkcsa_index* ix, uint64_t lo, uint64_t hi, uint8_t* out);
/* C[b] = #{j : T'[j] < b} for every byte value b (C[256] = n).  For bytes
 * present in T' this equals EnhancedFMIndex.count (utils/utils.py:16-24). */
int hkcsa_get_C(hkcsa_index* ix, uint64_t C[257]);
/* Sorted distinct bytes of T' (WaveletTree.alphabet, csa/wavelet_tree.py:68). */
int hkcsa_get_alphabet(hkcsa_index* ix, uint8_t syms[256], int* sigma);
/* Number of levels of the full balanced WT (ceil(log2 sigma)). */
int hkcsa_wt_levels(hkcsa_index* ix, int* levels);
/* Level `depth` bitvector, n bits, packed LSB-first into ceil(n/64) words
 * (words_out may be NULL to query nbits).  The reference's left-spine level
 * l (csa/wavelet_tree.py:82) is the prefix of depth-l of length |leftmost node|. */
int hkcsa_wt_level(hkcsa_index* ix, int depth, uint64_t* nbits, uint64_t* words_out);
/* Golomb-Rice code of the runs of ones in the first `nbits` bits of level
 * `depth` — GolombRiceEncoder(bitmap).encode(bitmap) of csa/wavelet_tree.py:27-63
 * as build_tree applies it (:84-86).  m = the reference's rule from the ones
 * density (float log2, truncated, at least 1) unless m_override > 0 (< 64).
 * Outputs: *m_out, *ones_out (popcount of the prefix), *code_bits (length of
 * the code); words_out (nullable: sizes only) receives ceil(code_bits/64)
 * words, code bit j at bit j%64 of word j/64; cap_words is its capacity. */
int hkcsa_wt_golomb(hkcsa_index* ix, int depth, uint64_t nbits, uint32_t m_override, uint32_t* m_out,
                    uint64_t* ones_out, uint64_t* code_bits, uint64_t* words_out, uint64_t cap_words);
/* occ(c_k, i_k) = #c_k in BWT[0:min(i_k, n)) for k < count, 0 for absent bytes.
 * EnhancedFMIndex.rank (csa/enhanced_fm_index.py:34-40). */
int hkcsa_rank(hkcsa_index* ix, const uint8_t* c, const uint64_t* i, uint64_t count, uint64_t* out);

/* ---- batched queries -------------------------------------------------- */
/* Patterns are concatenated bytes `pats` with offsets offs[0..P] (offs[0]=0,
 * non-decreasing).  The two batch calls copy straight from and into the caller's
 * (pageable) buffers and check the offsets on the device: offsets out of order
 * return HKCSA_E_INVALID before any output is written.
 * count: lr_out[2p], lr_out[2p+1] = (l, r) of EnhancedFMIndex.find_range
 * (csa/enhanced_fm_index.py:21-32), (-1,-1) on a miss. */
int hkcsa_count_batch(hkcsa_index* ix, const uint8_t* pats, const uint64_t* offs, uint64_t P,
                      int64_t* lr_out);
/* locate: EnhancedFMIndex.find (csa/enhanced_fm_index.py:15-19), positions in
 * SA order.  occ_offs (P+1 entries, CSR offsets) is required and always filled
 * first.  pos_out == NULL: sizes only.  Otherwise, when cap >= occ_offs[P], every
 * position is gathered into pos_out in one call; when cap is smaller the call
 * returns HKCSA_E_RANGE with occ_offs filled and nothing written to pos_out, so
 * the caller can size its buffer from occ_offs[P] and call again. */
int hkcsa_locate_batch(hkcsa_index* ix, const uint8_t* pats, const uint64_t* offs, uint64_t P,
                       uint64_t* occ_offs, uint64_t* pos_out, uint64_t cap);
/* Device-resident query sets (bench: inputs resident in HBM before timing). */
int hkcsa_queries_upload(hkcsa_index* ix, const uint8_t* pats, const uint64_t* offs, uint64_t P,
                         hkcsa_queries** out);
int hkcsa_queries_count(hkcsa_index* ix, hkcsa_queries* q);                 /* (l,r) on device */
int hkcsa_queries_locate(hkcsa_index* ix, hkcsa_queries* q, uint64_t* total); /* count+scan+gather */
int hkcsa_queries_download(hkcsa_index* ix, hkcsa_queries* q, int64_t* lr_out, uint64_t* occ_offs,
                           uint64_t* pos_out, uint64_t cap);
void hkcsa_queries_free(hkcsa_queries* q);
/* text[i:j) of T' (csa.CSA.extract; oracle: Python slicing). */
int hkcsa_extract(hkcsa_index* ix, uint64_t i, uint64_t j, uint8_t* out);   /* T'[i:j); LF walks when compacted */

/* ---- sharded (multi-GPU) suffix-array construction ------------------- */
/* RCCL unique id (128 bytes) to be broadcast by the caller from rank 0. */
int hkcsa_comm_unique_id(uint8_t id[128]);
/* Each rank holds the same T' (created on its own device).  Ranks split the
 * final SA into contiguous rank ranges from one RCCL all-reduce of a partition
 * histogram: for keyed alphabets (hkcsa_shard_scheme 1: DNA, binary, 16 or 256
 * symbols) the EXACT coarse histogram of every suffix's first 16 key bits, which
 * fixes the slice bounds by itself; for other alphabets a sampled key histogram
 * plus a second all-reduce of the N+1 exact counts below the splitters.  Each rank
 * sorts its slice independently; an RCCL all-gather of per-rank status records
 * checks that the slices tile [0, n).  Slices still tied after the chunk
 * refinement finish by prefix doubling with an ISA replica per rank, built by an
 * RCCL all-gather of the SA slices and refreshed per round by an all-gather of the
 * re-ranked suffixes' (position, ISA) pairs.  A failure on any rank makes every
 * rank return an error (no rank is left waiting in a collective).  After the call
 * ix holds SA[lo:hi) (and its BWT rows). */
int hkcsa_build_sa_sharded(hkcsa_index* ix, const uint8_t id[128], int nranks, int rank);
int hkcsa_shard_range(hkcsa_index* ix, uint64_t* lo, uint64_t* hi);
/* Replicas for batched queries (count/locate are replicas-only):
 * hkcsa_shard_replicate: RCCL all-gather (communicator of the last
 *   hkcsa_build_sa_sharded) of every rank's SA slice and BWT rows; afterwards the
 *   handle is a full index (hkcsa_build_wt, queries, hkcsa_get_sa/bwt work).
 *   Collective: every rank calls it.  Serves EnhancedFMIndex.find / find_range
 *   (csa/enhanced_fm_index.py:15-32) on every rank.
 * hkcsa_shard_adopt: the same from a host-assembled full SA (n entries) and BWT
 *   (n bytes), for hosts running their own collectives. */
int hkcsa_shard_replicate(hkcsa_index* ix);
int hkcsa_shard_adopt(hkcsa_index* ix, const uint64_t* sa, const uint8_t* bwt);
/* Sharded SA slice entries SA[lo+a : lo+b) (a,b relative to the slice). */
int hkcsa_get_shard_sa(hkcsa_index* ix, uint64_t a, uint64_t b, uint64_t* out);
/* BWT of the slice: out[j] = T'[SA[lo+a+j]-1] (wrapping), j < b-a — the rows
 * bwt_transform (csa/bwt.py:4-9) emits for this rank's SA range. */
int hkcsa_get_shard_bwt(hkcsa_index* ix, uint64_t a, uint64_t b, uint8_t* out);
/* The same construction in three host-visible phases, for hosts that do their own
 * collectives (and for single-GPU tests of the partitioning).  Two partition schemes,
 * chosen from the alphabet (hkcsa_shard_scheme):
 *   1 (keyed coarse: the keyed radix is 2^lb, lb in {1,2,4,8} — DNA, binary, 16 or 256
 *     symbols): the bucket of a suffix is the top 16 bits of its keyed sym field (its
 *     first 16/lb symbols); rank r's block is [n*r/N, n*(r+1)/N) with 16-aligned starts
 *     and hkcsa_shard_histogram counts EVERY suffix of it (exact), so the global
 *     histogram alone fixes the slices (hkcsa_build_sa_sharded skips the counts phase);
 *     the splitters are equal-width (r * 65536 / N) when N divides 65536 and no such slice
 *     is 2 % above n/N, else balanced (below);
 *   0 (partition key, any other alphabet): the bucket is the top 14 bits of a radix-(sigma+1)
 *     key over the positions p % hkcsa_shard_sample() == 0 of [n*r/N, n*(r+1)/N); bins past
 *     16384 stay 0; balanced splitters.
 * Balanced splitters: B_r = the smallest bucket with cum(B_r) >= floor(S*r/N), S = the
 * histogram total (hkcsa/shard.py split_buckets).
 *   hkcsa_shard_histogram: the block's histogram (hkcsa_shard_buckets() = 65536 bins);
 *   hkcsa_shard_counts: with G = the element-wise sum of every rank's histogram,
 *     below_out[j] (j = 0..N) = #suffixes of the block whose bucket is below
 *     splitter j (splitters derived from G; below_out[0] = 0);
 *   hkcsa_shard_build: builds SA[lo:hi) of this rank from G and the element-wise
 *     sum of every rank's below_out (lo, hi = its entries r and r+1). */
/* Host-side slice planner (no device work): the SA bounds below_out[0..nslices] that
 * hkcsa_build_sa's slice build (and the keyed sharded build) derive from an exact coarse
 * histogram of `nbins` buckets (equal-width or balanced splitters, as above).  Slots inside a
 * slice are 32-bit, so a slice of 2^32 - 1 or more suffixes — one coarse bucket too large to
 * split, e.g. a long run in a text of n > 2^32 — is refused with HKCSA_E_TOOBIG (the builds
 * refuse the same text the same way instead of wrapping). */
int hkcsa_slice_bounds(const uint64_t* hist, uint32_t nbins, int nslices, uint64_t* below_out);
int hkcsa_shard_buckets(void);
int hkcsa_shard_sample(void);
int hkcsa_shard_scheme(hkcsa_index* ix, int* scheme);   /* 1 keyed coarse, 0 partition key */
int hkcsa_shard_histogram(hkcsa_index* ix, int nranks, int rank, uint64_t* hist_out);
int hkcsa_shard_counts(hkcsa_index* ix, const uint64_t* global_hist, int nranks, int rank,
                       uint64_t* below_out);
int hkcsa_shard_build(hkcsa_index* ix, const uint64_t* global_hist, const uint64_t* global_below,
                      int nranks, int rank);
/* Prefix doubling across slices, host-driven (hkcsa_build_sa_sharded runs the
 * same steps over RCCL).  The SA must be exact for every text
 * (csa/suffix_array.py:131-134); a slice whose tied groups survive the chunk
 * refinement (long repeats / runs) is left pending after hkcsa_shard_build:
 *   hkcsa_shard_status: st = {lo, hi, A = tied suffixes left, h = common-prefix
 *     length of their groups}; A = 0 means the slice is final;
 *   hkcsa_shard_isa_segment: ISA replica: isa[sa[j]] = lo + j for one rank's
 *     slice (its hkcsa_get_shard_sa entries, readable while pending); call once
 *     per rank slice on every pending rank;
 *   hkcsa_shard_updates: the (position, ISA) pairs (2 u64 each) of this rank's
 *     last step — the tied suffixes at their group head's slot after the build,
 *     every re-ranked suffix after a round; NULL pairs: count only;
 *   hkcsa_shard_apply: isa[p] = v for pairs of any rank (every rank's, own included);
 *   hkcsa_shard_round: one doubling round: each tied group sorted by ISA[p+h],
 *     h += K, where K = min h over the ranks with A > 0.
 * Loop: segments -> {updates of all ranks -> apply -> round(K) -> status} until
 * every rank reports A = 0 (hkcsa/shard.py shard_doubling). */
int hkcsa_shard_status(hkcsa_index* ix, uint64_t st[4]);
int hkcsa_shard_isa_segment(hkcsa_index* ix, const uint64_t* sa, uint64_t count, uint64_t lo);
int hkcsa_shard_updates(hkcsa_index* ix, uint64_t* pairs, uint64_t cap, uint64_t* count);
int hkcsa_shard_apply(hkcsa_index* ix, const uint64_t* pairs, uint64_t count);
int hkcsa_shard_round(hkcsa_index* ix, uint64_t K);

/* Suffix-key geometry chosen for this text (parity export for the shard tests):
 * q symbols as a radix-`radix` number above a pb-bit preceding-symbol field. */
int hkcsa_key_geometry(hkcsa_index* ix, int* q, int* pb, uint64_t* radix, int* key_bits);

/* ---- diagnostics ------------------------------------------------------ */
/* Per-pass milliseconds of radix-pass variants over n synthetic DNA keys
 * (u32 values): out = {512x16, 512x16 without lookback, 512x16 without lookback
 * or LDS staging, 256x16, 256x16 without lookback, 1024x8, plain pair copy,
 * error flag}.  Ablations produce wrong orders by design; only times matter. */
int hkcsa_debug_radix_bench(uint64_t n, int reps, double* out, int nout);

/* ---- per-kernel timing (HIP events on the handle's stream) ------------ */
int hkcsa_timing_enable(hkcsa_index* ix, int on);
int hkcsa_timing_reset(hkcsa_index* ix);
/* Aggregated stats for kernels whose name matches `name` exactly.
 * alg_bytes is the algorithmic byte count summed over launches. */
int hkcsa_kernel_stats(hkcsa_index* ix, const char* name, uint64_t* launches, double* total_ms,
                       double* alg_bytes);
/* Build-stage counters of the last build: [0] radix / cursor scatter passes run, [1] skipped,
 * [2] refinement rounds (doubling rounds << 32), [3] symbols per key; bucket build:
 * [4] LDS work items, [5] big buckets, [6] suffixes in big buckets, [7] bit 0 = global path,
 * bit 1 = packed records (one u64 of key bits and position per suffix through the partition),
 * [8] LDS work items sorted by the stable LSD passes instead of the MSD bin fast path;
 * then tied suffixes per round (up to cap). */
int hkcsa_build_info(hkcsa_index* ix, uint64_t* info, int cap);

#ifdef __cplusplus
}
#endif
#endif /* HKCSA_H */
