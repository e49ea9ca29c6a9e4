// hk_index.hpp — the opaque hkcsa_index handle and the per-module drivers.
#pragma once

#include <cstring>
#include <memory>
#include <utility>

#include "hk_sort.hpp"

namespace hk {

constexpr int kMaxLevels = 8;
constexpr uint32_t kFlagPos64 = 1u;   // hkcsa_opts.flags: 64-bit positions in sharded builds at any n
constexpr uint32_t kFlagNoSplit = 2u; // ... and sort them as whole u64 values (no split low/high halves)
constexpr uint32_t kFlagGlobalSort = 4u; // full LSD sort of the keys (no bucket sorts)
constexpr uint32_t kFlagMulBins = 8u;    // sharded slices: force multiplicative bucket bins
constexpr uint32_t kFlagMaxBuckets = 16u; // single GPU: the most bucket bits at any n (diagnostic)
constexpr uint32_t kFlagSlices = 32u;     // single GPU: the multi-slice build at any n (4 slices; parity tests)
constexpr uint32_t kFlagLinks = 64u;      // single GPU: doubling links at any tie count (parity tests)
constexpr uint32_t kFlagNoLinks = 128u;   // single GPU: no doubling links (diagnostic)
constexpr int kLineBits = 448;   // 7 data words per 64-B rank line (word 0 = ones before the line)

struct WtTables {                // per level, per dense code (host mirror of the device tables)
  uint8_t bit[kMaxLevels][256];
  uint64_t start[kMaxLevels][256];
  uint64_t zeros[kMaxLevels][256];
  uint8_t depth[256];
};

// suffix key layout: [q dense codes as one mixed-radix number, radix R = sigma'+1, code 0 = end
// of text][code of the preceding symbol, pb bits].  Sorting uses bits [pb, key_bits).
struct KeyGeom {
  int q = 0, pb = 0, sym_bits = 0, key_bits = 0;
  uint64_t R = 2;
  uint16_t lut[256];   // byte -> dense code + 1 (0 = end of text)
  uint8_t inv[512];    // dense code + 1 -> byte
  // ---- keyed layout (single-GPU bucket build, hk_bucket.hip).  The sorted field is the first q
  // symbols in radix Rk over the *keyed* alphabet: every symbol except a terminal that occurs
  // once, at n-1 (the reference's '$').  There is no end-of-text code.  The suffixes whose
  // q-window reaches the end or the unkeyed terminal ("short" suffixes, positions
  // [s_start, n), at most q of them) get the exact boundary key B(s) (the smallest window value
  // that sorts after them) and are ordered among themselves by srank in the first refinement.
  bool keyed = false;
  uint64_t Rk = 2;
  uint16_t lutk[256];        // byte -> keyed code in the low byte | byte << 8
  uint16_t lutp[256];        // byte -> dense code (the prev field of keyed keys; inv[] is by dense code)
  uint64_t s_start = 0;      // first short suffix
  uint32_t nS = 0;           // n - s_start
  uint64_t skey[72];         // B(s) of the short suffixes (sym field, not shifted)
  uint32_t srank[72];        // exact order of the short suffixes among themselves
  int bucket_bits = 0;       // D: top bits of the sym field sorted by the LSD passes
  uint16_t kdig[256];        // byte -> number of keyed bytes below it (its keyed code when keyed)
  uint8_t kflag[256];        // byte -> 1 when keyed
  uint16_t k2d[256];         // keyed code -> dense code (the prev field of a keyed byte)
  int tcode = -1;            // dense code of the unkeyed terminal (-1: none); it precedes only suffix 0
};
int mixed_radix_bits(uint64_t R, int q);   // bits of R^q - 1 (65 when it does not fit 64 bits)

// kernel argument bundle for rank walks
struct WtView {
  const uint64_t* lines[kMaxLevels];
  const uint64_t* obn;     // [L][256]  ones before the code's node at level d
  const uint64_t* rbase;   // [L][256]  right-child base: start + zeros - obn
  const uint8_t* bit;      // [L][256]
  const uint8_t* depth;    // [256]
  const int16_t* code;     // [256] byte -> dense code, -1 when absent
  const uint64_t* Ccode;   // [257]
  int levels;
  int sigma;
  uint64_t n;
};

struct Index {
  int device = 0;
  uint32_t flags = 0;          // hkcsa_opts.flags
  hipStream_t stream = nullptr;
  hipStream_t aux_stream = nullptr;   // read-backs that overlap the main stream (cursor partition counts)
  uint64_t n = 0;
  DevBuf text;                 // T' (n bytes + 64 pad)

  // alphabet
  bool have_alpha = false;
  uint64_t byte_hist[256] = {0};
  uint8_t tail[72] = {0};      // the last min(n, 70) bytes of T' (short-suffix keys), read with the histogram
  bool tail_valid = false;
  int sigma = 0;
  uint8_t syms[256] = {0};
  int16_t code_of[256];
  uint64_t Cbyte[257] = {0};
  uint64_t Ccode[257] = {0};

  // products
  bool have_sa = false, have_bwt = false, have_wt = false;
  DevBuf sa;                   // u32[n]
  DevBuf bwt;                  // u8[n]
  int wt_levels = 0;
  DevBuf wt_lines[kMaxLevels];
  uint64_t wt_nlines = 0;
  DevBuf wt_obn, wt_rbase, wt_bit, wt_depth, wt_code, wt_C, wt_lut;
  WtTables tabs;

  // construction workspace (kept across builds so repeated builds do not allocate)
  SortWork sw;
  DevBuf keys[2], vals[2];
  DevBuf isa;
  DevBuf act[2][3];            // P, J, G of the active list (double-buffered)
  DevBuf act_b;                // BWT bytes of the first refinement round's list (global path), list order
  DevBuf head_slot;            // SA slot of each tied group's head (refinement -> doubling switch)
  DevBuf ties_k, ties_v, ties_n;   // unordered tie list of the bucket build (J<<1|head, P), count
  DevBuf big_k[2], big_v[2], big_j; // big buckets of the bucket build (sorted on the global path); the
                                    // members of large tied groups of a refinement / doubling round
  DevBuf grp_big;                   // refinement / doubling round: u8 per group, 1 = over SEG_MAX members
                                    // (LDS item rounds: over SR_W members)
  DevBuf sr_hp[2], sr_win[2], sr_items, sr_cnt;   // LDS item rounds (hk_seground.hip): group heads and window
                                                  // first / last heads of list act[i], items, counters
  const void* sr_plan_g = nullptr;   // the G buffer whose plan the last round wrote (next round reuses it)
  DevBuf lk_lnk, lk_gsz, lk_tops, lk_grec;   // doubling links (hk_seground.hip): per position {offset, slot delta},
                                             // the size of the tied group at each head slot, the link tiles' tops,
                                             // the linked groups {head slot, size, head position}
  DevBuf bk_items, bk_hist, bk_fb; // bucket work items, bucket histogram, fast-path fallback items
  DevBuf cp_part, cp_cur, cp_tiles; // cursor partition: per-span counts, destination cursors, pass-B tiles
  HostBuf cp_host;                  // ... and its pinned host side (bucket counts, region table)
  DevBuf sel;                     // sharded build: selection masks of the slice (u16 per 16 positions)
  DevBuf kmer;                    // count: backward-search state of every K-symbol string (build_wt)
  int kmer_k = 0;
  DevBuf occ_lines, occ_sb;       // count: flat occ directory of the BWT (sigma <= 8, build_wt)
  bool occ_ok = false;
  uint64_t occ_nsb = 0;
  // count: two-level 16-ary occ directory (8 < sigma <= 256, build_wt): level 0 = the BWT's WT node
  // at depth nib_g, level 1 = the WT's depth-nib_g sequence as code - node start; tables in nib_tab
  DevBuf nib_lines[2], nib_sb[2], nib_tab;
  bool nib_ok = false;
  int nib_g = 0;
  uint64_t nib_nsb = 0;
  DevBuf tile_a, tile_b, tile_c, tile_d, tile_e;
  DevBuf small;                // scratch for totals etc.
  HostBuf small_host;          // pinned staging of the geometry tables (one upload per geometry), with
                               // the byte histogram's landing slots [0, 2048) and the text tail's at 8192
  hipEvent_t geom_ev = nullptr;   // the last geometry upload (its staging is reused by the next one)
  HostBuf items_host;          // pinned staging of the bucket-sort work items
  HostBuf rb_host;             // pinned landing slots of the build's small read-backs (counts, totals)
  uint64_t* rb(int k = 4) {    // k u64 slots
    rb_host.ensure(64);
    (void)k;
    return static_cast<uint64_t*>(rb_host.p);
  }
  DevBuf seq[2];               // WT level code sequences
  DevBuf gr_tmp[2], gr_out;    // Golomb-Rice coding of a level (per-word carries/offsets, code words)

  // SA/ISA samples (compressed mode, hk_sample.hip)
  bool have_text = true;       // false after compact(): T' is then read back by LF walks
  bool bwt_in_wt = false;      // the BWT array was released; BWT[i] comes from the WT
  bool have_samples = false;
  uint32_t smp_rate = 0;
  uint64_t smp_count = 0, smp_fixn = 0;
  int smp_cstar = 0;
  bool smp_w64 = false;        // 8-byte samples (the SA was u64)
  DevBuf smp_mark, smp_sa, smp_isa, smp_fix, smp_inv;

  // sharded construction
  bool sharded = false;
  bool sa_pos64 = false;       // sharded slices of texts with n >= 2^32 hold u64 positions
  bool slices_local = false;   // build_sa_slices: the slices' doubling updates one local ISA (no exchange)
  std::shared_ptr<void> fused;  // build_sa_slices: a group's fused pass A (records + cursors per slice)
  DevBuf fused_recs, fused_ws;  // ... its records and cursor sets (kept across builds: allocating and freeing
  HostBuf fused_host;           // tens of GB per build stalled some builds by seconds)
  uint64_t shard_lo = 0, shard_hi = 0;
  std::vector<uint64_t> shard_bounds;   // SA slice starts of every rank (+ n), from the RCCL build

  // prefix doubling over the tied suffixes left by the chunk refinement (DblState): the active
  // list act[dbl.cur] (P, J = slot in the slice, G = dense group ordinal), A suffixes in `groups`
  // groups whose members share their first h symbols.  A sharded slice leaves this pending for
  // the rank exchange (isa = global ISA replica, upd = (position, ISA) pairs of the last step).
  struct DblState {
    int cur = 0;
    uint64_t A = 0, groups = 0, h = 0;
    uint64_t npairs = 0;       // pairs in upd from the last step
    bool pending = false;
    bool big = false;          // a round had a group over SEG_MAX members: the next ones sort the list at once
    bool link = false;         // one GPU, n < 2^31: groups that map whole onto one tied group are linked (hk_seground)
    uint64_t nlinked = 0;      // linked positions
    uint32_t ltag = 0;         // linking rounds run (links come from the first doubling round only)
    uint32_t lk_h = 0;         // that round's offset: a link names the position hops x lk_h further
    std::vector<uint64_t> lround;   // linked groups recorded up to each linking round
  } dbl;
  DevBuf upd;

  KernelTimer timer;
  std::vector<uint64_t> info;  // build counters (see hkcsa_build_info)

  WtView view() const;
};

void sa_to_host_u64(Index& ix, uint64_t lo, uint64_t c, uint64_t* out);
void byte_hist_range(Index& ix, uint64_t lo, uint64_t hi, unsigned long long* d_out);
void set_alphabet(Index& ix, const uint64_t* h);
void compute_alphabet(Index& ix);
void build_sa(Index& ix);
void build_bwt(Index& ix);
void bwt_gather64(Index& ix, const uint64_t* d_sa);   // BWT over a caller SA (u64)
void build_wt(Index& ix);
void release_workspace(Index& ix);
void synth_text(uint8_t* d_text, uint64_t n, const uint8_t* alphabet, int sigma, uint64_t seed,
                uint8_t terminator, hipStream_t s);

// queries (device-resident inputs and outputs)
// (a pattern whose end offset precedes its start or passes `lim` is not read; it sets *d_bad)
void query_count(Index& ix, const uint8_t* d_pats, const uint64_t* d_offs, uint64_t P,
                 int64_t* d_lr, uint64_t* d_cnt, uint64_t lim, uint32_t* d_bad);
void query_locate_gather(Index& ix, const int64_t* d_lr, const uint64_t* d_occ_offs, uint64_t P,
                         uint64_t* d_pos);
void query_rank(Index& ix, const uint8_t* d_c, const uint64_t* d_i, uint64_t k, uint64_t* d_out);
void wt_level_words(Index& ix, int depth, uint64_t* d_words);

// SA sampling: samples every `rate` text positions, exact-LF fix table; compact() drops SA, BWT
// array, text and workspace, after which SA / BWT / text are answered by LF walks
void build_samples(Index& ix, uint32_t rate);
void compact(Index& ix);
void sampled_locate_gather(Index& ix, const int64_t* d_lr, const uint64_t* d_occ_offs, uint64_t P, uint64_t* d_pos);
void sampled_sa_range(Index& ix, uint64_t lo, uint64_t count, uint64_t* d_out);
void wt_bwt_range(Index& ix, uint64_t lo, uint64_t count, uint8_t* d_out);
void sampled_extract(Index& ix, uint64_t i, uint64_t j, uint8_t* d_out);

// empirical k-th order entropy of T' (csa/high_order_entropy.py:4-32) from SA runs
double entropy_k(Index& ix, int k);

// Golomb-Rice code of the first nbits bits of a level (csa/wavelet_tree.py:27-63); with write,
// the code words are left in ix.gr_out
struct GolombResult {
  uint32_t m = 1;
  uint64_t ones = 0, bits = 0;
};
uint32_t golomb_m(uint64_t ones, uint64_t total);
GolombResult wt_golomb(Index& ix, int depth, uint64_t nbits, uint32_t m_override, bool write);

// sharded SA (RCCL)
int shard_buckets();
void shard_histogram(Index& ix, int nranks, int rank, uint64_t* d_hist);
void shard_counts(Index& ix, const uint64_t* h_global_hist, int nranks, int rank, uint64_t* d_below);
void shard_build(Index& ix, const uint64_t* h_global_hist, const uint64_t* h_global_below, int nranks, int rank);
int shard_sample();
void shard_get_sa(Index& ix, uint64_t a, uint64_t b, uint64_t* out);
void shard_get_bwt(Index& ix, uint64_t a, uint64_t b, uint8_t* out);
void build_sa_sharded(Index& ix, const uint8_t id[128], int nranks, int rank);
// one GPU, k slices of the final SA built one after another into one full SA / BWT (n >= 2^32 - 1, or
// kFlagSlices); slices_for(): the slice count build_sa uses
void build_sa_slices(Index& ix, int k);
int slices_for(const Index& ix);
// the keyed slice bounds of an exact coarse histogram (below[0..k]); throws when a slice would hold
// 2^32 - 1 or more suffixes (32-bit slots inside a slice)
std::vector<uint64_t> slice_bounds(const uint64_t* hist, int nbins, int k);
void check_slice_sizes(const uint64_t* below, int k);
void shard_replicate(Index& ix);                                          // RCCL: full SA + BWT on every rank
void shard_adopt(Index& ix, const uint64_t* h_sa, const uint8_t* h_bwt);  // host-assembled full SA + BWT
// host-driven rank exchange of the sharded prefix doubling (hkcsa_shard_status ... hkcsa_shard_round)
void shard_status(Index& ix, uint64_t st[4]);
void shard_isa_segment_host(Index& ix, const uint64_t* h_sa, uint64_t count, uint64_t lo);
uint64_t shard_updates(Index& ix, uint64_t* h_pairs, uint64_t cap);
void shard_apply_host(Index& ix, const uint64_t* h_pairs, uint64_t count);
void shard_round(Index& ix, uint64_t K);
void comm_unique_id(uint8_t id[128]);

// shared by the single-GPU and sharded builds
KeyGeom key_geometry(Index& ix, bool with_prev);
// keyed layout; reserve = low key bits kept free; q >= min_q, sym bits <= max_sb (sharded slices)
KeyGeom key_geometry_keyed(Index& ix, int reserve = 0, int min_q = 1, int max_sb = 64);
void build_sa_bucketed(Index& ix);       // single-GPU SA + BWT: 2 LSD passes + LDS bucket sorts
// Bucket bins of one slice's sym fields, all within [kmin, kmax]: shift bins (sym - kmin) >> bsh, or
// multiplicative bins hi64((sym - kmin) * mul) (exactly 2^16 over the range, stored in the key at
// bit binpos) where shift bins would waste half of the range.  D = 0: one bin.
struct SliceBins {
  uint64_t kmin = 0, kmax = 0, mul = 0;
  int bsh = 0;      // shift bins: the shift; mul bins: an upper bound on one bin's sym bits
  int D = 0, binpos = 0;
};
SliceBins slice_bins(uint64_t m, const KeyGeom& kg, int hb, uint64_t kmin, uint64_t kmax, bool force_mul);
// Bucket build of one sharded slice: m keyed keys [bin][sym][prev][position bits 32.., hb bits] in
// keys[0] (bin field in mul mode only), low position bits (u32) in vals[0], d_h0 = histogram of the
// bins' low byte.  Writes the slice's SA (V) and BWT and refines ties; false (nothing written) when
// a bucket exceeds one LDS sort.
template <typename V>
bool bucket_sort_slice(Index& ix, const KeyGeom& kg, uint64_t m, int hb, const SliceBins& bins, const uint64_t* d_h0);
// Keyed coarse scheme of the sharded build (texts whose keyed radix is 2^lb, lb in {1, 2, 4, 8}): the
// partition bucket of a suffix is the top 16 bits of its keyed sym field (its first 16 / lb symbols).
int shard_keyed_lb(Index& ix);                                               // lb, 0: scheme not applicable
bool shard_keyed(Index& ix);                                                 // the keyed scheme applies
void shard_coarse_hist(Index& ix, uint64_t lo, uint64_t hi, uint64_t* d_hist);   // exact, 65536 bins, [lo, hi)
// build_sa_slices: one fused pass A over T' for the slices [r0, r1) (coarse splitters B, SA bounds
// below); false (nothing kept) when the group does not qualify, else ix.fused holds the slices' records
// and cursors until build_slice_keyed consumes them
bool slices_fuse(Index& ix, const std::vector<uint32_t>& B, const std::vector<uint64_t>& below, int r0, int r1,
                 bool u64pos);
// SA + BWT of the slice of coarse buckets [c_lo, c_hi) (m suffixes): fused selection + cursor partition
// over the whole text, LDS bucket sorts, tie refinement (ties outlasting the chunk rounds left pending)
template <typename V>
void build_slice_keyed(Index& ix, uint32_t c_lo, uint32_t c_hi, uint64_t m);
// tie list (J << 1 | head, P) of m entries in (k, v) -> refinement loop (from symbol offset h)
template <typename V>
void refine_from_ties(Index& ix, const KeyGeom& kg, uint64_t A, bool allow_doubling);
template <typename V>
void refine_loop(Index& ix, const KeyGeom& kg, int cur, uint64_t A, uint64_t groups, bool allow_doubling,
                 const uint8_t* B0 = nullptr);

// Prefix doubling over the tied suffixes (hk_sa.hip).  allow_doubling = true above runs it locally
// (single GPU: ISA from the full SA); with false, refine_loop stops after its chunk rounds with
// ix.dbl pending and the sharded driver runs these steps around a rank exchange of ISA values.
void dbl_isa_segment(Index& ix, const void* d_sa, uint64_t count, uint64_t lo);   // isa[sa[j]] = lo + j
void dbl_emit_groups(Index& ix);            // upd = (P, slot of its group head) of the tied suffixes
void dbl_apply_pairs(Index& ix, const uint64_t* d_pairs, uint64_t count);   // isa[p] = v
void dbl_round(Index& ix, uint64_t K);      // one doubling round at offset dbl.h; dbl.h += K
void dbl_ensure_isa(Index& ix);
void dbl_isa_init_single(Index& ix);       // one GPU, u32 positions: ISA by bucketed scatter + tied head slots
// SA/BWT of A sorted (keys, P) at slots J; ties (compared >> cs) compacted to (oP, oJ, oG)
std::pair<uint64_t, uint64_t> refine_step_u32(Index& ix, const KeyGeom& kg, const uint64_t* keys,
                                              const uint32_t* P, const uint32_t* J, uint64_t A, int cs,
                                              uint32_t* oP, uint32_t* oJ, uint32_t* oG);
void upload_geometry(Index& ix, const KeyGeom& kg);
void pack_keys(const uint8_t* d_text, uint64_t n, uint64_t lo, uint64_t count, const uint16_t* d_lut, uint64_t R,
               int q, int pb, uint64_t* d_keys, hipStream_t s, uint64_t* d_hist0 = nullptr);
template <typename V>
void refine_after_sort(Index& ix, const KeyGeom& kg, int slot, uint64_t m, bool allow_doubling);

}  // namespace hk
