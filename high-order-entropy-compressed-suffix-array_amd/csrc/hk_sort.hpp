// hk_sort.hpp — device-wide primitives: exclusive scans and the onesweep LSD
// radix sort of (u64 key, V value) pairs used by prefix doubling.
#pragma once

#include "hk_common.hpp"
#include "hk_keys.hpp"

namespace hk {

// Workspace shared by the sort and scan primitives of one index/stream.
struct SortWork {
  DevBuf status;       // lookback granules: tiles x 256 x u64 (epoch | flag | value)
  DevBuf counters;     // dynamic tile-id counters, one per pass (64 x u32)
  DevBuf hist;         // 9 x 256 u64 digit histograms (row p = digit p of the current sort)
  DevBuf hpart;        // 64 x 256 u64 partial histograms of the next digit, written by a pass
  DevBuf offs;         // 8 x 256 u64 exclusive digit offsets
  DevBuf err;          // u32 error flag (lookback spin bound exceeded)
  HostBuf herr;        // its pinned landing slot
  DevBuf scan_tmp;     // scan partials (multi-level)
  uint32_t epoch = 0;  // lookback epoch of the last pass (16 bits used)
  uint64_t status_tiles = 0;
  // host mirror of the last histogram (digit skipping)
  uint64_t h_hist[8 * 256];
  // counters of the last sort
  uint32_t passes_run = 0, passes_skipped = 0;
};

// out[i] = sum(in[0:i)) for u64 arrays (in and out may alias). Returns total via *total (device ptr
// nullable) — the total is written to out[count] when write_total is set (out must hold count+1).
void scan_exclusive_u64(SortWork& w, const uint64_t* in, uint64_t* out, uint64_t count,
                        bool write_total, hipStream_t s);
// Same for u32 input counts (u64 output).
void scan_exclusive_u32_to_u64(SortWork& w, const uint32_t* in, uint64_t* out, uint64_t count,
                               bool write_total, hipStream_t s);
// out[i] = max(in[0:i)) with identity 0 (u64).
void scan_exclusive_max_u64(SortWork& w, const uint64_t* in, uint64_t* out, uint64_t count,
                            hipStream_t s);

// Stable LSD radix sort of n pairs on key bits [bit_lo, bit_hi).  Ping-pongs between
// (k[0],v[0]) and (k[1],v[1]); the input is in slot `in_slot`; returns the slot holding the
// result.  If vals_iota, the values of the input are taken to be 0..n-1 (v[in_slot] unused).
// d_hist0 (nullable): device histogram (256 x u64) of the first digit, if the key producer
// already computed it.  Each pass computes the next digit's histogram on the fly; digits whose
// histogram shows a single bucket are skipped.
// src (nullable): the first pass builds the keys from the text (k[in_slot] unused; vals_iota required).
// kbias: digits are taken from key - kbias (every key >= kbias; the keys themselves are unchanged).
template <typename V>
int radix_sort_pairs(SortWork& w, KernelTimer& tm, uint64_t* k[2], V* v[2], int in_slot, uint64_t n, int bit_lo,
                     int bit_hi, bool vals_iota, hipStream_t s, const uint64_t* d_hist0 = nullptr,
                     const TextKeySrc* src = nullptr, uint64_t kbias = 0);

// diagnostics: per-pass ms of onesweep variants {512x16, 512x16 no-lookback, 512x16 no-lookback
// no-staging, 256x16, 256x16 no-lookback, 1024x8} and of a plain pair copy; out[7] = error flag
void debug_radix_bench(SortWork& w, uint64_t* k[2], uint32_t* v[2], uint64_t n, int bit_lo, int reps,
                       double* out, int nout, hipStream_t s);

// fill v[i] = i
template <typename V>
void fill_iota(V* v, uint64_t n, hipStream_t s);

}  // namespace hk
