// hk_bucket.hpp — definitions shared by the bucket build (hk_bucket.hip) and its LDS item sorts
// (hk_bsort.hip): packed-record geometry, slice selection, the bucket plan, the item capacities.
#pragma once

#include <vector>

#include "hk_index.hpp"

namespace hk {

constexpr int BS_T = 1024;
constexpr int BS_W = BS_T / 64;       // 16 waves
constexpr int BS_I = 18;              // suffixes per thread
constexpr int BS_H = BS_I / 2;        // 16-bit per-item values are packed two to a register
constexpr int BS_CAP = BS_T * BS_I;   // 18432 suffixes per workgroup
constexpr int BS_WSPAN = BS_I * 64;
constexpr int BS_V = BS_W;            // per-wave digit histograms, in element order

// the record-plane sort's items (k_bucket_sort_rec, hk_bsort.hip)
constexpr uint32_t BR_CAP = 9056;                 // suffixes per item (the 512-thread items' plan cap)

// Packed records of the single-GPU cursor partition (k_cpart PK, the PK item sorts): one u64 per
// suffix, (key bits below pass A's 9-bit digit) << pbits | position.  Their prev field is the keyed
// code (pb2 bits) when the terminal is unkeyed (tcode >= 0, the dense code of the terminal, which
// precedes only suffix 0): the BWT byte of position 0 is the terminal, every other code maps back
// as code + (code >= tcode).
// phb: position bits above 32 (sharded slices of texts with >= 2^32 suffixes, u64 SA entries).
struct PkGeom {
  int pbits = 0, pb = 0, pb2 = 0, tcode = -1, phb = 0;
};

struct SliceSel {
  uint32_t base = 0, nb = 0;   // first global bin of the slice, bins in the slice
  int bsh = 0, DB = 0;         // sym bits below a bin; sym bits above them
  int hq = 0, wdrop = 0;       // window of hq symbols (hq * lb bits), low wdrop bits dropped
  uint32_t g = 1;              // sub-tiles of CP_TILE positions per unit (pass A workgroup)
  int sA = 0;                  // pass B digit bits (the pass A digit = bin >> sA)
  int pbits = 0, pb2 = 0;      // packed records: position bits, prev-code bits (0: key / value planes)
  int pbe = 0;                 // key planes: prev + position-high bits below the relative sym field
  uint32_t wb = 0, wn1 = 0;    // REG: base << (32 - DB), (nb << (32 - DB)) - 1: a 32-bit window w is
                               // in the slice iff w - wb <= wn1 (its bin: (w - wb) >> (32 - DB))
  uint32_t tl = 0, th = 0;     // REG: keyed code of byte b = byte ((b >> ps) & 7) of {th, tl}
  int ps = -1;                 // REG: the byte's bit field (-1: no 3-bit field separates the keyed bytes)
};

struct BucketPlan {
  std::vector<uint2> items_n, items_w;       // {start, count}: narrow / wide local keys
  std::vector<uint64_t> big_start, big_cstart;
  uint64_t big_total = 0;
  uint64_t cap = BS_CAP;                     // suffixes per item: 18 432, or 9216 (512-thread fast sorts)
};

// the cursor partition's packed records (section 1b): record = key bits below the pass A digit
// (klw of them) << pbits | position; the items that need full keys are unpacked to (kfull, vfull)
struct PackedRecs {
  PkGeom g;                           // g.pbits > 0: packed
  int klw = 0;                        // key bits below pass A's digit, full layout
  uint16_t lutp2[256];                // byte -> prev code of the records (keyed code when g.tcode >= 0)
  const uint64_t* startA = nullptr;   // region starts (ndA + 1)
  uint32_t ndA = 0;
  uint64_t* kfull = nullptr;
  uint32_t* vfull = nullptr;
  int uhb = 0;                        // u64 positions: hb of the unpacked key layout
  bool reg = false;                   // radix 2^2 with a perm table: the register pre-pass (rsl)
  SliceSel rsl;                       // ... as a slice of every bucket
};

// diagnostic stamps (TRACE): shader-clock time at the phase boundaries
__device__ __forceinline__ uint64_t stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}

// Launches the LDS sorts of the plan's work items (hk_bsort.hip); returns the tie count.
template <typename V>
uint64_t sort_bucket_items(Index& ix, const BucketPlan& plan, const uint64_t* keys, const uint32_t* vals, uint64_t m,
                           int pb, int sb, int hb, uint64_t symbias, V* sa, uint8_t* bwt,
                           const PackedRecs* pk = nullptr);

// packed items that take the LSD item sort: unpacked to (kfull, vfull) (hk_bucket.hip)
void unpack_items(Index& ix, const PackedRecs& pk, const uint64_t* rec, const uint2* d_items, uint32_t nitems);

}  // namespace hk
