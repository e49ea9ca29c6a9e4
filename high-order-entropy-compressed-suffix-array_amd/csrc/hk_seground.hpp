// hk_seground.hpp — one refinement / prefix-doubling round's sort + regroup over the tie list in LDS items of
// whole groups (hk_seground.hip); the groups of more than SR_W members take the global path (hk_sa.hip).
#pragma once

#include <utility>

#include "hk_index.hpp"

namespace hk {

// list entries per window; an item = the groups whose head is in one window.  1024 (51 KB of LDS per item
// workgroup) lets three 512-thread workgroups share a CU where 2048 (76 KB) allowed two: English-like 200 MiB
// 57.0-57.7 -> 56.4 ms per step, protein-like 1 GiB 125.3 -> 123.3 ms (the groups of 1025-2048 members move to
// the global big-group sort)
constexpr int SR_W = 1024;
constexpr int SR_CAP = 2 * SR_W;    // an item holds fewer entries than this

template <typename V>
struct SrRoundArgs {
  const uint64_t* keys;    // the round's keys (G in the top bits), list order
  const V* vals;           // positions, list order
  const uint32_t* G;       // group ordinals (ascending along the list)
  const uint32_t* J;       // SA slots (contiguous and ascending inside a group)
  const uint2* items;      // (sr_plan)
  unsigned long long* counter;   // next list: entries | groups << 33 (from 0; the items' output starts at
  uint64_t base_e, base_g;       //   entry base_e, group base_g: after the big groups')
  V* oP;
  uint32_t* oJ;
  uint32_t* oG;
  uint32_t* head_slot;
  V* sa;
  uint8_t* bwt;
  const uint8_t* t;
  const uint8_t* B;         // (nullable, chunk rounds) the entries' BWT bytes in list order: no text gather
  uint64_t n;
  V* isa;                  // doubling: ISA (single GPU or one-GPU slices; global slot = lo + slot)
  uint64_t lo;
  int keep_same;           // doubling: skip the ISA entries a round leaves unchanged
  uint32_t* hp_next;       // (nullable) the next round's plan: head entry of every new group, and
  uint32_t* win_next;      //   every window's {first, last} head entry (reset by sr_plan)
  // doubling links (nullable lnk: off).  A group whose members' keys are all ISA[p + h] = K (one tied group) and
  // whose size equals that group's (gsz[K], saturated at 255) is a shifted copy of it: its members leave the
  // list with lnk[p] = own head slot - K (never 0); the chain pass then marks isa[p] = LK_BIT | hops and
  // composes lnk, so ISA(p) = ISA(p + hops h) + lnk[p] at every later precision (csa/suffix_array.py:131-134:
  // suffix p orders as suffix p + h inside the group).
  uint32_t* lnk;
  const uint8_t* gsz;
  unsigned long long* lcount;   // linked entries of the round
  unsigned long long* gcount;   // linked groups (all rounds): records grec[] = {head slot, size, head position}
  uint4* grec;
  uint32_t h;
  int ib;                  // key bits below the group ordinal
};

constexpr uint32_t LK_BIT = 0x80000000u;   // isa[p] of a linked position

// Windows, items and big groups of list `slot` (A entries in `groups` groups): ix.sr_items, ix.grp_big (u8 per
// group, 1 = big).  heads_ready: the previous round already wrote the list's group heads and window bounds
// (ix.sr_hp[slot], ix.sr_win[slot]).  Also readies the next list's plan buffers (slot ^ 1: windows reset).
// Returns the entries in big groups (*big_groups: their number).
uint64_t sr_plan(Index& ix, int slot, const uint32_t* G, uint64_t A, uint64_t groups, bool heads_ready,
                 uint64_t* big_groups);
// group heads + window bounds of list entries [lo, hi) (lo a multiple of 64), into list `slot`'s plan
void sr_heads(Index& ix, int slot, const uint32_t* G, uint64_t lo, uint64_t hi, uint64_t A, uint64_t groups);

// The LDS items of the round (mode 0: chunk refinement, 1: doubling); the next list already holds tied0
// entries in groups0 groups (the big groups').  Returns the next list's (entries, groups).
template <typename V>
std::pair<uint64_t, uint64_t> sr_items_round(Index& ix, int mode, SrRoundArgs<V> args, uint64_t A, uint64_t tied0,
                                             uint64_t groups0, uint64_t* linked = nullptr);

// doubling links (u32 positions, n < 2^31): buffers (lk_begin); gsz of list `slot`'s groups before a round
// (lk_sizes); after the round that linked entries: resolve their chains (lk_after_round); SA / BWT of every
// linked group once the list is empty (lk_resolve)
void lk_begin(Index& ix);
uint64_t lk_max_offset();   // the largest doubling offset whose chains the link tiles resolve
void lk_sizes(Index& ix, int slot, uint64_t A, uint64_t groups);
void lk_after_round(Index& ix, uint64_t linked, uint32_t h);
void lk_resolve(Index& ix);

}  // namespace hk
