// hk_seground.hpp — one refinement / prefix-doubling round's sort + regroup over the tie list in LDS items of
// whole groups (hk_seground.hip); the groups of more than SR_W members take the global path (hk_sa.hip).
#pragma once

#include <utility>

#include "hk_index.hpp"

namespace hk {

constexpr int SR_W = 2048;          // list entries per window; an item = the groups whose head is in one window
constexpr int SR_CAP = 2 * SR_W;    // an item holds fewer entries than this

template <typename V>
struct SrRoundArgs {
  const uint64_t* keys;    // the round's keys (G in the top bits), list order
  const V* vals;           // positions, list order
  const uint32_t* G;       // group ordinals (ascending along the list)
  const uint32_t* J;       // SA slots (contiguous and ascending inside a group)
  const uint2* items;      // (sr_plan)
  unsigned long long* counter;   // next list: entries | groups << 33
  V* oP;
  uint32_t* oJ;
  uint32_t* oG;
  uint32_t* head_slot;
  V* sa;
  uint8_t* bwt;
  const uint8_t* t;
  uint64_t n;
  V* isa;                  // doubling: ISA (single GPU or one-GPU slices; global slot = lo + slot)
  uint64_t lo;
  int keep_same;           // doubling: skip the ISA entries a round leaves unchanged
};

// Windows, items and big groups of a list of A entries in `groups` groups: ix.sr_items, ix.grp_big (u8 per
// group, 1 = big).  Returns the entries in big groups (*big_groups: their number).
uint64_t sr_plan(Index& ix, const uint32_t* G, uint64_t A, uint64_t groups, uint64_t* big_groups);

// The LDS items of the round (mode 0: chunk refinement, 1: doubling); the next list already holds tied0
// entries in groups0 groups (the big groups').  Returns the next list's (entries, groups).
template <typename V>
std::pair<uint64_t, uint64_t> sr_items_round(Index& ix, int mode, SrRoundArgs<V> args, uint64_t A, uint64_t tied0,
                                             uint64_t groups0);

}  // namespace hk
