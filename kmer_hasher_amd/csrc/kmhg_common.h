// kmhg_common.h -- shared device/host definitions of the MI355X k-mer position index.
//
// Layout in HBM (one index, one GPU):
//   seq        u8[L]              the ASCII sequence (device copy, 16-B aligned)
//   table      Slot[cap + 1]      open-addressing hash table, linear probing, load <= 0.7;
//                                 slot[cap] is the side slot of the one key equal to the
//                                 empty sentinel (only possible at k = 32: GGG...G = ~0)
//   win_slot   u32[Nw]            build scratch: slot of every window start (or NONE)
//   ukeys      u64[U]   counts u32[U]   offsets u32[U+1]     CSR, keys in table-slot order
//   positions  i32[N]             1-based window starts of keys seen >= 2 times, ascending
//                                 inside every key (entries of keys seen once are unused)
// The table slot of a key also carries {count, aux}: aux = the position itself for a key seen
// once (the common case: a query probe then needs no second read), else one past the key's
// last position in `positions`, whose list is [aux - count, aux).
#pragma once
#include <stdint.h>

namespace kmhg {

constexpr uint64_t EMPTY_KEY = ~0ull;
constexpr uint32_t NONE = 0xFFFFFFFFu;

struct alignas(16) Slot {
  uint64_t key;    // EMPTY_KEY when free
  uint32_t count;  // occurrences of key
  uint32_t aux;    // count == 1: the 1-based position; count >= 2: end of its list in positions
};

// Table geometry: nb buckets x capb slots, plus one side slot at index nb*capb (kmhg_device.h).
// A part build (owner-computes multi-GPU build) holds buckets [b0, b0 + nb) of a table of nbh
// buckets: keys hash over nbh buckets, the part's arrays are indexed by bucket - b0.  A whole
// table has b0 = 0 and nbh = 0 (= nb).
struct Geom {
  uint32_t nb;
  uint32_t capb;
  uint32_t b0 = 0;
  uint32_t nbh = 0;
};

// Build-time tile geometry: one workgroup = 256 lanes x WPT windows, staged through LDS.
constexpr int BLOCK = 256;
constexpr int WPT = 8;
constexpr int TILE = BLOCK * WPT;          // windows per workgroup
constexpr int HALO = 32;                   // chars staged before/after the tile (k <= 32)
constexpr int STAGE = TILE + 2 * HALO + 16;  // chars staged per workgroup (+16: base aligned down)
constexpr int STAGE_W16 = STAGE / 16;      // 16-char words staged
// Partition tile of the radix passes of the partitioned build (longer digit runs per tile ->
// longer contiguous scatter writes)
constexpr int PWPT = 8;
constexpr int PTILE = BLOCK * PWPT;
constexpr int PSTAGE = PTILE + 2 * HALO + 16;
constexpr int PSTAGE_W16 = PSTAGE / 16;

// murmur3 fmix64: keys are structured (2-bit packed DNA); khash's (key>>33)^key^(key<<11)
// truncated to 32 bits is weak on them (SURVEY.md §7 "Random-access hash traffic").
__host__ __device__ inline uint64_t mix64(uint64_t h) {
  h ^= h >> 33; h *= 0xff51afd7ed558ccdull;
  h ^= h >> 33; h *= 0xc4ceb9fe1a85ec53ull;
  h ^= h >> 33;
  return h;
}

}  // namespace kmhg
