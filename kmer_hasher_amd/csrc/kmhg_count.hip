// kmhg_count.hip -- count.kmers: per-source k-mer counts held in a GPU counts index.
//
// Replaces count_kmers (reference src/kmer_hash.c:548-591) with seq_to_counts (:220-251) and
// kmer_count_insert (:185-208): every valid window of a sequence adds one to slot `source` of
// its key's vector of `source_n` counts; keys are kept in first-insertion order.
//
// A count.kmers call is one partitioned build of the batch (the distinct keys with their
// occurrence counts, in first-occurrence order = the readout permutation) merged into the
// counts index:
// perm_b = nullptr walks the batch table's slots instead (order-free merges: the read counts of
// kmhg_sh.hip), empty slots contributing nothing.
//   C_probe   batch key r -> one probe of the counts table; a known key adds its count to its
//             row (distinct keys own distinct rows: a plain read-modify-write), a new key
//             raises its flag
//   (k_scan_u32 of the flags: new rows keep first-occurrence order)
//   C_append  new key r -> row U0 + rank: key + a count vector with only `source` set
//   (table)   the table is rebuilt for the grown key list by the partitioned build run over the
//             key stream (values = row + 1), then C_fix gives each slot {key, count = source_n,
//             aux}, aux = the count itself for source_n = 1 (the inline convention of the
//             position index), else the end of the row's vector.  C_insert (global linear
//             probing, nb = 1) is the fallback should a bucket overflow.
//   C_canon   readout arrays in row order (perm, row offsets, keys owning pairs)
// The count matrix (U x source_n int32, row-major) takes the place of `positions`, so
// kmer.pos and seq.kmer.pos read a counts index with the position index's kernels -- the
// reference's kmer_positions / sequence_kmer_positions equally read count vectors as positions.
#include <hip/hip_runtime.h>
#include "kmhg_common.h"
#include "kmhg_device.h"
#include "kmhg_kernels.h"

namespace kmhg {

__global__ void __launch_bounds__(BLOCK)
k_count_probe(const uint32_t* __restrict__ perm_b, uint32_t Ub, const Slot* __restrict__ Tb,
              const Slot* __restrict__ Tc, Geom gc, const uint32_t* __restrict__ slot_row,
              uint32_t S, uint32_t source, int32_t* __restrict__ M, uint32_t* __restrict__ newf) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= Ub) return;
  const uint4 v = *reinterpret_cast<const uint4*>(&Tb[perm_b ? perm_b[r] : r]);
  if (!perm_b && !v.z) { newf[r] = 0; return; }        // slot walk: an empty slot adds nothing
  const uint64_t key = ((uint64_t)v.y << 32) | v.x;
  uint32_t f = 1;
  if (Tc) {
    uint32_t c = 0, aux = 0;
    const uint32_t slot = table_find(Tc, gc, key, c, aux);
    if (slot != NONE) {
      M[(uint64_t)slot_row[slot] * S + source] += (int32_t)v.z;
      f = 0;
    }
  }
  newf[r] = f;
}

__global__ void __launch_bounds__(BLOCK)
k_count_append(const uint32_t* __restrict__ perm_b, uint32_t Ub, const Slot* __restrict__ Tb,
               const uint32_t* __restrict__ rank, const uint32_t* __restrict__ n_new,
               uint32_t U0, uint32_t S, uint32_t source, uint64_t* __restrict__ ckeys,
               int32_t* __restrict__ M) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= Ub) return;
  const uint32_t o = rank[r];
  const uint32_t nx = r + 1 < Ub ? rank[r + 1] : *n_new;
  if (nx == o) return;                                  // known key (or an empty slot)
  const uint4 v = *reinterpret_cast<const uint4*>(&Tb[perm_b ? perm_b[r] : r]);
  const uint64_t row = (uint64_t)U0 + o;
  ckeys[row] = ((uint64_t)v.y << 32) | v.x;
  for (uint32_t j = 0; j < S; ++j) M[row * S + j] = j == source ? (int32_t)v.z : 0;
}

__global__ void __launch_bounds__(BLOCK)
k_count_insert(const uint64_t* __restrict__ ckeys, uint32_t U, Slot* __restrict__ T, Geom g,
               uint32_t S, const int32_t* __restrict__ M, uint32_t* __restrict__ slot_row,
               uint32_t* __restrict__ row_slot) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= U) return;
  const uint32_t slot = table_insert(T, g, ckeys[r]);   // distinct keys: always a fresh slot
  T[slot].count = S;
  T[slot].aux = S == 1 ? (uint32_t)M[r] : (r + 1) * S;
  slot_row[slot] = r;
  row_slot[r] = slot;
}

__global__ void __launch_bounds__(BLOCK)
k_count_canon(const uint32_t* __restrict__ row_slot, uint32_t U, uint32_t S,
              uint32_t* __restrict__ perm, uint32_t* __restrict__ canon_off,
              uint32_t* __restrict__ pkeys, uint64_t* __restrict__ pair_off) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r > U) return;
  canon_off[r] = r * S;
  if (r == U) return;
  perm[r] = row_slot[r];
  if (S >= 2) {
    pkeys[r] = r;
    pair_off[r] = (uint64_t)r * ((uint64_t)S * (S - 1) / 2);
  }
}

// C_adopt: the first batch merged into an empty counts index.  Every batch key is new, so the
// batch table itself becomes the counts table: item r (slot perm_b[r], row r; or slot r, whose
// row the scan of the occupancy flags gave) writes its row's key and count vector, the
// slot <-> row maps, and rewrites its slot in place with the counts-index fields.  One pass in
// place of probe / append / table rebuild / C_fix.
__global__ void __launch_bounds__(BLOCK)
k_count_adopt(const uint32_t* __restrict__ perm_b, uint32_t n_items, Slot* __restrict__ T,
              const uint32_t* __restrict__ rank, uint32_t S, uint32_t source,
              uint64_t* __restrict__ ckeys, int32_t* __restrict__ M,
              uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= n_items) return;
  const uint32_t slot = perm_b ? perm_b[r] : r;
  const uint4 v = *reinterpret_cast<const uint4*>(&T[slot]);
  if (!v.z) return;                                     // slot walk: an empty slot
  const uint32_t row = perm_b ? r : rank[r];
  ckeys[row] = ((uint64_t)v.y << 32) | v.x;
  int32_t* m = M + (uint64_t)row * S;
  for (uint32_t j = 0; j < S; ++j) m[j] = j == source ? (int32_t)v.z : 0;
  slot_row[slot] = row;
  row_slot[row] = slot;
  *reinterpret_cast<uint2*>(&T[slot].count) = make_uint2(S, S == 1 ? v.z : (row + 1) * S);
}

// values base, base + 1, ... of the key stream of a table rebuild
__global__ void __launch_bounds__(BLOCK) k_iota_u32(uint32_t* __restrict__ a, uint64_t n,
                                                    uint32_t base) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * BLOCK)
    a[i] = base + (uint32_t)i;
}

// C_fix: a table rebuilt by the partitioned build from the key list holds {key, 1, row + 1};
// give every occupied slot its counts-index fields and record the slot <-> row maps.
__global__ void __launch_bounds__(BLOCK)
k_count_fix(Slot* __restrict__ T, uint64_t nslots, uint32_t S, const int32_t* __restrict__ M,
            uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * BLOCK) {
    const uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
    if (!v.z) continue;
    const uint32_t r = v.w - 1;
    T[i].count = S;
    T[i].aux = S == 1 ? (uint32_t)M[r] : (r + 1) * S;
    slot_row[i] = r;
    row_slot[r] = (uint32_t)i;
  }
}

static inline unsigned grid_of(uint64_t n) { return (unsigned)((n + BLOCK - 1) / BLOCK); }
static inline unsigned grid_cap(uint64_t n) {
  const unsigned g = grid_of(n);
  return g > 16384 ? 16384 : (g ? g : 1);
}

void launch_count_probe(const uint32_t* perm_b, uint32_t Ub, const Slot* Tb, const Slot* Tc,
                        Geom gc, const uint32_t* slot_row, uint32_t S, uint32_t source,
                        int32_t* M, uint32_t* newf, hipStream_t s) {
  hipLaunchKernelGGL(k_count_probe, dim3(grid_of(Ub)), dim3(BLOCK), 0, s, perm_b, Ub, Tb, Tc, gc,
                     slot_row, S, source, M, newf);
}
void launch_count_append(const uint32_t* perm_b, uint32_t Ub, const Slot* Tb,
                         const uint32_t* rank, const uint32_t* n_new, uint32_t U0, uint32_t S,
                         uint32_t source, uint64_t* ckeys, int32_t* M, hipStream_t s) {
  hipLaunchKernelGGL(k_count_append, dim3(grid_of(Ub)), dim3(BLOCK), 0, s, perm_b, Ub, Tb, rank,
                     n_new, U0, S, source, ckeys, M);
}
void launch_count_insert(const uint64_t* ckeys, uint32_t U, Slot* T, Geom g, uint32_t S,
                         const int32_t* M, uint32_t* slot_row, uint32_t* row_slot,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_count_insert, dim3(grid_of(U)), dim3(BLOCK), 0, s, ckeys, U, T, g, S, M,
                     slot_row, row_slot);
}
void launch_count_adopt(const uint32_t* perm_b, uint32_t n_items, Slot* T, const uint32_t* rank,
                        uint32_t S, uint32_t source, uint64_t* ckeys, int32_t* M,
                        uint32_t* slot_row, uint32_t* row_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_count_adopt, dim3(grid_of(n_items)), dim3(BLOCK), 0, s, perm_b, n_items, T,
                     rank, S, source, ckeys, M, slot_row, row_slot);
}
void launch_iota_u32(uint32_t* a, uint64_t n, uint32_t base, hipStream_t s) {
  hipLaunchKernelGGL(k_iota_u32, dim3(grid_cap(n)), dim3(BLOCK), 0, s, a, n, base);
}
void launch_count_fix(Slot* T, uint64_t nslots, uint32_t S, const int32_t* M, uint32_t* slot_row,
                      uint32_t* row_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_count_fix, dim3(grid_cap(nslots)), dim3(BLOCK), 0, s, T, nslots, S, M,
                     slot_row, row_slot);
}
void launch_count_canon(const uint32_t* row_slot, uint32_t U, uint32_t S, uint32_t* perm,
                        uint32_t* canon_off, uint32_t* pkeys, uint64_t* pair_off,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_count_canon, dim3(grid_of((uint64_t)U + 1)), dim3(BLOCK), 0, s, row_slot,
                     U, S, perm, canon_off, pkeys, pair_off);
}

}  // namespace kmhg
