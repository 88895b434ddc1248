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
k_count_canon(const uint32_t* __restrict__ row_slot, const int32_t* __restrict__ M, uint32_t U,
              uint32_t S, uint32_t* __restrict__ perm, uint32_t* __restrict__ canon_off,
              uint32_t* __restrict__ pkeys, uint64_t* __restrict__ pair_off,
              uint2* __restrict__ rinfo) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r > U) return;
  canon_off[r] = r * S;
  if (r == U) return;
  perm[r] = row_slot[r];
  rinfo[r] = make_uint2(S, S == 1 ? (uint32_t)M[r] : (r + 1) * S);   // the slot's {count, aux}
  if (S >= 2) {
    pkeys[r] = r;
    pair_off[r] = (uint64_t)r * ((uint64_t)S * (S - 1) / 2);
  }
}

// The first batch of count.kmers into a new pointer, rows in first-occurrence order without a
// slot permutation: C_first scatters {slot, count, key} to the key's first position, C_order
// compacts that array in position order straight into the rows (key, count vector, row_slot,
// slot_row), C_slots rewrites the adopted table's slots in slot order.  The only random
// accesses left are C_first's 16-B stores and C_order's slot_row stores.
__global__ void __launch_bounds__(BLOCK)
k_count_first(const Slot* __restrict__ T, uint64_t nslots, const int32_t* __restrict__ positions,
              uint4* __restrict__ F) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * BLOCK) {
    const uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
    if (v.z)
      F[(v.z == 1 ? (int32_t)v.w : positions[v.w - v.z]) - 1] =
          make_uint4((uint32_t)i, v.z, v.x, v.y);
  }
}

// Compaction of one tile of TILE elements, element e = j * BLOCK + threadIdx.x (lane-contiguous:
// every load and store of a step is coalesced).  The flagged elements get consecutive ranks in
// element order -- (j, wave, lane) -- from per-(j, wave) ballots, offset by the flagged elements
// of the tiles before (one look-back chain).  `cw` = LDS for WPT * 4 u64.
template <int J = WPT>
__device__ __forceinline__ void tile_compact(const bool (&flag)[J], uint64_t (&rk)[J],
                                             uint64_t* cw, uint64_t* status, uint32_t tile) {
  const int wave = threadIdx.x >> 6, lane = lane_id();
  constexpr int NW = BLOCK / 64;
  uint64_t m[J];
#pragma unroll
  for (int j = 0; j < J; ++j) m[j] = __ballot(flag[j]);
  if (lane == 0) {
#pragma unroll
    for (int j = 0; j < J; ++j) cw[j * NW + wave] = (uint64_t)__popcll(m[j]);
  }
  __syncthreads();
  if (wave == 0) {                       // lanes 0 .. J*NW-1 own one (j, wave) count each
    const uint64_t c = lane < J * NW ? cw[lane] : 0;
    const uint64_t inc = wave_incl_scan(c);
    const uint64_t tot = __shfl(inc, 63);
    const uint64_t x = lookback_excl(status, tile, tot);
    if (lane < J * NW) cw[lane] = x + inc - c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j)
    rk[j] = cw[j * NW + wave] + (uint64_t)__popcll(m[j] & lanemask_lt());
}

// F: L entries in position order, slot NONE where no key starts.  `ticket` orders the tiles.
__global__ void __launch_bounds__(BLOCK)
k_count_order(const uint4* __restrict__ F, int64_t L, uint64_t* __restrict__ status,
              uint32_t* __restrict__ ticket, uint32_t S, uint32_t source,
              uint64_t* __restrict__ ckeys, int32_t* __restrict__ M,
              uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot) {
  __shared__ uint64_t cw[WPT * (BLOCK / 64)];
  __shared__ uint32_t tk;
  const uint32_t tile = take_ticket(ticket, &tk);
  const int64_t t0 = (int64_t)tile * TILE;
  uint4 f[WPT];
  bool fl[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int64_t p = t0 + (int64_t)j * BLOCK + threadIdx.x;
    f[j] = p < L ? F[p] : make_uint4(NONE, 0u, 0u, 0u);
    fl[j] = f[j].x != NONE;
  }
  uint64_t rk[WPT];
  tile_compact(fl, rk, cw, status, tile);
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (!fl[j]) continue;
    const uint64_t row = rk[j];
    ckeys[row] = ((uint64_t)f[j].w << 32) | f[j].z;
    int32_t* m = M + row * S;
    for (uint32_t q = 0; q < S; ++q) m[q] = q == source ? (int32_t)f[j].y : 0;
    row_slot[row] = f[j].x;
    slot_row[f[j].x] = (uint32_t)row;
  }
}

// The first batch into an empty suffix hash (order-free rows: slot order).  One pass over the
// adopted table in tiles of TILE slots: occupied slots are compacted into rows, each writes its
// row (key, count vector, row_slot), slot_row and its own slot fields -- every access coalesced.
// WALK_PER slots per thread: a longer tile halves the look-back chain over the sparse table
#ifndef KMHG_WALK_PER
#define KMHG_WALK_PER 16
#endif
constexpr int WALK_PER = KMHG_WALK_PER;
constexpr int WALK_TILE = BLOCK * WALK_PER;
// >= 3 waves per SIMD: unconstrained the walk holds 191 VGPRs (2 waves); capped, 166 with no
// spill.  A/B in one run (reads leg): k_count_walk 0.330 / 0.323 -> 0.309 / 0.303 ms.
#ifndef KMHG_WALK_WAVES
#define KMHG_WALK_WAVES 3
#endif
#if KMHG_WALK_WAVES
#define WALK_BOUNDS __launch_bounds__(BLOCK, KMHG_WALK_WAVES)
#else
#define WALK_BOUNDS __launch_bounds__(BLOCK)
#endif
__global__ void WALK_BOUNDS
k_count_walk(Slot* __restrict__ T, uint64_t nslots, uint64_t* __restrict__ status,
             uint32_t* __restrict__ ticket, uint32_t S, uint32_t source,
             uint64_t* __restrict__ ckeys, int32_t* __restrict__ M,
             uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot) {
  __shared__ uint64_t cw[WALK_PER * (BLOCK / 64)];
  __shared__ uint32_t tk;
  const uint32_t tile = take_ticket(ticket, &tk);
  const uint64_t t0 = (uint64_t)tile * WALK_TILE;
  uint4 v[WALK_PER];
  bool fl[WALK_PER];
#pragma unroll
  for (int j = 0; j < WALK_PER; ++j) {
    const uint64_t i = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    v[j] = i < nslots ? *reinterpret_cast<const uint4*>(&T[i]) : make_uint4(0u, 0u, 0u, 0u);
    fl[j] = v[j].z != 0;
  }
  uint64_t rk[WALK_PER];
  tile_compact<WALK_PER>(fl, rk, cw, status, tile);
#pragma unroll
  for (int j = 0; j < WALK_PER; ++j) {
    if (!fl[j]) continue;
    const uint64_t i = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    const uint64_t row = rk[j];
    ckeys[row] = ((uint64_t)v[j].y << 32) | v[j].x;
    int32_t* m = M + row * S;
    for (uint32_t q = 0; q < S; ++q) m[q] = q == source ? (int32_t)v[j].z : 0;
    row_slot[row] = (uint32_t)i;
    slot_row[i] = (uint32_t)row;
    *reinterpret_cast<uint2*>(&T[i].count) =
        make_uint2(S, S == 1 ? v[j].z : ((uint32_t)row + 1) * S);
  }
}

__global__ void __launch_bounds__(BLOCK)
k_count_slots(Slot* __restrict__ T, uint64_t nslots, uint32_t S,
              const uint32_t* __restrict__ slot_row) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * BLOCK) {
    const uint32_t c = T[i].count;
    if (!c) continue;
    *reinterpret_cast<uint2*>(&T[i].count) = make_uint2(S, S == 1 ? c : (slot_row[i] + 1) * S);
  }
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
void launch_count_first(const Slot* T, uint64_t nslots, const int32_t* positions, uint4* F,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_count_first, dim3(grid_cap(nslots)), dim3(BLOCK), 0, s, T, nslots,
                     positions, F);
}
void launch_count_order(const uint4* F, int64_t L, uint64_t* status, uint32_t* ticket, uint32_t S,
                        uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                        uint32_t* row_slot, hipStream_t s) {
  const unsigned nt = (unsigned)(((uint64_t)L + TILE - 1) / TILE);
  hipLaunchKernelGGL(k_count_order, dim3(nt), dim3(BLOCK), 0, s, F, L, status, ticket, S, source,
                     ckeys, M, slot_row, row_slot);
}
uint64_t count_walk_tiles(uint64_t nslots) { return (nslots + WALK_TILE - 1) / WALK_TILE; }
void launch_count_walk(Slot* T, uint64_t nslots, uint64_t* status, uint32_t* ticket, uint32_t S,
                       uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                       uint32_t* row_slot, hipStream_t s) {
  const unsigned nt = (unsigned)((nslots + WALK_TILE - 1) / WALK_TILE);
  hipLaunchKernelGGL(k_count_walk, dim3(nt), dim3(BLOCK), 0, s, T, nslots, status, ticket, S,
                     source, ckeys, M, slot_row, row_slot);
}
void launch_count_slots(Slot* T, uint64_t nslots, uint32_t S, const uint32_t* slot_row,
                        hipStream_t s) {
  hipLaunchKernelGGL(k_count_slots, dim3(grid_cap(nslots)), dim3(BLOCK), 0, s, T, nslots, S,
                     slot_row);
}
void launch_count_fix(Slot* T, uint64_t nslots, uint32_t S, const int32_t* M, uint32_t* slot_row,
                      uint32_t* row_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_count_fix, dim3(grid_cap(nslots)), dim3(BLOCK), 0, s, T, nslots, S, M,
                     slot_row, row_slot);
}
void launch_count_canon(const uint32_t* row_slot, const int32_t* M, uint32_t U, uint32_t S,
                        uint32_t* perm, uint32_t* canon_off, uint32_t* pkeys, uint64_t* pair_off,
                        uint2* rinfo, hipStream_t s) {
  hipLaunchKernelGGL(k_count_canon, dim3(grid_of((uint64_t)U + 1)), dim3(BLOCK), 0, s, row_slot,
                     M, U, S, perm, canon_off, pkeys, pair_off, rinfo);
}

}  // namespace kmhg
