// kmhg_count.hip -- count.kmers: per-source k-mer counts held in a GPU counts index.
//
// Replaces count_kmers (reference src/kmer_hash.c:548-591) with seq_to_counts (:220-251) and
// kmer_count_insert (:185-208): every valid window of a sequence adds one to slot `source` of
// its key's vector of `source_n` counts; keys are read out in first-insertion order.
//
// A count.kmers call is one partitioned build of the batch (the distinct keys with their
// occurrence counts in the slots of its table) merged into the counts index, the batch table's
// slots walked in slot order (perm_b = nullptr; empty slots contribute nothing).  Rows are
// appended in that order, each with its insertion-order key (rord, below), and sorted into
// first-insertion order only when a readout asks for rows (round 4: the batch's
// first-occurrence permutation used to come first -- one random 16-B store per key and a
// compaction of an L-entry array -- on every count.kmers call):
//   C_probe   batch item r -> one probe of the counts table; a known key adds its count to its
//             row (distinct keys own distinct rows: a plain read-modify-write), a new key
//             raises its flag
//   (k_scan_u32 of the flags)
//   C_append  new key r -> row U0 + rank: key + a count vector with only `source` set, and its
//             order key
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
#include <hipcub/hipcub.hpp>
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

// A batch slot's first position (1-based): a key seen once holds it inline, a repeated key's
// position list [aux - count, aux) starts with it.
__device__ __forceinline__ uint64_t first_pos(uint4 v, const int32_t* __restrict__ pos) {
  return v.z == 1 ? (uint64_t)v.w : (uint64_t)(uint32_t)pos[v.w - v.z];
}

__global__ void __launch_bounds__(BLOCK)
k_count_append(const uint32_t* __restrict__ perm_b, uint32_t Ub, const Slot* __restrict__ Tb,
               const uint32_t* __restrict__ rank, const uint32_t* __restrict__ n_new,
               uint32_t U0, uint32_t S, uint32_t source, uint64_t* __restrict__ ckeys,
               int32_t* __restrict__ M, const int32_t* __restrict__ bpos,
               uint64_t* __restrict__ rord, uint64_t base) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= Ub) return;
  const uint32_t o = rank[r];
  const uint32_t nx = r + 1 < Ub ? rank[r + 1] : *n_new;
  if (nx == o) return;                                  // known key (or an empty slot)
  const uint4 v = *reinterpret_cast<const uint4*>(&Tb[perm_b ? perm_b[r] : r]);
  const uint64_t row = (uint64_t)U0 + o;
  ckeys[row] = ((uint64_t)v.y << 32) | v.x;
  for (uint32_t j = 0; j < S; ++j) M[row * S + j] = j == source ? (int32_t)v.z : 0;
  if (rord) rord[row] = base + first_pos(v, bpos) - 1;
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
k_count_canon(const uint32_t* __restrict__ rorder, const uint32_t* __restrict__ row_slot,
              const int32_t* __restrict__ M, uint32_t U, uint32_t S, uint32_t* __restrict__ perm,
              uint32_t* __restrict__ canon_off, uint32_t* __restrict__ pkeys,
              uint64_t* __restrict__ pair_off, uint2* __restrict__ rinfo) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r > U) return;
  canon_off[r] = r * S;                  // output rows: S per key in readout order
  if (r == U) return;
  const uint32_t o = rorder ? rorder[r] : r;   // the row (in the count matrix) read out r-th
  perm[r] = row_slot[o];
  rinfo[r] = make_uint2(S, S == 1 ? (uint32_t)M[o] : (o + 1) * S);   // the slot's {count, aux}
  if (S >= 2) {
    pkeys[r] = r;
    pair_off[r] = (uint64_t)r * ((uint64_t)S * (S - 1) / 2);
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
    const uint64_t tot = lane63(inc);
    const uint64_t x = lookback_excl(status, tile, tot);
    if (lane < J * NW) cw[lane] = x + inc - c;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < J; ++j)
    rk[j] = cw[j * NW + wave] + (uint64_t)__popcll(m[j] & lanemask_lt());
}

// Row order of a count.kmers index (first insertion, the order kh_put saw the keys in, which the
// khash readout order replays): a batch's rows are written in slot order, each with its order
// key rord = base + first position - 1 (base = the characters counted before the batch); when a
// readout needs the order (kmhg_engine.cpp ensure_row_order), C_place puts row r at F[rord[r]]
// (F preset to NONE) and C_rows compacts F in order into rorder (rank -> row).  The rows never
// move: the readout arrays (C_canon) and the export (C_gather) go through rorder.
__global__ void __launch_bounds__(BLOCK)
k_rows_place(const uint64_t* __restrict__ rord, uint32_t U, uint32_t* __restrict__ F) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r < U) F[rord[r]] = r;
}

__global__ void __launch_bounds__(BLOCK)
k_rows_order(const uint32_t* __restrict__ F, int64_t n, uint64_t* __restrict__ status,
             uint32_t* __restrict__ ticket, uint32_t* __restrict__ rorder) {
  __shared__ uint64_t cw[WPT * (BLOCK / 64)];
  __shared__ uint32_t tk;
  const uint32_t tile = take_ticket(ticket, &tk);
  const int64_t t0 = (int64_t)tile * TILE;
  uint32_t o[WPT];
  bool fl[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int64_t p = t0 + (int64_t)j * BLOCK + threadIdx.x;
    o[j] = p < n ? F[p] : NONE;
    fl[j] = o[j] != NONE;
  }
  uint64_t rk[WPT];
  tile_compact(fl, rk, cw, status, tile);
#pragma unroll
  for (int j = 0; j < WPT; ++j)
    if (fl[j]) rorder[rk[j]] = o[j];
}

// rows in first-insertion order for an export: row r of the output is row rorder[r]
__global__ void __launch_bounds__(BLOCK)
k_rows_gather(const uint32_t* __restrict__ rorder, const uint64_t* __restrict__ ckeys,
              const int32_t* __restrict__ M, uint32_t U, uint32_t S, uint64_t* __restrict__ okeys,
              int32_t* __restrict__ oM) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r >= U) return;
  const uint64_t o = rorder[r];
  okeys[r] = ckeys[o];
  for (uint32_t q = 0; q < S; ++q) oM[(uint64_t)r * S + q] = M[o * S + q];
}

// The first batch into an empty counts index or suffix hash: the batch table becomes the counts
// table and its rows are written in slot order.  One pass over the adopted table in tiles of
// TILE slots: occupied slots are compacted into rows, each writes its row (key, count vector,
// row_slot, and for count.kmers its order key), slot_row and its own slot fields -- every access
// coalesced but the first-position load of a repeated key.
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
             uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot,
             const int32_t* __restrict__ bpos, uint64_t* __restrict__ rord, uint64_t base) {
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
    if (rord) rord[row] = base + first_pos(v[j], bpos) - 1;
    *reinterpret_cast<uint2*>(&T[i].count) =
        make_uint2(S, S == 1 ? v[j].z : ((uint32_t)row + 1) * S);
  }
}

// Bucket-aligned walk (round 4, the default for a batch from the partitioned build): a tile is
// WALK_B buckets of the adopted table (WALK_B * capb slots; the last tile also holds the side
// slot), and its rows start at the count of the distinct keys of the buckets before it -- the
// bucket kernel's per-bucket statistics, summed per tile (C_wcount) and scanned -- so the tiles
// need no look-back chain.  The slot-tiled walk above chains 36 K tiles at config 3 and was
// bound by that chain's hand-offs (~80 ns per tile, 2.9 ms).  A tile whose occupied slots
// disagree with the statistics raises `err` (the host fails loudly: an internal error).
constexpr uint32_t WALK_B = V2_CAPW <= 1536 ? 2 : 1;
constexpr int WALK_BPER = (int)(WALK_B * V2_CAPW / BLOCK);
static_assert(WALK_B * V2_CAPW % BLOCK == 0 && WALK_BPER * (BLOCK / 64) < 64, "walk tile shape");

__global__ void __launch_bounds__(BLOCK)
k_walk_counts(const BucketStats* __restrict__ bs, const Slot* __restrict__ T, Geom g,
              uint32_t* __restrict__ tc, uint32_t nt, uint32_t* __restrict__ err) {
  const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
  if (t == 0) *err = 0;
  if (t >= nt) return;
  uint32_t c = 0;
  const uint32_t b1 = min(g.nb, (t + 1) * WALK_B);
  for (uint32_t b = t * WALK_B; b < b1; ++b) c += bs[b].n_kmers;
  if (T[side_slot(g)].count) {           // the side key is counted by its bucket, stored last
    const uint32_t sb = bucket_of(mix64(EMPTY_KEY), g.nbh ? g.nbh : g.nb) - g.b0;
    if (sb / WALK_B == t) c -= 1;
    if (t == nt - 1) c += 1;
  }
  tc[t] = c;
}

__global__ void WALK_BOUNDS
k_count_walk_b(Slot* __restrict__ T, Geom g, const uint32_t* __restrict__ tbase, uint32_t S,
               uint32_t source,
               uint64_t* __restrict__ ckeys, int32_t* __restrict__ M,
               uint32_t* __restrict__ slot_row, uint32_t* __restrict__ row_slot,
               const int32_t* __restrict__ bpos, uint64_t* __restrict__ rord, uint64_t base,
               uint32_t* __restrict__ err) {
  __shared__ uint64_t cw[WALK_BPER * (BLOCK / 64) + 1];
  const uint32_t tile = blockIdx.x;
  const uint64_t side = side_slot(g);
  const uint64_t t0 = (uint64_t)tile * WALK_B * V2_CAPW;
  const uint64_t t1 = min(t0 + (uint64_t)WALK_B * V2_CAPW, side);
  const bool last = tile + 1 == gridDim.x;
  uint4 v[WALK_BPER];
  bool fl[WALK_BPER];
#pragma unroll
  for (int j = 0; j < WALK_BPER; ++j) {
    const uint64_t i = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    v[j] = i < t1 ? *reinterpret_cast<const uint4*>(&T[i]) : make_uint4(0u, 0u, 0u, 0u);
    fl[j] = v[j].z != 0;
  }
  const uint64_t r0 = tbase[tile];
  uint64_t rk[WALK_BPER];
  const uint32_t n = tile_rank_at<WALK_BPER>(fl, rk, cw, r0);
  uint4 sv = make_uint4(0u, 0u, 0u, 0u);
  if (last) sv = *reinterpret_cast<const uint4*>(&T[side]);
  const uint32_t ns = last && sv.z ? 1u : 0u;
  if (threadIdx.x == 0 && n + ns != tbase[tile + 1] - (uint32_t)r0) *err = 1;
  auto put = [&](uint64_t i, uint4 x, uint64_t row) {
    ckeys[row] = ((uint64_t)x.y << 32) | x.x;
    int32_t* m = M + row * S;
    if (S == 2)                        // the common two-source matrix: one 8-B store per row
      *reinterpret_cast<int2*>(m) = source ? make_int2(0, (int32_t)x.z) : make_int2((int32_t)x.z, 0);
    else
      for (uint32_t q = 0; q < S; ++q) m[q] = q == source ? (int32_t)x.z : 0;
    row_slot[row] = (uint32_t)i;
    slot_row[i] = (uint32_t)row;
    if (rord) rord[row] = base + first_pos(x, bpos) - 1;
    *reinterpret_cast<uint2*>(&T[i].count) =
        make_uint2(S, S == 1 ? x.z : ((uint32_t)row + 1) * S);
  };
#pragma unroll
  for (int j = 0; j < WALK_BPER; ++j)
    if (fl[j]) put(t0 + (uint64_t)j * BLOCK + threadIdx.x, v[j], rk[j]);
  if (ns && threadIdx.x == 0) put(side, sv, r0 + n);
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
                         uint32_t source, uint64_t* ckeys, int32_t* M, const int32_t* bpos,
                         uint64_t* rord, uint64_t base, hipStream_t s) {
  hipLaunchKernelGGL(k_count_append, dim3(grid_of(Ub)), dim3(BLOCK), 0, s, perm_b, Ub, Tb, rank,
                     n_new, U0, S, source, ckeys, M, bpos, rord, base);
}
void launch_count_insert(const uint64_t* ckeys, uint32_t U, Slot* T, Geom g, uint32_t S,
                         const int32_t* M, uint32_t* slot_row, uint32_t* row_slot,
                         hipStream_t s) {
  hipLaunchKernelGGL(k_count_insert, dim3(grid_of(U)), dim3(BLOCK), 0, s, ckeys, U, T, g, S, M,
                     slot_row, row_slot);
}
void launch_rows_place(const uint64_t* rord, uint32_t U, uint32_t* F, hipStream_t s) {
  hipLaunchKernelGGL(k_rows_place, dim3(grid_of(U)), dim3(BLOCK), 0, s, rord, U, F);
}
void launch_rows_order(const uint32_t* F, int64_t n, uint64_t* status, uint32_t* ticket,
                       uint32_t* rorder, hipStream_t s) {
  const unsigned nt = (unsigned)(((uint64_t)n + TILE - 1) / TILE);
  hipLaunchKernelGGL(k_rows_order, dim3(nt), dim3(BLOCK), 0, s, F, n, status, ticket, rorder);
}
// The O(U) way to the same rorder (advisor round 4: F takes 4 B per character ever counted
// into the pointer): the U (order key, row) pairs sorted by order key with rocPRIM's radix sort
// (hipcub), over the key's `bits` low bits.  Rows are distinct and their order keys too, so the
// result is the permutation k_rows_order compacts out of F.
static __global__ void __launch_bounds__(BLOCK) k_iota_u32(uint32_t* __restrict__ a, uint32_t n) {
  const uint32_t r = blockIdx.x * BLOCK + threadIdx.x;
  if (r < n) a[r] = r;
}
hipError_t rows_sort_temp_bytes(uint32_t U, int bits, size_t* bytes) {
  *bytes = 0;
  return hipcub::DeviceRadixSort::SortPairs(nullptr, *bytes, (const uint64_t*)nullptr,
                                            (uint64_t*)nullptr, (const uint32_t*)nullptr,
                                            (uint32_t*)nullptr, (int)U, 0, bits);
}
hipError_t launch_rows_sort(const uint64_t* rord, uint32_t U, int bits, uint64_t* keys_out,
                            uint32_t* rows_in, uint32_t* rorder, void* temp, size_t temp_bytes,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_iota_u32, dim3(grid_of(U)), dim3(BLOCK), 0, s, rows_in, U);
  if (hipError_t e = hipGetLastError(); e != hipSuccess) return e;
  return hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, rord, keys_out, rows_in, rorder,
                                            (int)U, 0, bits, s);
}
void launch_rows_gather(const uint32_t* rorder, const uint64_t* ckeys, const int32_t* M,
                        uint32_t U, uint32_t S, uint64_t* okeys, int32_t* oM, hipStream_t s) {
  hipLaunchKernelGGL(k_rows_gather, dim3(grid_of(U)), dim3(BLOCK), 0, s, rorder, ckeys, M, U, S,
                     okeys, oM);
}
uint64_t count_walk_tiles(uint64_t nslots) { return (nslots + WALK_TILE - 1) / WALK_TILE; }
void launch_count_walk(Slot* T, uint64_t nslots, uint64_t* status, uint32_t* ticket, uint32_t S,
                       uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                       uint32_t* row_slot, const int32_t* bpos, uint64_t* rord, uint64_t base,
                       hipStream_t s) {
  const unsigned nt = (unsigned)((nslots + WALK_TILE - 1) / WALK_TILE);
  hipLaunchKernelGGL(k_count_walk, dim3(nt), dim3(BLOCK), 0, s, T, nslots, status, ticket, S,
                     source, ckeys, M, slot_row, row_slot, bpos, rord, base);
}
uint32_t count_walk_b_tiles(uint32_t nb) { return (nb + WALK_B - 1) / WALK_B; }
void launch_walk_counts(const BucketStats* bs, const Slot* T, Geom g, uint32_t* tc, uint32_t nt,
                        uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_walk_counts, dim3(grid_of(nt)), dim3(BLOCK), 0, s, bs, T, g, tc, nt, err);
}
void launch_count_walk_b(Slot* T, Geom g, const uint32_t* tbase, uint32_t nt, uint32_t S,
                         uint32_t source, uint64_t* ckeys, int32_t* M, uint32_t* slot_row,
                         uint32_t* row_slot, const int32_t* bpos, uint64_t* rord, uint64_t base,
                         uint32_t* err, hipStream_t s) {
  hipLaunchKernelGGL(k_count_walk_b, dim3(nt), dim3(BLOCK), 0, s, T, g, tbase, S, source, ckeys, M,
                     slot_row, row_slot, bpos, rord, base, err);
}
void launch_count_fix(Slot* T, uint64_t nslots, uint32_t S, const int32_t* M, uint32_t* slot_row,
                      uint32_t* row_slot, hipStream_t s) {
  hipLaunchKernelGGL(k_count_fix, dim3(grid_cap(nslots)), dim3(BLOCK), 0, s, T, nslots, S, M,
                     slot_row, row_slot);
}
void launch_count_canon(const uint32_t* rorder, const uint32_t* row_slot, const int32_t* M,
                        uint32_t U, uint32_t S, uint32_t* perm, uint32_t* canon_off,
                        uint32_t* pkeys, uint64_t* pair_off, uint2* rinfo, hipStream_t s) {
  hipLaunchKernelGGL(k_count_canon, dim3(grid_of((uint64_t)U + 1)), dim3(BLOCK), 0, s, rorder,
                     row_slot, M, U, S, perm, canon_off, pkeys, pair_off, rinfo);
}

}  // namespace kmhg
