// kmhg_kernels.hip -- CDNA4 (gfx950) kernels of the k-mer position index.
//
// Reference hot loops replaced (lmjakt/kmer_hasheR):
//   K_insert   seq_to_hash window walk + kmer_h_insert  (src/kmer_pos.c:36-50, 66-98;
//              init_kmer src/kmer_util.c:18-32; UPDATE_OFFSET/LC src/kmer_util.h:8,10)
//   K_compact  kvec sizing -> CSR offsets                (kvec growth, src/kvec.h:74-80)
//   K_scatter  kv_push(pos)                               (src/kmer_pos.c:47)
//   K_sort     sort_kmer_pos / ascending order            (src/kmer_pos.c:21-33)
//   Q_probe,
//   Q_emit     seq_kmer_positions + pair_positions_push   (src/kmer_pos.c:101-136)
//   R_*        kmer_positions bucket walk                 (src/kmer_hash.c:1054-1147)
//              and kmer_seq decode                        (src/kmer_hash.c:123-133)
//
// Integer/byte work only: every kernel is bounded by HBM (or by random-access latency on the
// table), none by arithmetic; nothing here is matmul-shaped.
#include <hip/hip_runtime.h>
#include "kmhg_common.h"
#include "kmhg_kernels.h"
#include "kmhg_device.h"

namespace kmhg {

// ================================================================== build kernels
__global__ void __launch_bounds__(BLOCK) k_table_init(Slot* __restrict__ T, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (; i < n; i += stride) {
    uint4 v = make_uint4(0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0u);
    *reinterpret_cast<uint4*>(&T[i]) = v;
  }
}

// Part export (owner-computes multi-GPU build): a part's slots with their list ends moved by the
// part's first position index in the whole index (count >= 2: aux += base; a key seen once keeps
// its position inline, an empty slot is copied as is).
__global__ void __launch_bounds__(BLOCK) k_part_rebase(const Slot* __restrict__ src,
                                                        Slot* __restrict__ dst, uint64_t n,
                                                        uint32_t base) {
  uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const uint64_t stride = (uint64_t)gridDim.x * BLOCK;
  for (; i < n; i += stride) {
    uint4 v = *reinterpret_cast<const uint4*>(&src[i]);
    if (v.z > 1u) v.w += base;
    *reinterpret_cast<uint4*>(&dst[i]) = v;
  }
}

// K_insert: encode + N-mask + find-or-insert + count.  One lane per window, TILE windows per
// workgroup, lane-consecutive windows so the win_slot stores are coalesced.
__global__ void __launch_bounds__(BLOCK)
k_build_insert(const uint8_t* __restrict__ seq, int64_t L, int k, Slot* __restrict__ T,
               Geom g, uint32_t* __restrict__ win_slot, int64_t Nw, int aligned) {
  __shared__ Stage st;
  const int64_t tile0 = (int64_t)blockIdx.x * TILE;
  stage_tile(seq, L, tile0 - HALO, st, aligned != 0);   // tile0 % 16 == 0: window o = HALO + w
  __syncthreads();
  uint32_t* cnt0 = &T[0].count;
  const size_t stride = sizeof(Slot) / sizeof(uint32_t);
#pragma unroll 2
  for (int j = 0; j < WPT; ++j) {
    const int w = j * BLOCK + threadIdx.x;
    const int64_t s = tile0 + w;
    uint64_t key = 0;
    bool valid = (s < Nw) && window_key(st, HALO + w, s, L, k, key);
    uint32_t slot = NONE;
    if (valid) slot = table_insert(T, g, key);
    wave_agg_add(cnt0, valid, slot, stride);
    if (s < Nw) win_slot[s] = slot;
  }
}

// K_compact: one pass over the table (ticketed tiles, look-back scan of {occupied, count}).
// Occupied slot -> dense id (slot order), CSR offset; slot.end := offset (K_scatter advances it).
// Also collects ids of keys with count >= 2 into the small/large sort lists, sum C(n,2), max n.
__global__ void __launch_bounds__(BLOCK)
k_build_compact(Slot* __restrict__ T, uint64_t nslots, uint64_t* __restrict__ status,
                uint32_t* __restrict__ ticket, uint64_t* __restrict__ ukeys,
                uint32_t* __restrict__ counts, uint32_t* __restrict__ offsets,
                uint32_t* __restrict__ small_ids, uint32_t* __restrict__ large_ids,
                BuildMeta* __restrict__ meta, uint32_t ntiles, uint32_t large_min) {
  __shared__ uint64_t sh[8];
  __shared__ uint32_t tk;
  __shared__ uint32_t sh_smallbase, sh_largebase;
  const uint32_t tile = take_ticket(ticket, &tk);
  const uint64_t t0 = (uint64_t)tile * TILE;
  uint64_t keyv[WPT];
  uint32_t cnt[WPT];
  uint64_t lane_excl[WPT];
  // pass 1: load (coalesced 16-B slots), per-j block scans
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    uint64_t i = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    cnt[j] = 0; keyv[j] = EMPTY_KEY;
    if (i < nslots) {
      uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
      keyv[j] = ((uint64_t)v.y << 32) | v.x;
      cnt[j] = v.z;
    }
  }
  // packed value: occupied in the high 32 bits, count in the low 32 (no carry inside a tile)
  uint64_t row_tot[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    uint64_t v = cnt[j] ? ((1ull << 32) | cnt[j]) : 0ull;
    lane_excl[j] = block_excl_scan(v, sh, row_tot[j]);
  }
  uint64_t tile_tot = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    uint64_t base = tile_tot;
    tile_tot += row_tot[j];
    lane_excl[j] += base;
  }
  // global prefix: payload = occupied << 31 | count (each < 2^31 overall)
  if (threadIdx.x < 64) {
    uint64_t agg = ((tile_tot >> 32) << 31) | (tile_tot & 0xFFFFFFFFull);
    uint64_t ex = lookback_excl(status, tile, agg);
    if (threadIdx.x == 0) sh[6] = ex;
    if (threadIdx.x == 0 && tile == ntiles - 1) {
      uint64_t inc = ex + agg;
      meta->n_kmers = inc >> 31;
      meta->n_positions = inc & ((1ull << 31) - 1);
      offsets[meta->n_kmers] = (uint32_t)meta->n_positions;
    }
  }
  __syncthreads();
  const uint64_t gex = sh[6];
  const uint64_t g_occ = gex >> 31, g_cnt = gex & ((1ull << 31) - 1);
  uint64_t pairs = 0;
  uint32_t mx = 0, nsmall = 0, nlarge = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (!cnt[j]) continue;
    uint64_t i = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    uint32_t id = (uint32_t)(g_occ + (lane_excl[j] >> 32));
    uint32_t off = (uint32_t)(g_cnt + (lane_excl[j] & 0xFFFFFFFFull));
    ukeys[id] = keyv[j];
    counts[id] = cnt[j];
    offsets[id] = off;
    T[i].aux = off;
    uint64_t n = cnt[j];
    pairs += n * (n - 1) / 2;
    mx = max(mx, cnt[j]);
    if (cnt[j] >= 2) { if (cnt[j] >= large_min) ++nlarge; else ++nsmall; }
  }
  // list appends: per-thread count -> block scan -> one atomic per block per list
  uint64_t tot_s, tot_l;
  uint64_t ex_s = block_excl_scan(nsmall, sh, tot_s);
  uint64_t ex_l = block_excl_scan(nlarge, sh, tot_l);
  if (threadIdx.x == 0) {
    sh_smallbase = tot_s ? atomicAdd(&meta->n_small, (uint32_t)tot_s) : 0;
    sh_largebase = tot_l ? atomicAdd(&meta->n_large, (uint32_t)tot_l) : 0;
  }
  __syncthreads();
  uint32_t ps = sh_smallbase + (uint32_t)ex_s, pl = sh_largebase + (uint32_t)ex_l;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (cnt[j] < 2) continue;
    uint32_t id = (uint32_t)(g_occ + (lane_excl[j] >> 32));
    if (cnt[j] >= large_min) large_ids[pl++] = id; else small_ids[ps++] = id;
  }
  // tile reductions for P and max n
  for (int d = 32; d >= 1; d >>= 1) {
    pairs += __shfl_xor(pairs, d);
    mx = max(mx, (uint32_t)__shfl_xor(mx, d));
  }
  if (lane_id() == 0) {
    if (pairs) atomicAdd((unsigned long long*)&meta->n_pairs, (unsigned long long)pairs);
    if (mx) atomicMax(&meta->max_count, mx);
  }
}

// K_scatter: positions[slot.aux++] = s + 1 for every valid window (wave-aggregated, lane-order
// ranks inside a group).  Order across waves is arbitrary; K_sort restores ascending order.
__global__ void __launch_bounds__(BLOCK)
k_build_scatter(const uint32_t* __restrict__ win_slot, int64_t Nw, Slot* __restrict__ T,
                int32_t* __restrict__ positions) {
  uint32_t* end0 = &T[0].aux;
  const size_t stride = sizeof(Slot) / sizeof(uint32_t);
  const int64_t tile0 = (int64_t)blockIdx.x * TILE;
#pragma unroll 2
  for (int j = 0; j < WPT; ++j) {
    const int64_t s = tile0 + j * BLOCK + threadIdx.x;
    uint32_t slot = (s < Nw) ? win_slot[s] : NONE;
    bool act = slot != NONE;
    uint32_t r = wave_agg_add(end0, act, slot, stride);
    if (act) positions[r] = (int32_t)(s + 1);
  }
}

// K_sort (small): one lane per key with 2 <= n < large_min; insertion sort in place.
__global__ void __launch_bounds__(BLOCK)
k_sort_small(const uint32_t* __restrict__ ids, const BuildMeta* __restrict__ meta,
             const uint32_t* __restrict__ counts, const uint32_t* __restrict__ offsets,
             int32_t* __restrict__ positions) {
  const uint32_t n_ids = meta->n_small;
  for (uint32_t t = blockIdx.x * BLOCK + threadIdx.x; t < n_ids; t += gridDim.x * BLOCK) {
    uint32_t id = ids[t];
    int32_t* a = positions + offsets[id];
    uint32_t n = counts[id];
    for (uint32_t i = 1; i < n; ++i) {
      int32_t x = a[i];
      int32_t j = (int32_t)i - 1;
      while (j >= 0 && a[j] > x) { a[j + 1] = a[j]; --j; }
      a[j + 1] = x;
    }
  }
}

// Block bitonic sort of a segment of up to SORT_CHUNK ints held in LDS (padded with INT_MAX).
__device__ void lds_bitonic(int32_t* s, uint32_t pow2) {
  for (uint32_t size = 2; size <= pow2; size <<= 1) {
    for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
      for (uint32_t t = threadIdx.x; t < pow2 / 2; t += BLOCK) {
        uint32_t lo = 2 * t - (t & (stride - 1));
        uint32_t hi = lo + stride;
        bool up = ((lo & size) == 0);
        int32_t a = s[lo], b = s[hi];
        if ((a > b) == up) { s[lo] = b; s[hi] = a; }
      }
      __syncthreads();
    }
  }
}

// K_sort (large): one workgroup per key with n >= large_min.  Chunks of SORT_CHUNK are sorted
// in LDS; longer segments are then merged pairwise (each element finds its rank in the partner
// run by binary search -- positions are unique) ping-ponging with `tmp`.
__global__ void __launch_bounds__(BLOCK)
k_sort_large(const uint32_t* __restrict__ ids, const BuildMeta* __restrict__ meta,
             const uint32_t* __restrict__ counts, const uint32_t* __restrict__ offsets,
             int32_t* __restrict__ positions, int32_t* __restrict__ tmp) {
  __shared__ int32_t s[SORT_CHUNK];
  const uint32_t n_ids = meta->n_large;
  for (uint32_t t = blockIdx.x; t < n_ids; t += gridDim.x) {
    const uint32_t id = ids[t];
    const uint32_t n = counts[id];
    int32_t* a = positions + offsets[id];
    int32_t* b = tmp + offsets[id];
    for (uint32_t c0 = 0; c0 < n; c0 += SORT_CHUNK) {
      uint32_t m = min((uint32_t)SORT_CHUNK, n - c0);
      uint32_t p2 = 1;
      while (p2 < m) p2 <<= 1;
      for (uint32_t i = threadIdx.x; i < p2; i += BLOCK) s[i] = (i < m) ? a[c0 + i] : INT32_MAX;
      __syncthreads();
      lds_bitonic(s, p2);
      for (uint32_t i = threadIdx.x; i < m; i += BLOCK) a[c0 + i] = s[i];
      __syncthreads();
    }
    int32_t* src = a;
    int32_t* dst = b;
    for (uint32_t w = SORT_CHUNK; w < n; w <<= 1) {
      for (uint32_t i = threadIdx.x; i < n; i += BLOCK) {
        uint32_t run = i / (2 * w), r0 = run * 2 * w;
        uint32_t a0 = r0, a1 = min(r0 + w, n), b1 = min(r0 + 2 * w, n);
        int32_t x = src[i];
        uint32_t lo, hi, out;
        if (i < a1) {           // element of run A: rank in B = #B < x
          lo = a1; hi = b1;
          while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (src[mid] < x) lo = mid + 1; else hi = mid; }
          out = r0 + (i - a0) + (lo - a1);
        } else {                // element of run B: rank in A = #A < x
          lo = a0; hi = a1;
          while (lo < hi) { uint32_t mid = (lo + hi) >> 1; if (src[mid] < x) lo = mid + 1; else hi = mid; }
          out = r0 + (i - a1) + (lo - a0);
        }
        dst[out] = x;
      }
      __syncthreads();
      int32_t* tp = src; src = dst; dst = tp;
    }
    if (src != a)
      for (uint32_t i = threadIdx.x; i < n; i += BLOCK) a[i] = src[i];
    __syncthreads();
  }
}

// K_inline: a key seen once keeps its position inline in the slot (Slot::aux), as the
// partitioned build writes it.
__global__ void __launch_bounds__(BLOCK)
k_inline_singles(Slot* __restrict__ T, uint64_t nslots, const int32_t* __restrict__ positions) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * BLOCK)
    if (T[i].count == 1) T[i].aux = (uint32_t)positions[T[i].aux - 1];
}

// ================================================================== query kernels
// V_diag_valid (once per index, before its first diagonal query): uniq word a = the indexed
// windows among [32a, 32a + 32), from the N flags the build kept -- no N in [s, s + k), s < Nw,
// and the end-drop rule of the last window (src/kmer_pos.c:81-83).  One
// thread per word: u16 flag words 2a .. 2a + 3 hold chars [32a, 32a + 64), char 32a at bit 63.
__global__ void __launch_bounds__(BLOCK)
k_diag_valid(const uint16_t* __restrict__ nbit, int64_t L, int k, uint32_t* __restrict__ uniq,
             uint64_t n_words, int multi_in) {
  const uint64_t a = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (a >= n_words) return;
  const int64_t Nw = L - k + 1;
  const uint64_t x = ((uint64_t)nbit[2 * a] << 48) | ((uint64_t)nbit[2 * a + 1] << 32) |
                     ((uint64_t)nbit[2 * a + 2] << 16) | (uint64_t)nbit[2 * a + 3];
  uint32_t u = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) {
    const int64_t s = (int64_t)(32 * a) + i;
    bool v = s < Nw && ((x << i) >> (64 - k)) == 0;
    if (v && s == Nw - 1 && s + k == L) {      // the end-drop rule
      const int64_t p = s - 1;
      v = p >= 0 && !((nbit[p >> 4] >> (15 - (p & 15))) & 1u);
    }
    u |= (v ? 1u : 0u) << i;
  }
  if (multi_in) u &= ~uniq[a];                 // the build's repeated-key bits
  uniq[a] = u;
}

// V_diag_prep (after V_diag_valid): the slot tags TG, one byte per table slot, and the `uniq`
// bits (DiagIdx) of every position of a key seen more than once cleared.  One thread per slot;
// a key with more than DP_LANE positions is cleared by the whole wave.  Keys seen once (all but
// a few of an i.i.d. sequence's) cost one 16-B slot read and one tag byte.
constexpr uint32_t DP_LANE = 16;
__device__ __forceinline__ void uniq_clear(uint32_t* uniq, int32_t pos) {
  const uint32_t j = (uint32_t)(pos - 1);
  atomicAnd(&uniq[j >> 5], ~(1u << (j & 31)));
}
__global__ void __launch_bounds__(BLOCK)
k_diag_prep(const Slot* __restrict__ T, uint64_t nslots, const int32_t* __restrict__ positions,
            uint32_t* __restrict__ uniq, uint8_t* __restrict__ TG) {
  const int lane = lane_id();
  for (uint64_t i0 = (uint64_t)blockIdx.x * BLOCK; i0 < nslots; i0 += (uint64_t)gridDim.x * BLOCK) {
    const uint64_t i = i0 + threadIdx.x;
    uint64_t key = EMPTY_KEY;
    uint32_t count = 0, aux = 0;
    if (i < nslots) {
      const uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
      key = ((uint64_t)v.y << 32) | v.x; count = v.z; aux = v.w;
    }
    if (i < nslots) TG[i] = key == EMPTY_KEY ? (uint8_t)0 : slot_tag(mix64(key));
    if (count > 1 && count <= DP_LANE)
      for (uint32_t q = aux - count; q < aux; ++q) uniq_clear(uniq, positions[q]);
    uint64_t heavy = __ballot(count > DP_LANE);
    while (heavy) {                            // long lists: the wave strides over them
      const int src = __ffsll((unsigned long long)heavy) - 1;
      heavy &= heavy - 1;
      const uint32_t c = __shfl(count, src), a = __shfl(aux, src);
      for (uint32_t q = a - c + lane; q < a; q += 64) uniq_clear(uniq, positions[q]);
    }
  }
}

void launch_diag_valid(const uint16_t* nbit, int64_t L, int k, uint32_t* uniq, bool multi_in,
                       hipStream_t s) {
  const uint64_t nw = diag_uniq_words(L - k + 1);
  hipLaunchKernelGGL(k_diag_valid, dim3((unsigned)((nw + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                     nbit, L, k, uniq, nw, multi_in ? 1 : 0);
}

void launch_diag_prep(const uint16_t* nbit, int64_t L, int k, uint32_t* uniq, const Slot* T,
                      uint64_t nslots, const int32_t* positions, uint8_t* TG, hipStream_t s) {
  const uint64_t nw = diag_uniq_words(L - k + 1);
  hipLaunchKernelGGL(k_diag_valid, dim3((unsigned)((nw + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                     nbit, L, k, uniq, nw, 0);
  uint64_t g = (nslots + BLOCK - 1) / BLOCK;
  if (g > 65536) g = 65536;
  hipLaunchKernelGGL(k_diag_prep, dim3((unsigned)(g ? g : 1)), dim3(BLOCK), 0, s, T, nslots,
                     positions, uniq, TG);
}

// A window's probe result as Q_emit reads it: qrec[s] = 0 (no hit), the 1-based index position
// (one hit: a key seen once keeps its position inline, < 2^31), or QREC_MULTI with qmulti[s] =
// {count, first index into positions} -- 4 B per window written and read back instead of 8 (only
// windows with several hits, rare outside repeats, touch qmulti).
constexpr uint32_t QREC_MULTI = 0x80000000u;
__device__ __forceinline__ void put_qrec(uint32_t* qrec, uint2* qmulti, int64_t i, uint32_t count,
                                         uint32_t aux) {
  qrec[i] = count == 0 ? 0u : (count == 1 ? aux : QREC_MULTI);
  if (count > 1) qmulti[i] = make_uint2(count, aux - count);
}

// Q_probe: per query window (query k) probe the table; qrec / qmulti (put_qrec); per-tile row
// totals go through the look-back so each tile learns its first output row.
// Diagonal path (X.code != nullptr: query k = index k, a position index): dot plots hit along
// diagonals, so a window whose predecessor matched index position j usually matches j + 1.  Every
// DG_STRIDE-th window of the tile ("anchor") probes the table; an anchor with a unique hit at j
// predicts j + d for the window d after it, and the later windows of the tile follow the last
// anchor that predicted.  A prediction p is VERIFIED against the index sequence itself (DiagIdx):
// if index window p - 1 is indexed with a key seen once (its `uniq` bit) and that key -- read from
// the index's 2-bit code words -- equals the window's key, the window's slot is {count 1, aux p}
// (exact: the only slot of that key holds exactly that); otherwise the window probes the table
// as before.  Consecutive windows read the same few code and bit words, so a wave's verification
// loads touch one or two cache lines: ~0.4 B per window, where the position-indexed slot copy
// this replaced streamed 16 B per window (and took 16 B per index window of HBM, built by a
// random scatter on the first query).  Queries unrelated to the index pay the anchors and one
// failed check.
// Anchor stride.  Round 2 (config 2 self dot plot, probe): 16 / 32 / 64 / 128 -> 97 / 86 / 82 /
// 76 us, 64 kept for short misses after a tile start.  Round 4, A/B in one run against variant
// builds (`profiles/rd4w_ab_dg_stride_*`): 128 beats 64 at every size -- config 2 probe 42-44 ->
// 37-39 us (query 117-120 -> 123-125 Gbp/s, unrelated 46.5 -> 47.6), config 3 0.346-0.350 ->
// 0.319-0.320 ms (167 -> 175 Gbp/s), config 5 4.75-4.77 -> 4.55-4.56 ms (72.1 -> 74.1 Gbp/s);
// 32 loses (config 2 111 Gbp/s).  256 against 128 (`profiles/rd4x_ab_dg_stride_*`): config 3
// probe 0.319-0.321 -> 0.297-0.298 ms (174 -> 181 Gbp/s), config 5 4.55-4.56 -> 4.52-4.53 ms,
// config 2 probe 38.8-40.0 -> 37.2-39.9 us; 64 again slower.  512 / 1024 against 256
// (`profiles/rd4ae_ab_dg_stride_*`): config 3 181 -> 186 Gbp/s, but config 5 (the cross query:
// an anchor on an SNV leaves the windows up to the next one to probe) 90.9 -> 86.0 / 73.8.
// Anchors only establish a
// diagonal: a window after an SNV is verified again against the same anchor's prediction, and
// only a shifted diagonal (an indel, a rearrangement) probes until the next anchor.
#ifndef KMHG_DG_STRIDE
#define KMHG_DG_STRIDE 256
#endif
constexpr int DG_STRIDE = KMHG_DG_STRIDE;
constexpr int DG_ANCHORS = TILE / DG_STRIDE;
constexpr int DG_SCAN = (DG_ANCHORS + 63) / 64 * 64;   // whole waves run the anchor scan
static_assert(DG_SCAN <= BLOCK && DG_SCAN <= 128, "anchors: one thread each, at most two waves");

static_assert(DG_ANCHORS <= 64, "the probed-anchor mask is one wave's ballot");
struct DiagAnchors {
  uint32_t anc[DG_ANCHORS];      // anchor's unique hit (1-based index position), 0 none
  int32_t last[DG_ANCHORS];      // last anchor <= a that predicts, -1 none
  uint2 info[DG_ANCHORS];        // anchor's {count, aux} (probed anchors)
  uint64_t probed;               // bit a: anchor a's window was probed
  __device__ __forceinline__ bool was_probed(int a) const { return (probed >> a) & 1ull; }
};

// Anchor probes of a staged tile (threads < DG_ANCHORS) and the last-predicting-anchor scan;
// called by every thread of the block (two barriers inside).  PART: only the anchors whose key
// the part owns probe (the others record no hit and predict nothing).
template <bool NT, bool PART = false, class ST>
__device__ __forceinline__ void diag_anchors(const ST& st, int o0, int64_t t_start, int64_t w1,
                                             int64_t L, int kq, const Slot* __restrict__ T,
                                             Geom g, DiagAnchors& A) {
  if (threadIdx.x < DG_SCAN) {
    const bool is_anchor = threadIdx.x < DG_ANCHORS;
    const int w = threadIdx.x * DG_STRIDE;
    const int64_t s = t_start + w;
    uint64_t key = 0;
    uint32_t count = 0, aux = 0;
    const bool kv = is_anchor && s < w1 && window_key(st, o0 + w, s, L, kq, key) &&
                    (!PART || part_owns(key, g));
    // Adaptive anchors: the even ones are always probed; an odd one only while no even anchor
    // before it predicts (the tile's head after a miss), since behind a predicting anchor the
    // windows verify against its diagonal anyway.  A self dot plot probes every 512th window, a
    // cross query keeps every 256th where the tile head needs it.
    const bool primary = (threadIdx.x & 1) == 0;
    if (kv && primary) table_find<NT, PART>(T, g, key, count, aux);
    const uint64_t pm = __ballot(is_anchor && primary && count == 1);
    // (and only in a tile where some even anchor predicts: with none, the tile is unrelated to
    // the index and its windows probe the table whatever the odd anchors find)
    const bool second = kv && !primary && pm != 0 && (pm & lanemask_lt()) == 0;
    if (second) table_find<NT, PART>(T, g, key, count, aux);
    const uint64_t probed = __ballot(is_anchor && (primary || second));
    if (threadIdx.x == 0) A.probed = probed;
    if (is_anchor) {
      A.anc[threadIdx.x] = count == 1 ? aux : 0u;
      A.info[threadIdx.x] = make_uint2(count, aux);
    }
    int32_t v = count == 1 ? (int32_t)threadIdx.x : -1;   // max-scan over the anchor indices
    // by DPP (identity -1 for lanes without a source): VALU moves, not LDS permutes
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x111, 0xf, 0xf, false));   // row_shr:1
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x112, 0xf, 0xf, false));   // row_shr:2
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x114, 0xf, 0xf, false));   // row_shr:4
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x118, 0xf, 0xf, false));   // row_shr:8
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x142, 0xa, 0xf, false));   // row_bcast:15
    v = max(v, __builtin_amdgcn_update_dpp(-1, v, 0x143, 0xc, 0xf, false));   // row_bcast:31
    if (is_anchor) A.last[threadIdx.x] = v;
  }
  __syncthreads();
  if (threadIdx.x >= 64 && threadIdx.x < DG_ANCHORS) {   // carry across the (two) anchor waves
    const int32_t carry = A.last[(threadIdx.x & ~63) - 1];
    if (A.last[threadIdx.x] < 0) A.last[threadIdx.x] = carry;
  }
  __syncthreads();
}

// The diagonal path of a staged tile, every lane's WPT windows: the verification words of every
// prediction are loaded first, all in flight at once (a window without a prediction loads word
// 0, so every lane issues a static number of loads), then resolved; windows whose prediction
// fails probe through the slot tags (TG) or the table.
// `out(w, s, count, aux)` receives every window of the tile, s = t_start + w (s >= w1: none).
template <bool NT, class ST, class Out>
__device__ __forceinline__ void diag_resolve(const ST& st, int o0, int64_t t_start, int64_t w0,
                                             int64_t w1, int64_t L, int kq,
                                             const Slot* __restrict__ T, Geom g, DiagIdx X,
                                             const uint8_t* __restrict__ TG,
                                             const DiagAnchors& A, Out out) {
  (void)w0;
  uint32_t ca[WPT], cb[WPT], cc[WPT], ub[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int w = j * BLOCK + threadIdx.x;
    const int la = A.last[w / DG_STRIDE];
    int64_t pj = la >= 0 ? (int64_t)A.anc[la] + (w - la * DG_STRIDE) : 1;
    if (pj > X.nA || (w % DG_STRIDE == 0 && A.was_probed(w / DG_STRIDE))) pj = 1;
    const uint64_t q0 = (uint64_t)(pj - 1) >> 4;
    ca[j] = X.code[q0];
    cb[j] = X.code[q0 + 1];
    cc[j] = X.code[q0 + 2];
    ub[j] = X.uniq[(uint64_t)(pj - 1) >> 5];
  }
#pragma unroll                 // static indices into the loaded words
  for (int j = 0; j < WPT; ++j) {
    const int w = j * BLOCK + threadIdx.x;
    const int64_t s = t_start + w;
    uint64_t key = 0;
    uint32_t count = 0, aux = 0;
    if (s < w1 && window_key(st, o0 + w, s, L, kq, key)) {
      bool hit;
      if (w % DG_STRIDE == 0 && A.was_probed(w / DG_STRIDE)) {
        const uint2 ai = A.info[w / DG_STRIDE];
        count = ai.x; aux = ai.y;
        hit = true;
      } else {
        const int la = A.last[w / DG_STRIDE];
        const int64_t pj = la >= 0 ? (int64_t)A.anc[la] + (w - la * DG_STRIDE) : 0;
        hit = la >= 0 && pj <= X.nA && ((ub[j] >> ((pj - 1) & 31)) & 1u) &&
              code_key(ca[j], cb[j], cc[j], pj - 1, kq) == key;
        count = 1; aux = (uint32_t)pj;
      }
      if (!hit) {
        count = 0; aux = 0;
        if (TG) table_find_tag<NT>(T, TG, g, key, count, aux);   // mostly misses here
        else
#ifndef KMHG_NO_FIND4
          table_find4<NT>(T, g, key, count, aux);
#else
          table_find<NT>(T, g, key, count, aux);
#endif
      }
    }
    out(w, s, count, aux);
  }
}

// The same in two phases.  Phase 1, per lane over 8 CONSECUTIVE windows w0 .. w0 + 7 of the tile
// (w0 = 8 t): they share one anchor (64 | 8), so their predictions are consecutive index windows
// p0 .. p0 + 7 and their verification needs 4 code words and 2 uniq words for the lot, read once
// (6 loads, not 32); their own keys come from Win8 (8 LDS reads, not 48); their records leave as
// two 16-B stores.  Phase 2 probes the windows phase 1 did not resolve, with the strided window
// -> lane map (window j * BLOCK + t): a miss run (the k windows over an SNV) would otherwise be
// one lane's serial chain of random reads (config 5: probe 5.1 -> 6.4 ms with phase 1's map).
// Writes qrec / qmulti itself; returns the lane's row count.
struct DiagProbeLDS {
  uint64_t key[TILE];            // unresolved windows' keys
  uint8_t todo[TILE];            // 1: window w needs a table probe
};
// PART (owner-routed query over a part): only the windows whose key the part owns can hit (the
// code words and window bits are the whole index sequence's, the repeated-key bits the part's
// own keys'); a verified window of another part's key records no hit and is not probed.
template <bool NT, bool PART, class ST>
__device__ __forceinline__ uint64_t diag_resolve8(const ST& st, int o0, int64_t t_start,
                                                  int64_t w0r, int64_t w1, int64_t L, int kq,
                                                  const Slot* __restrict__ T, Geom g, DiagIdx X,
                                                  const uint8_t* __restrict__ TG,
                                                  const DiagAnchors& A, uint32_t* __restrict__ qrec,
                                                  uint2* __restrict__ qmulti, DiagProbeLDS& P) {
  static_assert(DG_STRIDE % 8 == 0 && WPT == 8, "a lane's 8 windows share one anchor");
  const int w0 = 8 * (int)threadIdx.x;
  const int64_t s0 = t_start + w0;
  const Win8 win(st, o0 + w0, s0, L, kq);
  const int la = A.last[w0 / DG_STRIDE];
  const int64_t pbase = la >= 0 ? (int64_t)A.anc[la] + (w0 - la * DG_STRIDE) : 0;
  const bool pred = la >= 0 && pbase <= X.nA;             // anc > 0, so pbase >= 1
  const uint64_t p0 = pred ? (uint64_t)(pbase - 1) : 0ull;  // 0-based index window of j = 0
  const uint64_t cq = p0 >> 4, uq = p0 >> 5;
  const uint64_t ulast = X.nA > 0 ? (uint64_t)(X.nA - 1) >> 5 : 0ull;
  const uint64_t ih = ((uint64_t)X.code[cq] << 32) | X.code[cq + 1];
  const uint64_t il = ((uint64_t)X.code[cq + 2] << 32) | X.code[cq + 3];
  const uint64_t ub = ((uint64_t)X.uniq[min(uq + 1, ulast)] << 32) | X.uniq[uq];
  const int ro = (int)(p0 & 15), rb = (int)(p0 & 31);
  uint32_t rec[8];
  uint64_t rows = 0;
  uint32_t todo = 0;                                       // byte j: window j left to phase 2
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int64_t s = s0 + j;
    uint32_t count = 0, aux = 0;
    if (s < w1 && win.valid(j)) {
      const uint64_t key = win.key(j);
      const bool own = !PART || part_owns(key, g);
      bool hit;
      if (j == 0 && w0 % DG_STRIDE == 0 && A.was_probed(w0 / DG_STRIDE)) {   // probed already
        const uint2 ai = A.info[w0 / DG_STRIDE];
        count = ai.x; aux = ai.y;
        hit = true;
      } else {
        const int sh = 2 * (ro + j);                       // <= 44
        const uint64_t top = sh ? (ih << sh) | (il >> (64 - sh)) : ih;
        const uint64_t ikey = top >> (64 - 2 * kq);
        hit = own && pred && (int64_t)(p0 + j) < X.nA && ((ub >> (rb + j)) & 1ull) && ikey == key;
        count = 1; aux = (uint32_t)(p0 + 1 + j);
      }
      if (!hit) {
        count = 0; aux = 0;
        if (own) {
          P.key[w0 + j] = key;
          todo |= 1u << (8 * (j & 3));
        }
      }
    }
    if (j == 3) {
      *reinterpret_cast<uint32_t*>(&P.todo[w0]) = todo;
      todo = 0;
    }
    rec[j] = count == 0 ? 0u : (count == 1 ? aux : QREC_MULTI);
    if (count > 1 && s < w1) qmulti[s - w0r] = make_uint2(count, aux - count);
    rows += count;
  }
  *reinterpret_cast<uint32_t*>(&P.todo[w0 + 4]) = todo;
  if (s0 + 7 < w1) {                                       // 32-B aligned: s0 - w0r = 8 (. . .)
    uint4* o = reinterpret_cast<uint4*>(qrec + (s0 - w0r));
    o[0] = make_uint4(rec[0], rec[1], rec[2], rec[3]);
    o[1] = make_uint4(rec[4], rec[5], rec[6], rec[7]);
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (s0 + j < w1) qrec[s0 + j - w0r] = rec[j];
  }
  __syncthreads();             // phase 1's keys, flags and records (vmcnt drained) are in place
#ifndef KMHG_P2_UNROLL
#define KMHG_P2_UNROLL 2
#endif
#pragma unroll KMHG_P2_UNROLL
  for (int j = 0; j < 8; ++j) {
    const int w = j * BLOCK + (int)threadIdx.x;
    if (P.todo[w]) {
      const int64_t s = t_start + w;
      uint32_t count = 0, aux = 0;
      if (TG) table_find_tag<NT, PART>(T, TG, g, P.key[w], count, aux);
      else table_find4<NT, PART>(T, g, P.key[w], count, aux);
      put_qrec(qrec, qmulti, s - w0r, count, aux);
      rows += count;
    }
  }
  return rows;
}

// At least 6 waves per SIMD: the diagonal probe needs 81 VGPRs unconstrained (5 waves / SIMD);
// capped it fits 72 with no spill (7 waves).  A/B in one run, config 2: self query 87.0 / 90.0 ->
// 90.9 / 95.4 Gbp/s, unrelated 41.4 -> 44.3; 8 waves (64 VGPRs) spills 44 B / lane and is slower.
#ifndef KMHG_PROBE_WAVES
#define KMHG_PROBE_WAVES 6
#endif
#if KMHG_PROBE_WAVES
#define PROBE_BOUNDS __launch_bounds__(BLOCK, KMHG_PROBE_WAVES)
#else
#define PROBE_BOUNDS __launch_bounds__(BLOCK)
#endif
// PART (owner-routed query over a part of an owner-computes build): table probes only, and only
// for the windows whose key this part owns; every other window records no hit here (its owner's
// rank emits its rows).
template <bool DIAG, bool NT, bool PART = false>
__global__ void PROBE_BOUNDS
k_query_probe(const uint8_t* __restrict__ seq, int64_t L, int kq, const Slot* __restrict__ T,
              Geom g, uint32_t* __restrict__ qrec, uint2* __restrict__ qmulti, int64_t w0,
              int64_t w1, int aligned,
              uint64_t* __restrict__ tile_rows, DiagIdx X, const uint8_t* __restrict__ TG,
              uint32_t* __restrict__ ecount) {
  __shared__ Stage st;
  __shared__ uint64_t sh[8];
  __shared__ DiagAnchors A;
#ifndef KMHG_PROBE_STRIDED
  __shared__ DiagProbeLDS PL;
#endif
  const uint32_t tile = blockIdx.x;
  if (tile == 0 && threadIdx.x == 0 && ecount) *ecount = 0;   // Q_emit1's list, filled later
  // windows [w0, w1) of the FULL sequence: halo chars come from the real neighbours, so the
  // N / end-of-sequence rules at a shard boundary are those of the unsharded walk
  const int64_t t_start = w0 + (int64_t)tile * TILE;
  const int64_t base = (t_start & ~15ll) - HALO;
  const int o0 = (int)(t_start - base);
  stage_tile(seq, L, base, st, aligned != 0);
  __syncthreads();
  if (DIAG) diag_anchors<NT, PART>(st, o0, t_start, w1, L, kq, T, g, A);
  uint64_t rows = 0;
#ifndef KMHG_PROBE_UNROLL
#define KMHG_PROBE_UNROLL 2
#endif
  if (DIAG) {
#ifndef KMHG_PROBE_STRIDED
    rows = diag_resolve8<NT, PART>(st, o0, t_start, w0, w1, L, kq, T, g, X, TG, A, qrec, qmulti,
                                   PL);
    uint64_t tot8;
    block_excl_scan(rows, sh, tot8);
    if (threadIdx.x == 0) tile_rows[tile] = tot8;
    return;
#else
    static_assert(!(PART && DIAG),
                  "the strided diagonal variant (-DKMHG_PROBE_STRIDED) has no part form");
#endif
    diag_resolve<NT>(st, o0, t_start, w0, w1, L, kq, T, g, X, TG, A,
                 [&](int w, int64_t s, uint32_t count, uint32_t aux) {
                   if (s < w1) put_qrec(qrec, qmulti, s - w0, count, aux);
                   rows += count;
                 });
    uint64_t tot;
    block_excl_scan(rows, sh, tot);
    if (threadIdx.x == 0) tile_rows[tile] = tot;
    return;
  }
  // (measured: issuing all WPT home-slot loads before resolving any cost occupancy -- 94
  // VGPRs, 5 waves/SIMD -- and ran 15 % slower than this two-deep loop; a per-lane state
  // machine walking two probe streams one slot per step ran 30 % slower, and compacting the
  // windows not resolved at their home slot into LDS queue rounds 40 % slower)
#pragma unroll KMHG_PROBE_UNROLL
  for (int j = 0; j < WPT; ++j) {
    const int w = j * BLOCK + threadIdx.x;
    const int64_t s = t_start + w;
    uint64_t key = 0;
    uint32_t count = 0, aux = 0;
    if (s < w1 && window_key(st, o0 + w, s, L, kq, key) && (!PART || part_owns(key, g)))
      table_find<NT, PART>(T, g, key, count, aux);
    // {count, position} for a key seen once, {count, first index} otherwise
    if (s < w1) put_qrec(qrec, qmulti, s - w0, count, aux);
    rows += count;
  }
  uint64_t tot;
  block_excl_scan(rows, sh, tot);
  if (threadIdx.x == 0) tile_rows[tile] = tot;
}

// Exclusive scan of n per-tile u64 totals in one workgroup, any n (the fallback beyond
// SCAN1_MAX: serial loads per thread, a Hillis-Steele pass over 1024 partials).
__global__ void __launch_bounds__(1024)
k_scan_tiles_u64_any(uint64_t* __restrict__ a, uint32_t n, uint64_t* __restrict__ total) {
  __shared__ uint64_t part[1024];
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t i0 = threadIdx.x * per, i1 = min(n, i0 + per);
  uint64_t s = 0;
  for (uint32_t i = i0; i < i1; ++i) s += a[i];
  part[threadIdx.x] = s;
  __syncthreads();
  for (uint32_t d = 1; d < 1024; d <<= 1) {
    uint64_t v = threadIdx.x >= d ? part[threadIdx.x - d] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  uint64_t run = part[threadIdx.x] - s;
  for (uint32_t i = i0; i < i1; ++i) { uint64_t x = a[i]; a[i] = run; run += x; }
  if (threadIdx.x == 1023) *total = part[1023];
}

// Exclusive scan of n <= SCAN1_MAX per-tile u64 totals in one workgroup.
__global__ void __launch_bounds__(1024)
k_scan_tiles_u64(uint64_t* __restrict__ a, uint32_t n, uint64_t* __restrict__ total) {
  // thread t owns entries [t per, t per + per), per <= SCAN1_MAX / 1024, all loaded at once; the
  // wave scans by DPP, the 16 wave totals by one more wave scan (was: a serial load loop and a
  // Hillis-Steele pass over 1024 partials, 20 barriers)
  constexpr int MAXPER = (int)(SCAN1_MAX / 1024);
  __shared__ uint64_t wtot[16];
  const uint32_t per = (n + 1023) / 1024;
  const uint32_t i0 = threadIdx.x * per;
  uint64_t v[MAXPER];
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < MAXPER; ++j) {
    v[j] = ((uint32_t)j < per && i0 + j < n) ? a[i0 + j] : 0ull;
    s += v[j];
  }
  const int wave = threadIdx.x >> 6;
  const uint64_t inc = wave_incl_scan(s);
  if (lane_id() == 63) wtot[wave] = inc;
  __syncthreads();
  if (wave == 0) {
    const uint64_t w = lane_id() < 16 ? wtot[lane_id()] : 0ull;
    const uint64_t wi = wave_incl_scan(w);
    if (lane_id() < 16) wtot[lane_id()] = wi - w;       // exclusive wave offsets
    if (lane_id() == 15) *total = wi;
  }
  __syncthreads();
  uint64_t run = wtot[wave] + inc - s;
#pragma unroll
  for (int j = 0; j < MAXPER; ++j) {
    if ((uint32_t)j < per && i0 + j < n) {
      a[i0 + j] = run;
      run += v[j];
    }
  }
}

// Long u64 scans (many query tiles, e.g. 244K for a 500 Mbp query): reduce-then-scan over
// 2048-entry blocks instead of one workgroup walking the whole array.
__global__ void __launch_bounds__(BLOCK)
k_block_sum_u64(const uint64_t* __restrict__ a, uint64_t n, uint64_t* __restrict__ bsum) {
  __shared__ uint64_t sh[8];
  const uint64_t base = (uint64_t)blockIdx.x * TILE;
  uint64_t sum = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const uint64_t i = base + (uint64_t)j * BLOCK + threadIdx.x;
    if (i < n) sum += a[i];
  }
  uint64_t tot;
  block_excl_scan(sum, sh, tot);
  if (threadIdx.x == 0) bsum[blockIdx.x] = tot;
}

__global__ void __launch_bounds__(BLOCK)
k_block_scan_u64(uint64_t* __restrict__ a, uint64_t n, const uint64_t* __restrict__ bbase) {
  __shared__ uint64_t sh[8];
  const uint64_t base = (uint64_t)blockIdx.x * TILE + (uint64_t)threadIdx.x * WPT;
  uint64_t v[WPT];
  uint64_t sum = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    v[j] = (base + j < n) ? a[base + j] : 0ull;
    sum += v[j];
  }
  uint64_t tot;
  uint64_t run = block_excl_scan(sum, sh, tot) + bbase[blockIdx.x];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (base + j < n) a[base + j] = run;
    run += v[j];
  }
}

// Q_emit: output rows (i = 1-based window end, j = 1-based index position), ordered by i then j
// as in the reference.  Per tile: LDS prefix of the windows' hit counts; windows with at most
// EMIT_DIRECT hits write their rows themselves, lane-consecutive windows so that the common
// one-hit rows are consecutive (coalesced) stores; windows with more hits are then dealt to the
// whole workgroup one at a time, so a window with thousands of hits does not serialise a lane.
// Rows at or beyond `cap` are dropped: the host launches the emit before it knows the total and
// re-runs it into an exact-size buffer in the rare case the guess was short.
constexpr uint32_t EMIT_DIRECT = 4;
__global__ void __launch_bounds__(BLOCK)
k_query_emit(const uint32_t* __restrict__ qrec, const uint2* __restrict__ qmulti, int64_t Nw,
             int64_t w0, int kq,
             const int32_t* __restrict__ positions, const uint64_t* __restrict__ tile_row0,
             int2* __restrict__ out, uint64_t cap, const uint32_t* __restrict__ elist,
             const uint32_t* __restrict__ ecount) {
  __shared__ uint64_t incl[TILE];
  __shared__ uint32_t start[TILE];
  using HeavyT = uint16_t;            // a window of the tile (< TILE): 28.7 KB of LDS, 5 groups / CU
  static_assert(TILE <= 65536, "heavy[] holds tile-local window indices");
  __shared__ HeavyT heavy[TILE];
  __shared__ uint32_t n_heavy;
  __shared__ uint64_t sh[8];
  const uint32_t nlist = *ecount;
  for (uint32_t li = blockIdx.x; li < nlist; li += gridDim.x) {
  const uint32_t tile = elist[li];
  const int64_t tile0 = (int64_t)tile * TILE;
  __syncthreads();                      // the previous tile's reads of the LDS arrays are done
  if (threadIdx.x == 0) n_heavy = 0;
  // load counts / starts (coalesced), then thread-contiguous prefix over WPT entries
  for (int j = 0; j < WPT; ++j) {
    int w = j * BLOCK + threadIdx.x;
    int64_t s = tile0 + w;
    const uint32_t rc = (s < Nw) ? qrec[s] : 0u;
    uint2 v = make_uint2(rc ? 1u : 0u, rc);
    if (rc == QREC_MULTI) v = qmulti[s];
    incl[w] = v.x;
    start[w] = v.y;
  }
  __syncthreads();
  uint64_t run = 0;
  uint64_t loc[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) { run += incl[threadIdx.x * WPT + j]; loc[j] = run; }
  uint64_t tot;
  uint64_t ex = block_excl_scan(run, sh, tot);
#pragma unroll
  for (int j = 0; j < WPT; ++j) incl[threadIdx.x * WPT + j] = loc[j] + ex;
  __syncthreads();
  if (tot == 0) continue;               // uniform: every thread skips the tile
  const uint64_t r0 = tile_row0[tile];
  const int32_t i0 = (int32_t)(w0 + tile0 + kq);
#pragma unroll 2
  for (int j = 0; j < WPT; ++j) {
    const int w = j * BLOCK + threadIdx.x;
    const uint64_t before = w ? incl[w - 1] : 0;
    const uint64_t n = incl[w] - before;
    if (n == 0) continue;
    if (n > EMIT_DIRECT) {
      heavy[atomicAdd(&n_heavy, 1u)] = (HeavyT)w;
      continue;
    }
    const uint64_t r = r0 + before;
    const uint32_t st0 = start[w];
    if (n == 1) {
      if (r < cap) out[r] = make_int2(i0 + w, (int32_t)st0);
    } else {
      for (uint32_t q = 0; q < (uint32_t)n; ++q)
        if (r + q < cap) out[r + q] = make_int2(i0 + w, positions[st0 + q]);
    }
  }
  __syncthreads();
  const uint32_t nh = n_heavy;
  for (uint32_t h = 0; h < nh; ++h) {
    const uint32_t w = heavy[h];
    const uint64_t before = w ? incl[w - 1] : 0;
    const uint64_t n = incl[w] - before;
    const uint64_t r = r0 + before;
    const uint32_t st0 = start[w];
    for (uint64_t q = threadIdx.x; q < n; q += BLOCK)
      if (r + q < cap) out[r + q] = make_int2(i0 + (int32_t)w, positions[st0 + (uint32_t)q]);
  }
  }
}

// Q_emit1 (round 4): the tiles whose windows have at most one hit each -- a dot plot's
// diagonals, an unrelated query's misses, most of any query.  The rows of such a tile are its
// hit windows in window order, so one ballot per (element row, wave) and one wave scan from the
// tile's first row place them: no LDS arrays (Q_emit's 29 KB hold it to 5 workgroups per CU),
// 8-B rows from consecutive lanes to consecutive rows.  A tile with a multi-hit window goes on
// `elist` for Q_emit instead (append = 0 on a re-emit into an exact buffer: the list is complete).
__global__ void __launch_bounds__(BLOCK)
k_query_emit1(const uint32_t* __restrict__ qrec, int64_t Nw, int64_t w0, int kq,
              const uint64_t* __restrict__ tile_row0, int2* __restrict__ out, uint64_t cap,
              uint32_t* __restrict__ elist, uint32_t* __restrict__ ecount, int append) {
  __shared__ uint64_t cw[WPT * (BLOCK / 64) + 1];
  const uint32_t tile = blockIdx.x;
  const int64_t tile0 = (int64_t)tile * TILE;
  uint32_t rec[WPT];
  bool hit[WPT];
  int multi = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int64_t e = tile0 + j * BLOCK + threadIdx.x;
    rec[j] = e < Nw ? qrec[e] : 0u;
    multi |= rec[j] == QREC_MULTI;
    hit[j] = rec[j] != 0u;
  }
  if (__syncthreads_or(multi)) {
    if (append && threadIdx.x == 0) elist[atomicAdd(ecount, 1u)] = tile;
    return;
  }
  uint64_t rk[WPT];
  tile_rank_at<WPT>(hit, rk, cw, tile_row0[tile]);
  const int32_t i0 = (int32_t)(w0 + tile0 + kq);
#pragma unroll
  for (int j = 0; j < WPT; ++j)
    if (hit[j] && rk[j] < cap) out[rk[j]] = make_int2(i0 + j * BLOCK + (int)threadIdx.x, (int32_t)rec[j]);
}

// ================================================================== readout kernels
// The index is the table + positions: a key's slot carries {key, count, end} and its
// positions are [end - count, end).  Canonical k-mer order (first occurrence) is a slot
// permutation `perm` built once per index (R_first + R_order) and cached.

// R_first: F[first position - 1] = {slot, count}, for every occupied slot (positions ascend per
// key).  The count travels with the slot so that R_order reads F alone, in position order,
// instead of gathering every key's slot again (a random 16-B read per key).
__global__ void __launch_bounds__(BLOCK)
k_read_first(const Slot* __restrict__ T, uint64_t nslots, const int32_t* __restrict__ positions,
             uint2* __restrict__ F) {
  for (uint64_t i = (uint64_t)blockIdx.x * BLOCK + threadIdx.x; i < nslots;
       i += (uint64_t)gridDim.x * BLOCK) {
    uint4 v = *reinterpret_cast<const uint4*>(&T[i]);
    if (v.z)
      F[(v.z == 1 ? (int32_t)v.w : positions[v.w - v.z]) - 1] = make_uint2((uint32_t)i, v.z);
  }
}

// R_order: compact F in position order -> perm (canonical order = first occurrence), with the
// canonical pos-row offsets, the list of keys that own pair rows with their pair offsets, and
// rinfo.  Three look-back chains: {keys, pos rows} packed 31|31, {multi keys}, {pair rows}.
// Tiles are lane-contiguous (element j * BLOCK + t: every load and store of a step coalesced);
// ranks come from per-(j, wave) ballots and wave scans, so compaction order == position order.
__global__ void __launch_bounds__(BLOCK)
k_read_order(const uint2* __restrict__ F, int64_t L, const Slot* __restrict__ T,
             uint64_t* __restrict__ st_a, uint64_t* __restrict__ st_b, uint64_t* __restrict__ st_c,
             uint32_t* __restrict__ ticket, uint32_t* __restrict__ perm,
             uint32_t* __restrict__ canon_off, uint32_t* __restrict__ pkeys,
             uint64_t* __restrict__ pair_off, uint2* __restrict__ rinfo, uint32_t ntiles,
             ReadMeta* __restrict__ rmeta) {
  constexpr int NW = BLOCK / 64;
  __shared__ uint64_t wk[WPT * NW], wr[WPT * NW], wm[WPT * NW], wp[WPT * NW];
  __shared__ uint32_t tk;
  const uint32_t tile = take_ticket(ticket, &tk);
  const int64_t t0 = (int64_t)tile * TILE;
  const int wave = threadIdx.x >> 6, lane = lane_id();
  uint32_t id[WPT], nn[WPT];
  uint64_t mk[WPT], mm[WPT], rinc[WPT], pinc[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const int64_t p = t0 + (int64_t)j * BLOCK + threadIdx.x;
    const uint2 f = (p < L) ? F[p] : make_uint2(NONE, 0u);
    id[j] = f.x;
    nn[j] = (id[j] != NONE) ? f.y : 0u;
    const uint64_t n = nn[j];
    mk[j] = __ballot(id[j] != NONE);
    mm[j] = __ballot(n >= 2);
    rinc[j] = wave_incl_scan(n);
    pinc[j] = wave_incl_scan(n * (n - (n ? 1 : 0)) / 2);
    if (lane == 63) {
      wk[j * NW + wave] = (uint64_t)__popcll(mk[j]);
      wr[j * NW + wave] = rinc[j];
      wm[j * NW + wave] = (uint64_t)__popcll(mm[j]);
      wp[j * NW + wave] = pinc[j];
    }
  }
  __syncthreads();
  if (wave == 0) {                          // lanes 0 .. WPT*NW-1: one (j, wave) group each
    const bool own = lane < WPT * NW;
    const uint64_t ck = own ? wk[lane] : 0, cr = own ? wr[lane] : 0;
    const uint64_t cm = own ? wm[lane] : 0, cp = own ? wp[lane] : 0;
    const uint64_t ik = wave_incl_scan(ck), ir = wave_incl_scan(cr);
    const uint64_t im = wave_incl_scan(cm), ip = wave_incl_scan(cp);
    const uint64_t tk_ = lane63(ik), tr = lane63(ir), tm = lane63(im), tp = lane63(ip);
    const uint64_t agga = (tk_ << 31) | tr;
    const uint64_t xa = lookback_excl(st_a, tile, agga);
    const uint64_t xb = lookback_excl(st_b, tile, tm);
    const uint64_t xc = lookback_excl(st_c, tile, tp);
    if (lane == 0 && tile == ntiles - 1) {
      rmeta->n_keys = (xa + agga) >> 31;
      rmeta->n_rows = (xa + agga) & ((1ull << 31) - 1);
      rmeta->n_multi = xb + tm;
      rmeta->n_pairs = xc + tp;
    }
    if (own) {
      wk[lane] = (xa >> 31) + ik - ck;
      wr[lane] = (xa & ((1ull << 31) - 1)) + ir - cr;
      wm[lane] = xb + im - cm;
      wp[lane] = xc + ip - cp;
    }
  }
  __syncthreads();
  const uint64_t lt = lanemask_lt();
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (id[j] == NONE) continue;
    const int g = j * NW + wave;
    const uint32_t n = nn[j];
    const uint64_t ca = wk[g] + (uint64_t)__popcll(mk[j] & lt);
    perm[ca] = id[j];
    canon_off[ca] = (uint32_t)(wr[g] + rinc[j] - n);
    // the row's slot fields {count, aux}: a key seen once starts here (aux = its position),
    // only a repeated key's list end needs its slot
    rinfo[ca] = make_uint2(n, n == 1 ? (uint32_t)(t0 + (int64_t)j * BLOCK + threadIdx.x + 1)
                                     : T[id[j]].aux);
    if (n >= 2) {
      const uint64_t cb = wm[g] + (uint64_t)__popcll(mm[j] & lt);
      const uint64_t c2 = (uint64_t)n * (n - 1) / 2;
      pkeys[cb] = (uint32_t)ca;
      pair_off[cb] = wp[g] + pinc[j] - c2;
    }
  }
}

// R_keys: counts (opt 8) and k-mer strings (opt 1) in canonical order.
__global__ void __launch_bounds__(BLOCK)
k_read_keys(const uint32_t* __restrict__ perm, const uint2* __restrict__ rinfo, uint32_t U,
            const Slot* __restrict__ T, int k, int32_t* __restrict__ out_counts,
            char* __restrict__ out_kmers) {
  const char NUC[4] = {'A', 'C', 'T', 'G'};             // src/kmer_hash.c:21
  for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < U; c += gridDim.x * BLOCK) {
    if (out_counts) out_counts[c] = (int32_t)rinfo[c].x;
    if (out_kmers) {                                    // the key needs the slot itself
      uint64_t key = T[perm[c]].key;
      char* o = out_kmers + (size_t)c * (k + 1);
      for (int i = k - 1; i >= 0; --i) { o[i] = NUC[key & 3]; key >>= 2; }
      o[k] = 0;
    }
  }
}

// Keys of the readout order (khash row-order replay input): out[c] = key of perm[c].
__global__ void __launch_bounds__(BLOCK)
k_gather_keys(const uint32_t* __restrict__ perm, uint32_t U, const Slot* __restrict__ T,
              uint64_t* __restrict__ out_keys) {
  for (uint32_t c = blockIdx.x * BLOCK + threadIdx.x; c < U; c += gridDim.x * BLOCK)
    out_keys[c] = T[perm[c]].key;
}

// R_pos: rows (i, pos) in canonical order.  Each workgroup owns TILE output rows; every key
// owns >= 1 row so its key range fits the LDS copy of the canonical offsets.  The key holding
// each tile's first row comes from R_tiles (no per-workgroup search of the global offsets);
// rows are staged in LDS and leave as 16-B stores.
// R_tiles: tile_key[t] = the key holding row t*tile (every row belongs to one key);
// tile_key[ntiles] = nkeys - 1.
template <class Off>
__global__ void __launch_bounds__(BLOCK)
k_row_tiles(const Off* __restrict__ off, uint32_t nkeys, uint64_t nrows, uint32_t tile,
            uint32_t* __restrict__ tile_key, uint32_t ntiles) {
  // one lane per key writes the tiles whose first row the key holds; a key spanning more than
  // RT_LANE tiles (a heavy key's pairs: C(14,097, 2) rows = 48 K tiles at config 4) is handed
  // to the whole wave, which strides over its tiles, instead of one lane storing them in turn
  constexpr uint64_t RT_LANE = 8;
  const int lane = lane_id();
  const uint32_t stride = gridDim.x * BLOCK;
  for (uint32_t m0 = blockIdx.x * BLOCK + (threadIdx.x & ~63u); m0 < nkeys; m0 += stride) {
    const uint32_t m = m0 + lane;                // wave-uniform trip count: m0 is per wave
    uint64_t t0 = 0, t1 = 0;
    if (m < nkeys) {
      const uint64_t lo = off[m], hi = m + 1 < nkeys ? (uint64_t)off[m + 1] : nrows;
      t0 = (lo + tile - 1) / tile;
      t1 = (hi + tile - 1) / tile;               // tiles t with t * tile in [lo, hi)
      if (t1 > t0 && t1 - t0 <= RT_LANE)
        for (uint64_t t = t0; t < t1; ++t) tile_key[t] = m;
    }
    uint64_t heavy = __ballot(t1 > t0 + RT_LANE);
    while (heavy) {
      const int src = __ffsll((unsigned long long)heavy) - 1;
      heavy &= heavy - 1;
      const uint64_t a = __shfl(t0, src), b = __shfl(t1, src);
      const uint32_t key = m0 + (uint32_t)src;
      for (uint64_t t = a + (uint64_t)lane; t < b; t += 64) tile_key[t] = key;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) tile_key[ntiles] = nkeys - 1;
}

__global__ void __launch_bounds__(BLOCK)
k_read_pos(const uint2* __restrict__ rinfo, const uint32_t* __restrict__ canon_off,
           const uint32_t* __restrict__ tile_key, uint64_t nrows,
           const int32_t* __restrict__ positions, int2* __restrict__ out) {
  __shared__ uint32_t off[TILE + 1];
  __shared__ __attribute__((aligned(16))) int2 stage[TILE];
  const uint64_t r0 = (uint64_t)blockIdx.x * TILE;
  const uint64_t r1 = min(nrows, r0 + TILE);
  const uint32_t c0 = tile_key[blockIdx.x];
  uint32_t c1 = tile_key[blockIdx.x + 1];
  if (r1 < nrows && canon_off[c1] == r1) --c1;
  const uint32_t nk = c1 - c0 + 1;
  for (uint32_t i = threadIdx.x; i < nk; i += BLOCK) off[i] = canon_off[c0 + i];
  __syncthreads();
  // thread t: the WPT consecutive rows r0 + t*WPT ...; one binary search, then row by row
  const uint64_t rb = r0 + (uint64_t)threadIdx.x * WPT;
  if (rb < r1) {
    uint32_t lo = 0, hi = nk - 1;
    while (lo < hi) { uint32_t mid = (lo + hi + 1) >> 1; if (off[mid] <= rb) lo = mid; else hi = mid - 1; }
    uint2 v = rinfo[c0 + lo];
    uint32_t t = (uint32_t)(rb - off[lo]);
    const uint32_t nr = (uint32_t)min<uint64_t>(WPT, r1 - rb);
    for (uint32_t i = 0; i < nr; ++i) {
      if (i > 0 && ++t == v.x) { v = rinfo[c0 + ++lo]; t = 0; }
      const int32_t p = v.x == 1 ? (int32_t)v.y : positions[v.y - v.x + t];
      stage[threadIdx.x * WPT + i] = make_int2((int32_t)(c0 + lo + 1), p);
    }
  }
  __syncthreads();
  const uint32_t nrow = (uint32_t)(r1 - r0);
  int2* dst = out + r0;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {        // two rows per 16-B store
    for (uint32_t i = threadIdx.x; i < nrow / 2; i += BLOCK)
      reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(stage)[i];
    if ((nrow & 1) && threadIdx.x == 0) dst[nrow - 1] = stage[nrow - 1];
  } else {
    for (uint32_t i = threadIdx.x; i < nrow; i += BLOCK) dst[i] = stage[i];
  }
}

// R_pairs: rows (i, x, y), x < y, j-outer / k-inner inside a key (src/kmer_hash.c:1113-1121).
// Keys without pairs are excluded from pkeys, so again every listed key owns >= 1 row.  A
// workgroup owns PR_TILE rows; R_tiles has recorded the key holding each tile's first row, so
// no workgroup binary-searches the global offsets.  The tile is produced in two halves; in each,
// thread t makes the PR_HALF consecutive rows h0 + t*PR_HALF ...: one LDS binary search and one
// triangular-root inversion for the first, then (j, q) advance row by row; all position loads
// are issued before any is used; the half's rows are staged in LDS and leave as 16-B stores
// over its contiguous 12*BLOCK*PR_HALF bytes.  (Round 4: the kernel waits on its chain of
// dependent loads -- tile key, offsets, key, run, positions -- so what counts is the rows in
// flight per CU.  The whole-tile 24-KB stage ran 4 waves per SIMD; the 12-KB half stage and
// 16-bit offsets run 6 (80 VGPRs): config 4 2.49 -> 2.29 ms.  Forcing 8 (64 VGPRs, spills)
// 4.19 ms; stores straight from registers -- each lane's 96 contiguous bytes -- 3.57 ms.
// A/B in one run, profiles/rd4z_*.)
constexpr int PR_PER = 8;
constexpr int PR_HALF = PR_PER / 2;
constexpr int PR_TILE = BLOCK * PR_PER;
static_assert(PR_TILE <= 65536, "offsets inside a tile are 16-bit");

__global__ void __launch_bounds__(BLOCK, 6)
k_read_pairs(const uint32_t* __restrict__ pkeys, const uint64_t* __restrict__ pair_off,
             const uint32_t* __restrict__ tile_key, uint64_t nrows,
             const uint2* __restrict__ rinfo, const int32_t* __restrict__ positions,
             int32_t* __restrict__ out) {
  __shared__ uint16_t offr[PR_TILE];        // key start rows - r0 (the first key's clamped to 0)
  __shared__ __attribute__((aligned(16))) int32_t stage[3 * BLOCK * PR_HALF];
  __shared__ uint64_t first_off;
  const uint32_t b = blockIdx.x;
  const uint64_t r0 = (uint64_t)b * PR_TILE;
  const uint64_t r1 = min(nrows, r0 + PR_TILE);
  // keys of the tile: m0 holds row r0; the last holds row r1 - 1
  const uint32_t m0 = tile_key[b];
  uint32_t m1 = tile_key[b + 1];
  if (r1 < nrows && pair_off[m1] == r1) --m1;
  const uint32_t nk = m1 - m0 + 1;
  for (uint32_t i = threadIdx.x; i < nk; i += BLOCK) {
    const uint64_t o = pair_off[m0 + i];
    offr[i] = (uint16_t)(o > r0 ? o - r0 : 0u);
    if (i == 0) first_off = o;
  }
  __syncthreads();
#pragma unroll 1
  for (int half = 0; half < 2; ++half) {
    const uint32_t hrel = (uint32_t)half * BLOCK * PR_HALF;
    const uint32_t rel = hrel + threadIdx.x * PR_HALF;
    const uint64_t rb = r0 + rel;
    if (rb < r1) {
      uint32_t lo = 0, hi = nk - 1;
      while (lo < hi) { uint32_t mid = (lo + hi + 1) >> 1; if (offr[mid] <= rel) lo = mid; else hi = mid - 1; }
      uint32_t c = pkeys[m0 + lo];
      uint2 v = rinfo[c];
      uint32_t n = v.x;
      const uint64_t t = lo == 0 ? rb - first_off : (uint64_t)(rel - offr[lo]);
      // largest j with S(j) = j*(2n-j-1)/2 <= t
      const uint64_t n64 = n;
      double dn = (double)(2 * n64 - 1);
      double disc = dn * dn - 8.0 * (double)t;
      int64_t jj = (int64_t)((dn - sqrt(disc > 0 ? disc : 0)) * 0.5);
      if (jj < 0) jj = 0;
      if (jj > (int64_t)n64 - 2) jj = (int64_t)n64 - 2;
      auto S = [n64](int64_t x) -> uint64_t { return (uint64_t)x * (2 * n64 - (uint64_t)x - 1) / 2; };
      while (jj > 0 && S(jj) > t) --jj;
      while (jj + 1 <= (int64_t)n64 - 2 && S(jj + 1) <= t) ++jj;
      uint32_t j = (uint32_t)jj;
      uint32_t q = j + 1 + (uint32_t)(t - S(jj));
      uint32_t base = v.y - v.x;
      const uint32_t nr = (uint32_t)min<uint64_t>(PR_HALF, r1 - rb);
      uint32_t ij[PR_HALF], iq[PR_HALF], cc[PR_HALF];
#pragma unroll
      for (int i = 0; i < PR_HALF; ++i) {
        if ((uint32_t)i >= nr) break;
        // advance before every row but the first (no key past this thread's rows is touched)
        if (i > 0 && ++q == n) {               // next j; past the last pair: the next key
          if (++j == n - 1) {
            c = pkeys[m0 + ++lo];
            v = rinfo[c];
            n = v.x;
            base = v.y - v.x;
            j = 0;
          }
          q = j + 1;
        }
        ij[i] = base + j;
        iq[i] = base + q;
        cc[i] = c + 1;
      }
      int32_t pj[PR_HALF], pq[PR_HALF];
#pragma unroll
      for (int i = 0; i < PR_HALF; ++i)
        if ((uint32_t)i < nr) { pj[i] = positions[ij[i]]; pq[i] = positions[iq[i]]; }
      int32_t* o = stage + 3 * threadIdx.x * PR_HALF;
#pragma unroll
      for (int i = 0; i < PR_HALF; ++i)
        if ((uint32_t)i < nr) { o[3 * i] = (int32_t)cc[i]; o[3 * i + 1] = pj[i]; o[3 * i + 2] = pq[i]; }
    }
    __syncthreads();
    // the half's rows are the contiguous ints [3 h0, 3 h1) of out
    const uint64_t h0 = r0 + hrel;
    const uint32_t nint = h0 < r1 ? 3 * (uint32_t)(min<uint64_t>(r1, h0 + BLOCK * PR_HALF) - h0) : 0u;
    int32_t* dst = out + 3 * h0;
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      const uint32_t n4 = nint / 4;
      for (uint32_t i = threadIdx.x; i < n4; i += BLOCK)
        reinterpret_cast<int4*>(dst)[i] = reinterpret_cast<const int4*>(stage)[i];
      for (uint32_t i = 4 * n4 + threadIdx.x; i < nint; i += BLOCK) dst[i] = stage[i];
    } else {
      for (uint32_t i = threadIdx.x; i < nint; i += BLOCK) dst[i] = stage[i];
    }
    if (half == 0) __syncthreads();          // the stage is refilled by the second half
  }
}

// ================================================================== launchers
static inline unsigned grid_for(uint64_t n, unsigned per) {
  uint64_t g = (n + per - 1) / per;
  return (unsigned)(g ? g : 1);
}

void launch_part_rebase(const Slot* src, Slot* dst, uint64_t n, uint32_t base, hipStream_t s) {
  if (!n) return;
  unsigned g = grid_for(n, BLOCK);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_part_rebase, dim3(g), dim3(BLOCK), 0, s, src, dst, n, base);
}
void launch_table_init(Slot* T, uint64_t n, hipStream_t s) {
  unsigned g = grid_for(n, BLOCK);
  if (g > 8192) g = 8192;
  hipLaunchKernelGGL(k_table_init, dim3(g), dim3(BLOCK), 0, s, T, n);
}
void launch_build_insert(const uint8_t* seq, int64_t L, int k, Slot* T, Geom g,
                         uint32_t* win_slot, int64_t Nw, bool aligned, hipStream_t s) {
  hipLaunchKernelGGL(k_build_insert, dim3(grid_for(Nw, TILE)), dim3(BLOCK), 0, s, seq, L, k, T,
                     g, win_slot, Nw, aligned ? 1 : 0);
}
void launch_build_compact(Slot* T, uint64_t nslots, uint64_t* status, uint32_t* ticket,
                          uint64_t* ukeys, uint32_t* counts, uint32_t* offsets,
                          uint32_t* small_ids, uint32_t* large_ids, BuildMeta* meta,
                          hipStream_t s) {
  uint32_t nt = grid_for(nslots, TILE);
  hipLaunchKernelGGL(k_build_compact, dim3(nt), dim3(BLOCK), 0, s, T, nslots, status, ticket,
                     ukeys, counts, offsets, small_ids, large_ids, meta, nt,
                     (uint32_t)LARGE_MIN);
}
void launch_build_scatter(const uint32_t* win_slot, int64_t Nw, Slot* T, int32_t* positions,
                          hipStream_t s) {
  hipLaunchKernelGGL(k_build_scatter, dim3(grid_for(Nw, TILE)), dim3(BLOCK), 0, s, win_slot, Nw,
                     T, positions);
}
void launch_sort_small(const uint32_t* small_ids, const BuildMeta* meta, const uint32_t* counts,
                       const uint32_t* offsets, int32_t* positions, hipStream_t s) {
  hipLaunchKernelGGL(k_sort_small, dim3(2048), dim3(BLOCK), 0, s, small_ids, meta, counts,
                     offsets, positions);
}
void launch_sort_large(const uint32_t* large_ids, const BuildMeta* meta, const uint32_t* counts,
                       const uint32_t* offsets, int32_t* positions, int32_t* tmp, hipStream_t s) {
  hipLaunchKernelGGL(k_sort_large, dim3(1024), dim3(BLOCK), 0, s, large_ids, meta, counts,
                     offsets, positions, tmp);
}
void launch_inline_singles(Slot* T, uint64_t nslots, const int32_t* positions, hipStream_t s) {
  unsigned g = grid_for(nslots, BLOCK);
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_inline_singles, dim3(g), dim3(BLOCK), 0, s, T, nslots, positions);
}
#ifndef KMHG_NT_PROBE_MB
#define KMHG_NT_PROBE_MB 4096
#endif
constexpr uint64_t NT_PROBE_BYTES = (uint64_t)KMHG_NT_PROBE_MB << 20;
void launch_query_probe(const uint8_t* seq, int64_t L, int kq, const Slot* T, Geom g,
                        uint32_t* qrec, uint2* qmulti, int64_t w0, int64_t w1, bool aligned,
                        uint64_t* tile_rows,
                        hipStream_t s, DiagIdx X, const uint8_t* TG, uint32_t* ecount) {
  uint32_t nt = grid_for(w1 - w0, TILE);
  if (g.capb % 16 != 0) TG = nullptr;           // the tag groups are aligned 16-slot spans
  // nontemporal slot reads for a table of more than NT_PROBE_BYTES.  A/B in one run
  // (profiles/r5n_ab_ntslot_*): the 12-GB table of the 500 Mbp record 5.40 -> 5.20 ms per
  // query, config 3's 2.4 GB +-0, config 2's 0.24 GB -4 % (its table lines are reused)
  const bool ntl = (uint64_t)g.nb * g.capb * sizeof(Slot) > NT_PROBE_BYTES;
  if (g.nbh) {                                  // a part's table: the windows it owns
    if (X.code && ntl)
      hipLaunchKernelGGL((k_query_probe<true, true, true>), dim3(nt), dim3(BLOCK), 0, s, seq, L,
                         kq, T, g, qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows, X, TG, ecount);
    else if (X.code)
      hipLaunchKernelGGL((k_query_probe<true, false, true>), dim3(nt), dim3(BLOCK), 0, s, seq, L,
                         kq, T, g, qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows, X, TG, ecount);
    else
      hipLaunchKernelGGL((k_query_probe<false, false, true>), dim3(nt), dim3(BLOCK), 0, s, seq, L,
                         kq, T, g, qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows,
                         DiagIdx{nullptr, nullptr, 0}, nullptr, ecount);
    return;
  }
  if (X.code) {
    if (ntl)
      hipLaunchKernelGGL((k_query_probe<true, true>), dim3(nt), dim3(BLOCK), 0, s, seq, L, kq, T, g,
                         qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows, X, TG, ecount);
    else
      hipLaunchKernelGGL((k_query_probe<true, false>), dim3(nt), dim3(BLOCK), 0, s, seq, L, kq, T, g,
                         qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows, X, TG, ecount);
  } else {
    hipLaunchKernelGGL((k_query_probe<false, false>), dim3(nt), dim3(BLOCK), 0, s, seq, L, kq, T, g,
                       qrec, qmulti, w0, w1, aligned ? 1 : 0, tile_rows,
                       DiagIdx{nullptr, nullptr, 0}, nullptr, ecount);
  }
}
// ---------------------------------------------------------------- owner-routed query merge
// dist.owner_query: rank r queried every window against its part of an owner-computes build and
// holds the rows of the windows whose k-mer it owns, in window order, with its tile offsets
// tile_off[r * (nt + 1) + t] (exclusive, [nt] = its total).  A window's rows all come from one
// rank (its key's owner), in j order; merged, query tile t's rows start at the sum over the
// ranks of their offset of t and are ordered by window.  One workgroup per tile: count the rows
// of every window of the tile in LDS (and where each window's run starts in its rank's
// segment), scan the counts, then place every row at its window's start + its index in the run.
// Two reads of the rows and one write: the merge moves 24 B per row.
__global__ void __launch_bounds__(BLOCK)
k_merge_part_rows(const int2* __restrict__ rows, const uint64_t* __restrict__ seg_base,
                  const uint64_t* __restrict__ tile_off, uint32_t n_parts, uint32_t nt, int kq,
                  int64_t w0, int2* __restrict__ out) {
  __shared__ uint32_t cnt[TILE];
  __shared__ uint32_t first[TILE];
  __shared__ uint64_t sh[8];
  const uint32_t t = blockIdx.x;
  const int64_t wt = w0 + (int64_t)t * TILE;              // the tile's first window
  for (uint32_t o = threadIdx.x; o < TILE; o += BLOCK) cnt[o] = 0;
  uint64_t out0 = 0;
  for (uint32_t r = 0; r < n_parts; ++r) out0 += tile_off[(uint64_t)r * (nt + 1) + t];
  __syncthreads();
  for (uint32_t r = 0; r < n_parts; ++r) {
    const uint64_t a = tile_off[(uint64_t)r * (nt + 1) + t];
    const uint64_t b = tile_off[(uint64_t)r * (nt + 1) + t + 1];
    const int2* R = rows + seg_base[r];
    for (uint64_t p = a + threadIdx.x; p < b; p += BLOCK) {
      const int i = R[p].x;
      const uint32_t o = (uint32_t)((int64_t)i - kq - wt);   // window start - tile start
      atomicAdd(&cnt[o], 1u);
      if (p == a || R[p - 1].x != i) first[o] = (uint32_t)(p - a);
    }
  }
  __syncthreads();
  // exclusive scan of the TILE counts: 8 consecutive windows per thread
  uint32_t c8[WPT], sum = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    c8[j] = cnt[threadIdx.x * WPT + j];
    sum += c8[j];
  }
  uint64_t tot;
  uint32_t run = (uint32_t)block_excl_scan((uint64_t)sum, sh, tot);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    cnt[threadIdx.x * WPT + j] = run;                      // now each window's first row
    run += c8[j];
  }
  __syncthreads();
  for (uint32_t r = 0; r < n_parts; ++r) {
    const uint64_t a = tile_off[(uint64_t)r * (nt + 1) + t];
    const uint64_t b = tile_off[(uint64_t)r * (nt + 1) + t + 1];
    const int2* R = rows + seg_base[r];
    for (uint64_t p = a + threadIdx.x; p < b; p += BLOCK) {
      const int2 v = R[p];
      const uint32_t o = (uint32_t)((int64_t)v.x - kq - wt);
      out[out0 + cnt[o] + ((uint32_t)(p - a) - first[o])] = v;
    }
  }
}

__global__ void k_fill_u64(uint64_t* __restrict__ p, uint64_t v) { *p = v; }

void launch_merge_part_rows(const int2* rows, const uint64_t* seg_base, const uint64_t* tile_off,
                            uint32_t n_parts, uint32_t nt, int kq, int64_t w0, int2* out,
                            hipStream_t s) {
  hipLaunchKernelGGL(k_merge_part_rows, dim3(nt), dim3(BLOCK), 0, s, rows, seg_base, tile_off,
                     n_parts, nt, kq, w0, out);
}
void launch_fill_u64(uint64_t* p, uint64_t v, hipStream_t s) {
  hipLaunchKernelGGL(k_fill_u64, dim3(1), dim3(1), 0, s, p, v);
}

// ---------------------------------------------------------------- diagonal runs (row gather)
// The sharded query's rows travel to the root as diagonal runs: a run is a maximal stretch of
// consecutive rows (i, j), (i + 1, j + 1), ... -- a dot plot's diagonal -- sent as {its first
// row's index in the rank's rows, i, j} (12 B) instead of 8 B per row.  Config 5 (B = A + 1 %
// SNVs) has 133 rows per run.  run_start decides a row's start: row 0, or i / j not both one
// past the previous row's.  Tiles of TILE rows, element e = j * BLOCK + t (lane-contiguous).
__device__ __forceinline__ bool run_start(const int2* __restrict__ rows, uint64_t r) {
  if (r == 0) return true;
  const int2 v = rows[r], p = rows[r - 1];
  return (uint32_t)v.x != (uint32_t)p.x + 1u || (uint32_t)v.y != (uint32_t)p.y + 1u;
}

// R_count: run starts per tile -> tile_cnt (scanned by launch_scan_u64 into tile offsets)
__global__ void __launch_bounds__(BLOCK)
k_runs_count(const int2* __restrict__ rows, uint64_t n, uint64_t* __restrict__ tile_cnt) {
  __shared__ uint32_t wc[BLOCK / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  uint32_t c = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const uint64_t r = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    c += (uint32_t)__popcll(__ballot(r < n && run_start(rows, r)));
  }
  if (lane_id() == 0) wc[threadIdx.x >> 6] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t t = 0;
#pragma unroll
    for (int w = 0; w < BLOCK / 64; ++w) t += wc[w];
    tile_cnt[blockIdx.x] = t;
  }
}

// R_emit: every run start as {row index, i, j} at its tile's offset + its rank in the tile
__global__ void __launch_bounds__(BLOCK)
k_runs_emit(const int2* __restrict__ rows, uint64_t n, const uint64_t* __restrict__ tile_off,
            int32_t* __restrict__ runs) {
  __shared__ uint64_t cw[WPT * (BLOCK / 64) + 1];
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  bool st[WPT];
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const uint64_t r = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    st[j] = r < n && run_start(rows, r);
  }
  uint64_t rk[WPT];
  tile_rank_at<WPT>(st, rk, cw, tile_off[blockIdx.x]);
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    if (st[j]) {
      const uint64_t r = t0 + (uint64_t)j * BLOCK + threadIdx.x;
      const int2 v = rows[r];
      int32_t* o = runs + 3 * rk[j];
      o[0] = (int32_t)r;
      o[1] = v.x;
      o[2] = v.y;
    }
  }
}

// R_cover: for every output tile t, the run covering its first row t * TILE (the last run
// starting at or before it): a binary search over the run starts, one thread per tile
__global__ void __launch_bounds__(BLOCK)
k_runs_cover(const int32_t* __restrict__ runs, uint64_t n_runs, uint32_t nt,
             uint32_t* __restrict__ cover) {
  const uint32_t t = blockIdx.x * BLOCK + threadIdx.x;
  if (t >= nt) return;
  const uint64_t row = (uint64_t)t * TILE;
  uint64_t lo = 0, hi = n_runs;                 // runs[0] starts at row 0
  while (hi - lo > 1) {
    const uint64_t mid = (lo + hi) >> 1;
    if ((uint64_t)(uint32_t)runs[3 * mid] <= row) lo = mid; else hi = mid;
  }
  cover[t] = (uint32_t)lo;
}

// R_expand: one workgroup per output tile [t0, t0 + TILE): the runs from the covering one on
// (at most TILE + 1 reach into the tile) into LDS, a flag at every later run's first row, an
// inclusive scan of the flags = each row's run (relative to the covering run), then every row
// written as its run's {i, j} + its distance from the run's first row -- coalesced 8-B stores.
__global__ void __launch_bounds__(BLOCK)
k_runs_expand(const int32_t* __restrict__ runs, uint64_t n_runs, uint64_t n,
              const uint32_t* __restrict__ cover, int2* __restrict__ out) {
  __shared__ uint32_t rs[TILE + 1], ri[TILE + 1], rj[TILE + 1];
  __shared__ uint16_t fl[TILE];
  __shared__ uint64_t sh[8];
  const uint64_t t0 = (uint64_t)blockIdx.x * TILE;
  const uint64_t t1 = min(n, t0 + (uint64_t)TILE);
  const uint64_t f = cover[blockIdx.x];
  for (uint32_t x = threadIdx.x; x < TILE; x += BLOCK) fl[x] = 0;
  __syncthreads();
  for (uint32_t q = threadIdx.x; q <= TILE; q += BLOCK) {
    const uint64_t g = f + q;
    const uint64_t s0 = g < n_runs ? (uint64_t)(uint32_t)runs[3 * g] : n;
    if (s0 < t1) {
      rs[q] = (uint32_t)s0;
      ri[q] = (uint32_t)runs[3 * g + 1];
      rj[q] = (uint32_t)runs[3 * g + 2];
      if (q > 0 && s0 > t0) fl[s0 - t0] = 1;  // q = 0 starts at or before t0 (runs ascend)
    }
  }
  __syncthreads();
  // inclusive scan of the flags: thread t owns rows [8 t, 8 t + 8) of the tile
  uint32_t c[WPT], sum = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    sum += fl[threadIdx.x * WPT + j];
    c[j] = sum;
  }
  uint64_t tot;
  const uint32_t ex = (uint32_t)block_excl_scan((uint64_t)sum, sh, tot);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < WPT; ++j) fl[threadIdx.x * WPT + j] = (uint16_t)(ex + c[j]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const uint64_t r = t0 + (uint64_t)j * BLOCK + threadIdx.x;
    if (r < t1) {
      const uint32_t q = fl[r - t0];
      const uint32_t d = (uint32_t)(r - rs[q]);
      out[r] = make_int2((int32_t)(ri[q] + d), (int32_t)(rj[q] + d));
    }
  }
}

// ---------------------------------------------------------------- packed sequence (C1 transfers)
// A sequence crosses xGMI (C1 scatter / broadcast, the owner-computes build's broadcast) as the
// two things every kernel reads from a char -- its 2-bit code (c >> 1) & 3 and its N flag
// ((c | 0x20) == 'n') -- 16 chars per u32 code word and u16 flag word, MSB first: 6 B per 16
// chars instead of 16.  Unpacked, a char is "ACTG"[code] or 'N', which every kernel reads as the
// original (lower case, IUPAC letters and the like map to the code they already had).
__global__ void __launch_bounds__(BLOCK)
k_seq_pack(const uint8_t* __restrict__ seq, int64_t L, uint32_t* __restrict__ code,
           uint16_t* __restrict__ nbit, uint64_t words) {
  const uint64_t w = (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  if (w >= words) return;
  const int64_t c0 = (int64_t)w * 16;
  uint8_t ch[16];
  if (c0 + 16 <= L && (reinterpret_cast<uintptr_t>(seq + c0) & 15) == 0) {
    const uint4 v = *reinterpret_cast<const uint4*>(seq + c0);
    const uint32_t x[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int q = 0; q < 16; ++q) ch[q] = (uint8_t)(x[q >> 2] >> (8 * (q & 3)));
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q) ch[q] = c0 + q < L ? seq[c0 + q] : (uint8_t)'A';
  }
  uint32_t cw = 0, nw = 0;
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    cw |= (uint32_t)((ch[q] >> 1) & 3u) << (30 - 2 * q);
    nw |= (uint32_t)((ch[q] | 0x20) == 'n') << (15 - q);
  }
  code[w] = cw;
  nbit[w] = (uint16_t)nw;
}

// chars [a, b) of seq from the words [w0, ...) held at code / nbit (word w at index w - w0)
__global__ void __launch_bounds__(BLOCK)
k_seq_unpack(const uint32_t* __restrict__ code, const uint16_t* __restrict__ nbit, uint64_t w0,
             int64_t a, int64_t b, uint8_t* __restrict__ seq) {
  const uint64_t w = (uint64_t)(a >> 4) + (uint64_t)blockIdx.x * BLOCK + threadIdx.x;
  const int64_t c0 = (int64_t)w * 16;
  if (c0 >= b) return;
  const uint32_t cw = code[w - w0], nw = nbit[w - w0];
  uint8_t ch[16];
#pragma unroll
  for (int q = 0; q < 16; ++q) {
    const uint32_t c = (cw >> (30 - 2 * q)) & 3u;
    ch[q] = ((nw >> (15 - q)) & 1u) ? (uint8_t)'N'
                                     : (uint8_t)(c == 0 ? 'A' : c == 1 ? 'C' : c == 2 ? 'T' : 'G');
  }
  if (c0 >= a && c0 + 16 <= b && (reinterpret_cast<uintptr_t>(seq + c0) & 15) == 0) {
    uint32_t x[4] = {0u, 0u, 0u, 0u};
#pragma unroll
    for (int q = 0; q < 16; ++q) x[q >> 2] |= (uint32_t)ch[q] << (8 * (q & 3));
    *reinterpret_cast<uint4*>(seq + c0) = make_uint4(x[0], x[1], x[2], x[3]);
  } else {
#pragma unroll
    for (int q = 0; q < 16; ++q)
      if (c0 + q >= a && c0 + q < b) seq[c0 + q] = ch[q];
  }
}

void launch_seq_pack(const uint8_t* seq, int64_t L, uint32_t* code, uint16_t* nbit,
                     hipStream_t s) {
  const uint64_t words = ((uint64_t)L + 15) / 16;
  hipLaunchKernelGGL(k_seq_pack, dim3((unsigned)((words + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0, s,
                     seq, L, code, nbit, words);
}
void launch_seq_unpack(const uint32_t* code, const uint16_t* nbit, uint64_t w0, int64_t a,
                       int64_t b, uint8_t* seq, hipStream_t s) {
  const uint64_t words = (uint64_t)((b + 15) >> 4) - (uint64_t)(a >> 4);
  hipLaunchKernelGGL(k_seq_unpack, dim3((unsigned)((words + BLOCK - 1) / BLOCK)), dim3(BLOCK), 0,
                     s, code, nbit, w0, a, b, seq);
}

// ---------------------------------------------------------------- a query's rows as runs
// A range query whose rows leave the device only as diagonal runs (the senders of the sharded
// query's gather, kmhg_query_run_device_range_runs) makes the runs from its per-window records
// (qrec / qmulti) and never writes the rows.  The row of a single-hit window w continues the
// previous row's run when window w - 1 is a single hit one index position earlier; every row of
// a multi-hit window is a run of its own (its rows share i).  That is a valid run encoding, not
// always the maximal one (a single hit right after a multi-hit window starts a run even where
// it extends one): kmhg_runs_expand gives the query's rows either way.  Thread t takes the 8
// consecutive windows [8 t, 8 t + 8) of a TILE-window tile (window order = thread order).
struct QRun { uint32_t n, st; };   // a window's rows, and how many of them start a run
__device__ __forceinline__ QRun qrun_window(uint32_t rec, uint32_t prev, const uint2* qmulti,
                                            uint64_t w) {
  if (rec == 0) return {0u, 0u};
  if (rec == QREC_MULTI) {
    const uint32_t m = qmulti[w].x;
    return {m, m};
  }
  return {1u, (prev != 0 && prev != QREC_MULTI && prev + 1u == rec) ? 0u : 1u};
}

// a thread's 8 window records: two 16-B loads (wa is a multiple of 8 windows and qrec starts
// 256-B aligned), element loads at the range's end.  (Element loads throughout, lanes 32 B
// apart, ran both kernels at ~2 TB/s.)
static_assert(WPT == 8, "load_rec8 reads 8 records per thread");
__device__ __forceinline__ void load_rec8(const uint32_t* __restrict__ qrec, uint64_t wa,
                                          uint64_t Nw, uint32_t (&rec)[WPT]) {
  if (wa + WPT <= Nw) {
    const uint4 a = *reinterpret_cast<const uint4*>(qrec + wa);
    const uint4 b = *reinterpret_cast<const uint4*>(qrec + wa + 4);
    rec[0] = a.x; rec[1] = a.y; rec[2] = a.z; rec[3] = a.w;
    rec[4] = b.x; rec[5] = b.y; rec[6] = b.z; rec[7] = b.w;
  } else {
#pragma unroll
    for (int j = 0; j < WPT; ++j) rec[j] = wa + j < Nw ? qrec[wa + j] : 0u;
  }
}

__global__ void __launch_bounds__(BLOCK)
k_qruns_count(const uint32_t* __restrict__ qrec, const uint2* __restrict__ qmulti, uint64_t Nw,
              uint64_t* __restrict__ tile_cnt) {
  __shared__ uint64_t sh[8];
  const uint64_t wa = (uint64_t)blockIdx.x * TILE + WPT * threadIdx.x;
  uint32_t prev = wa > 0 && wa - 1 < Nw ? qrec[wa - 1] : 0u;
  uint32_t rec[WPT];
  load_rec8(qrec, wa, Nw, rec);
  uint64_t c = 0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    c += qrun_window(rec[j], prev, qmulti, wa + j).st;
    prev = rec[j];
  }
  uint64_t tot;
  block_excl_scan(c, sh, tot);
  if (threadIdx.x == 0) tile_cnt[blockIdx.x] = tot;
}

// (the per-window counts are recomputed from rec[] in the write loop rather than kept in arrays
// across the scans: the arrays version came out of the compiler with wrong row counts on gfx950)
__global__ void __launch_bounds__(BLOCK)
k_qruns_emit(const uint32_t* __restrict__ qrec, const uint2* __restrict__ qmulti,
             const int32_t* __restrict__ positions, uint64_t Nw, int64_t w0, int kq,
             const uint64_t* __restrict__ tile_row0, const uint64_t* __restrict__ tile_run0,
             uint64_t n_runs, int32_t* __restrict__ runs) {
  __shared__ uint64_t sh[8];
  // the records' loads go out first; the tile offsets (scalar loads) resolve meanwhile
  const uint64_t wa = (uint64_t)blockIdx.x * TILE + WPT * threadIdx.x;
  const uint32_t prev0 = wa > 0 && wa - 1 < Nw ? qrec[wa - 1] : 0u;
  uint32_t rec[WPT];
  load_rec8(qrec, wa, Nw, rec);
  const uint64_t q0 = tile_run0[blockIdx.x];
  const uint64_t row0 = tile_row0[blockIdx.x];
  if (q0 == (blockIdx.x + 1 < gridDim.x ? tile_run0[blockIdx.x + 1] : n_runs)) return;  // no run starts here
  uint64_t nr = 0, ns = 0;
  uint32_t prev = prev0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const QRun x = qrun_window(rec[j], prev, qmulti, wa + j);
    nr += x.n;
    ns += x.st;
    prev = rec[j];
  }
  // one scan for both prefixes: rows in the high half, run starts (<= rows) in the low half --
  // the host emits runs only for H <= 2^31 - 1 rows, so neither half carries over
  uint64_t tot;
  const uint64_t ex = block_excl_scan((nr << 32) | ns, sh, tot);
  uint64_t r = row0 + (ex >> 32);
  uint64_t q = q0 + (ex & 0xffffffffull);
  prev = prev0;
#pragma unroll
  for (int j = 0; j < WPT; ++j) {
    const uint64_t w = wa + j;
    const QRun x = qrun_window(rec[j], prev, qmulti, w);
    prev = rec[j];
    if (!x.n) continue;
    const int32_t i = (int32_t)(w0 + (int64_t)w + kq);
    if (rec[j] != QREC_MULTI) {
      if (x.st) {
        int32_t* o = runs + 3 * q++;
        o[0] = (int32_t)r; o[1] = i; o[2] = (int32_t)rec[j];
      }
      ++r;
    } else {
      const uint32_t first = qmulti[w].y;
      for (uint32_t t = 0; t < x.n; ++t, ++r) {
        int32_t* o = runs + 3 * q++;
        o[0] = (int32_t)r; o[1] = i; o[2] = positions[first + t];
      }
    }
  }
}

void launch_qruns_count(const uint32_t* qrec, const uint2* qmulti, uint64_t Nw,
                        uint64_t* tile_cnt, hipStream_t s) {
  hipLaunchKernelGGL(k_qruns_count, dim3((unsigned)((Nw + TILE - 1) / TILE)), dim3(BLOCK), 0, s,
                     qrec, qmulti, Nw, tile_cnt);
}
void launch_qruns_emit(const uint32_t* qrec, const uint2* qmulti, const int32_t* positions,
                       uint64_t Nw, int64_t w0, int kq, const uint64_t* tile_row0,
                       const uint64_t* tile_run0, uint64_t n_runs, int32_t* runs, hipStream_t s) {
  hipLaunchKernelGGL(k_qruns_emit, dim3((unsigned)((Nw + TILE - 1) / TILE)), dim3(BLOCK), 0, s,
                     qrec, qmulti, positions, Nw, w0, kq, tile_row0, tile_run0, n_runs, runs);
}

void launch_runs_count(const int2* rows, uint64_t n, uint64_t* tile_cnt, hipStream_t s) {
  hipLaunchKernelGGL(k_runs_count, dim3((unsigned)((n + TILE - 1) / TILE)), dim3(BLOCK), 0, s,
                     rows, n, tile_cnt);
}
void launch_runs_emit(const int2* rows, uint64_t n, const uint64_t* tile_off, int32_t* runs,
                      hipStream_t s) {
  hipLaunchKernelGGL(k_runs_emit, dim3((unsigned)((n + TILE - 1) / TILE)), dim3(BLOCK), 0, s,
                     rows, n, tile_off, runs);
}
void launch_runs_expand(const int32_t* runs, uint64_t n_runs, uint64_t n, uint32_t* cover,
                        int2* out, hipStream_t s) {
  const uint32_t nt = (uint32_t)((n + TILE - 1) / TILE);
  hipLaunchKernelGGL(k_runs_cover, dim3((nt + BLOCK - 1) / BLOCK), dim3(BLOCK), 0, s, runs,
                     n_runs, nt, cover);
  hipLaunchKernelGGL(k_runs_expand, dim3(nt), dim3(BLOCK), 0, s, runs, n_runs, n, cover, out);
}

void launch_scan_tiles_u64(uint64_t* a, uint32_t n, uint64_t* total, hipStream_t s) {
  if (n <= SCAN1_MAX)
    hipLaunchKernelGGL(k_scan_tiles_u64, dim3(1), dim3(1024), 0, s, a, n, total);
  else
    hipLaunchKernelGGL(k_scan_tiles_u64_any, dim3(1), dim3(1024), 0, s, a, n, total);
}
void launch_scan_u64(uint64_t* a, uint64_t n, uint64_t* total, uint64_t* scratch, hipStream_t s) {
  if (n <= SCAN1_MAX) {
    launch_scan_tiles_u64(a, (uint32_t)n, total, s);
    return;
  }
  const uint32_t nb = grid_for(n, TILE);
  hipLaunchKernelGGL(k_block_sum_u64, dim3(nb), dim3(BLOCK), 0, s, a, n, scratch);
  launch_scan_tiles_u64(scratch, nb, total, s);
  hipLaunchKernelGGL(k_block_scan_u64, dim3(nb), dim3(BLOCK), 0, s, a, n,
                     (const uint64_t*)scratch);
}
void launch_query_emit(const uint32_t* qrec, const uint2* qmulti, int64_t Nw, int64_t w0, int kq,
                       const int32_t* positions, const uint64_t* tile_row0, int2* out,
                       uint64_t cap, uint32_t* elist, uint32_t* ecount, bool append,
                       hipStream_t s) {
  const uint32_t nt = grid_for(Nw, TILE);
  hipLaunchKernelGGL(k_query_emit1, dim3(nt), dim3(BLOCK), 0, s, qrec, Nw, w0, kq, tile_row0, out,
                     cap, elist, ecount, append ? 1 : 0);
  static const unsigned cap_g = [] {
    int per = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)k_query_emit, BLOCK, 0) !=
            hipSuccess || per < 1)
      per = 1;
    int dev = 0, cus = 0;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    return (unsigned)(per * (cus > 0 ? cus : 1));
  }();
  hipLaunchKernelGGL(k_query_emit, dim3(std::min<unsigned>(nt, cap_g)), dim3(BLOCK), 0, s, qrec,
                     qmulti, Nw, w0, kq, positions, tile_row0, out, cap, elist, ecount);
}
void launch_read_first(const Slot* T, uint64_t nslots, const int32_t* positions, uint2* F,
                       hipStream_t s) {
  unsigned g = grid_for(nslots, BLOCK);
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_read_first, dim3(g), dim3(BLOCK), 0, s, T, nslots, positions, F);
}
void launch_read_order(const uint2* F, int64_t L, const Slot* T, uint64_t* st_a, uint64_t* st_b,
                       uint64_t* st_c, uint32_t* ticket, uint32_t* perm, uint32_t* canon_off,
                       uint32_t* pkeys, uint64_t* pair_off, uint2* rinfo, ReadMeta* rmeta,
                       hipStream_t s) {
  uint32_t nt = grid_for(L, TILE);
  hipLaunchKernelGGL(k_read_order, dim3(nt), dim3(BLOCK), 0, s, F, L, T, st_a, st_b, st_c,
                     ticket, perm, canon_off, pkeys, pair_off, rinfo, nt, rmeta);
}
void launch_read_keys(const uint32_t* perm, const uint2* rinfo, uint32_t U, const Slot* T, int k,
                      int32_t* out_counts, char* out_kmers, hipStream_t s) {
  unsigned g = grid_for(U, BLOCK);
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_read_keys, dim3(g), dim3(BLOCK), 0, s, perm, rinfo, U, T, k, out_counts,
                     out_kmers);
}
void launch_gather_keys(const uint32_t* perm, uint32_t U, const Slot* T, uint64_t* out_keys,
                        hipStream_t s) {
  unsigned g = grid_for(U, BLOCK);
  if (g > 16384) g = 16384;
  hipLaunchKernelGGL(k_gather_keys, dim3(g), dim3(BLOCK), 0, s, perm, U, T, out_keys);
}
void launch_read_pos(const uint2* rinfo, const uint32_t* canon_off, uint32_t U, uint64_t nrows,
                     const int32_t* positions, uint32_t* tile_key, int2* out, hipStream_t s) {
  if (!nrows) return;
  const uint32_t nt = grid_for(nrows, TILE);
  hipLaunchKernelGGL(k_row_tiles<uint32_t>, dim3(std::min(grid_for(U, BLOCK), 16384u)),
                     dim3(BLOCK), 0, s, canon_off, U, nrows, (uint32_t)TILE, tile_key, nt);
  hipLaunchKernelGGL(k_read_pos, dim3(nt), dim3(BLOCK), 0, s, rinfo, canon_off, tile_key, nrows,
                     positions, out);
}
uint32_t read_pos_tiles(uint64_t nrows) { return grid_for(nrows, TILE); }
void launch_read_pairs(const uint32_t* pkeys, const uint64_t* pair_off, uint32_t M,
                       uint64_t nrows, const uint2* rinfo, const int32_t* positions,
                       uint32_t* tile_key, int32_t* out, hipStream_t s) {
  if (!nrows) return;
  const uint32_t nt = grid_for(nrows, PR_TILE);
  hipLaunchKernelGGL(k_row_tiles<uint64_t>, dim3(std::min(grid_for(M, BLOCK), 16384u)),
                     dim3(BLOCK), 0, s, pair_off, M, nrows, (uint32_t)PR_TILE, tile_key, nt);
  hipLaunchKernelGGL(k_read_pairs, dim3(nt), dim3(BLOCK), 0, s, pkeys, pair_off, tile_key, nrows,
                     rinfo, positions, out);
}
uint32_t read_pairs_tiles(uint64_t nrows) { return grid_for(nrows, PR_TILE); }

}  // namespace kmhg
